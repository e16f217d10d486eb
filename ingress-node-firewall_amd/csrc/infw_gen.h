// infw_gen.h — deterministic synthetic packet workloads (bench / test infrastructure).
//
// Packet i of a workload is a pure function of (params, i): a counter-based
// RNG keyed on the global packet index, so a shard [a, b) is identical at any
// GPU count and the host (frames for the oracle) and the
// device (SoA tuples for the classifier) produce the same packets.
// Integer arithmetic only, identical on host and gfx950.
#pragma once
#include <stdint.h>

#include "infw_pack.h"

struct infw_gen_prefix {   // a source prefix packets may be drawn from
    uint8_t addr[16];      // v4: bytes 0..3
    uint32_t ifindex;
    uint8_t plen;          // address bits (0..32 v4, 0..128 v6)
    uint8_t family;        // 4 or 6
    uint8_t pad[2];
};

struct infw_gen_params {
    uint64_t seed;
    const struct infw_gen_prefix *prefixes;  // sampled for "hit" packets (by popularity rank)
    const uint64_t *zipf_cdf;                // n_prefixes thresholds, or NULL = uniform
    uint32_t n_prefixes;
    uint32_t hit_permille;     // sourced inside a sampled prefix
    uint32_t v6_permille;      // family of non-hit packets
    uint32_t cross_permille;   // hit packets emitted in the other family (unified key space)
    uint32_t p_tcp, p_udp, p_icmp, p_sctp;  // per-mille; the rest: proto 47 (GRE, unsupported)
    uint32_t p_special;        // per-mille of TCP/UDP/SCTP dports from special_ports
    uint32_t n_special;
    uint16_t special_ports[16];
    uint32_t n_icmp;           // ICMP/ICMPv6 (type<<8|code) choices (0 = uniform 16-bit)
    uint16_t icmp_tc[16];
    uint32_t len_min, len_max; // frame length U[len_min, len_max], raised to the headers
    uint32_t p_nonip;          // per-mille non-IP ethertype (ARP, VLAN, LLDP)
    uint32_t p_trunc;          // per-mille truncated headers (caplen == len < needed)
    uint32_t n_ifindex;        // ifindexes of non-hit packets
    uint32_t ifindexes[8];
};

INFW_HD uint64_t infw_mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
INFW_HD uint64_t infw_rng(uint64_t seed, uint64_t idx, uint32_t stream) {
    return infw_mix64(seed ^ infw_mix64(idx * 0x100000001B3ull + stream));
}
INFW_HD uint32_t infw_below(uint64_t r, uint32_t n) {  // uniform in [0, n) from the top 32 bits
    return (uint32_t)(((r >> 32) * (uint64_t)n) >> 32);
}
INFW_HD uint64_t infw_rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

// Rank -> prefix index by the integer CDF (binary search on thresholds).
INFW_HD uint32_t infw_zipf_pick(const uint64_t *cdf, uint32_t n, uint64_t r) {
    uint32_t lo = 0, hi = n - 1;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (r < cdf[mid]) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

// Build the header snapshot (first INFW_HDR_SNAP bytes, zero beyond caplen) of packet idx.
INFW_HD void infw_gen_header(const struct infw_gen_params *p, uint64_t idx, uint8_t *hdr,
                             uint32_t *caplen, uint32_t *pkt_len, uint32_t *ifindex) {
    for (int i = 0; i < INFW_HDR_SNAP; i++) hdr[i] = 0;
    uint64_t r0 = infw_rng(p->seed, idx, 0);
    uint64_t r1 = infw_rng(p->seed, idx, 1);
    uint64_t r2 = infw_rng(p->seed, idx, 2);
    uint64_t r3 = infw_rng(p->seed, idx, 3);
    uint64_t r4 = infw_rng(p->seed, idx, 4);
    uint64_t r5 = infw_rng(p->seed, idx, 5);

    uint8_t addr[16];
    int fam;
    uint32_t ifx;
    if (p->n_prefixes && infw_below(r0, 1000) < p->hit_permille) {
        uint32_t k = p->zipf_cdf ? infw_zipf_pick(p->zipf_cdf, p->n_prefixes, r1)
                                 : infw_below(r1, p->n_prefixes);
        const struct infw_gen_prefix *px = &p->prefixes[k];
        ifx = px->ifindex;
        fam = px->family;
        // random host bits below the prefix
        for (int w = 0; w < 2; w++) {
            uint64_t rb = infw_rng(p->seed, idx, 10 + w);
            for (int b = 0; b < 8; b++) addr[8 * w + b] = (uint8_t)(rb >> (8 * b));
        }
        uint32_t alen = fam == 4 ? 32u : 128u;
        uint32_t pl = px->plen;
        for (uint32_t i = 0; i < 16; i++) {
            uint32_t bit0 = 8 * i;
            if (pl >= bit0 + 8) addr[i] = px->addr[i];
            else if (pl > bit0) {
                uint8_t m = (uint8_t)(0xFFu << (8 - (pl - bit0)));
                addr[i] = (uint8_t)((px->addr[i] & m) | (addr[i] & ~m));
            }
        }
        (void)alen;
        // cross-family: same leading bits, the other header format
        if (infw_below(infw_rotl(r0, 16), 1000) < p->cross_permille) {
            if (fam == 4) fam = 6;
            else if (pl <= 32) fam = 4;
        }
    } else {
        fam = infw_below(r1, 1000) < p->v6_permille ? 6 : 4;
        for (int w = 0; w < 2; w++) {
            uint64_t rb = infw_rng(p->seed, idx, 12 + w);
            for (int b = 0; b < 8; b++) addr[8 * w + b] = (uint8_t)(rb >> (8 * b));
        }
        ifx = p->n_ifindex ? p->ifindexes[infw_below(infw_rotl(r1, 8), p->n_ifindex)] : 1u;
    }

    // protocol and L4 fields
    uint32_t pr = infw_below(r2, 1000);
    uint8_t proto;
    int l4len;
    if (pr < p->p_tcp) { proto = 6; l4len = 20; }
    else if (pr < p->p_tcp + p->p_udp) { proto = 17; l4len = 8; }
    else if (pr < p->p_tcp + p->p_udp + p->p_icmp) { proto = fam == 4 ? 1 : 58; l4len = 8; }
    else if (pr < p->p_tcp + p->p_udp + p->p_icmp + p->p_sctp) { proto = 132; l4len = 12; }
    else { proto = 47; l4len = 4; }
    // a small share of ICMP packets carry the other family's ICMP number
    if ((proto == 1 || proto == 58) && infw_below(infw_rotl(r2, 20), 1000) < 20) proto = proto == 1 ? 58 : 1;
    uint16_t dport;
    if (p->n_special && infw_below(r3, 1000) < p->p_special)
        dport = p->special_ports[infw_below(infw_rotl(r3, 12), p->n_special)];
    else
        dport = (uint16_t)(r3 >> 40);
    uint16_t tc = p->n_icmp ? p->icmp_tc[infw_below(r4, p->n_icmp)] : (uint16_t)(r4 >> 48);

    // lengths
    uint32_t l3 = fam == 4 ? 20u : 40u;
    uint32_t need = 14u + l3 + (uint32_t)l4len;
    uint32_t span = p->len_max > p->len_min ? p->len_max - p->len_min + 1 : 1;
    uint32_t len = p->len_min + infw_below(r5, span);
    if (len < need) len = need;
    uint32_t cap = len;
    uint16_t ethertype = fam == 4 ? 0x0800 : 0x86DD;
    uint32_t odd = infw_below(infw_rotl(r5, 16), 1000);
    if (odd < p->p_nonip) {
        const uint16_t et[4] = {0x0806, 0x8100, 0x88CC, 0x88A8};
        ethertype = et[infw_below(infw_rotl(r4, 8), 4)];
    } else if (odd < p->p_nonip + p->p_trunc) {
        // truncated: anywhere from a bare Ethernet header to one byte short of L4
        cap = 14u + infw_below(infw_rotl(r4, 16), l3 + (uint32_t)l4len);
        len = cap;
    }

    // Ethernet
    const uint8_t mac[12] = {0x02, 0, 0, 0, 0, 0x01, 0x02, 0, 0, 0, 0, 0x02};
    for (int i = 0; i < 12; i++) hdr[i] = mac[i];
    hdr[12] = (uint8_t)(ethertype >> 8);
    hdr[13] = (uint8_t)ethertype;
    uint32_t l4off;
    if (fam == 4) {
        hdr[14] = infw_below(infw_rotl(r4, 24), 16) == 0 ? 0x46 : 0x45;  // IHL is ignored by the program
        uint32_t tot = len - 14;
        hdr[16] = (uint8_t)(tot >> 8); hdr[17] = (uint8_t)tot;
        hdr[22] = 64;
        hdr[23] = proto;
        for (int i = 0; i < 4; i++) hdr[26 + i] = addr[i];
        hdr[30] = 192; hdr[31] = 0; hdr[32] = 2; hdr[33] = 1;
        l4off = 34;
    } else {
        hdr[14] = 0x60;
        uint32_t pl = len > 54 ? len - 54 : 0;
        hdr[18] = (uint8_t)(pl >> 8); hdr[19] = (uint8_t)pl;
        hdr[20] = proto;
        hdr[21] = 64;
        for (int i = 0; i < 16; i++) hdr[22 + i] = addr[i];
        hdr[38] = 0x20; hdr[39] = 0x01; hdr[40] = 0x0d; hdr[41] = 0xb8; hdr[53] = 1;
        l4off = 54;
    }
    uint16_t sport = (uint16_t)(1024 + infw_below(infw_rotl(r5, 32), 60000));
    if (proto == 6 || proto == 17 || proto == 132) {
        hdr[l4off] = (uint8_t)(sport >> 8); hdr[l4off + 1] = (uint8_t)sport;
        hdr[l4off + 2] = (uint8_t)(dport >> 8); hdr[l4off + 3] = (uint8_t)dport;
        if (proto == 6) { hdr[l4off + 12] = 0x50; hdr[l4off + 13] = 0x02; }
        if (proto == 17) { uint32_t ul = len - l4off; hdr[l4off + 4] = (uint8_t)(ul >> 8); hdr[l4off + 5] = (uint8_t)ul; }
    } else if (proto == 1 || proto == 58) {
        hdr[l4off] = (uint8_t)(tc >> 8);
        hdr[l4off + 1] = (uint8_t)tc;
    } else {
        hdr[l4off] = 0x00; hdr[l4off + 2] = 0x08; hdr[l4off + 3] = 0x00;
    }
    for (uint32_t i = cap; i < INFW_HDR_SNAP; i++) hdr[i] = 0;
    *caplen = cap;
    *pkt_len = len;
    *ifindex = ifx;
}

INFW_HD void infw_gen_tuple(const struct infw_gen_params *p, uint64_t idx, struct infw_tuple *t) {
    uint8_t hdr[INFW_HDR_SNAP];
    uint32_t cap, len, ifx;
    infw_gen_header(p, idx, hdr, &cap, &len, &ifx);
    infw_pack_header(hdr, cap, len, ifx, t);
}
