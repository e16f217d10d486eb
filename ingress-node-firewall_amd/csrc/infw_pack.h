// infw_pack.h — frame header -> 32-byte SoA tuple (include/infw.h: infw_batch_soa).
//
// The tuple keeps exactly the bytes bpf/ingress_node_firewall_kernel.c reads
// from a frame, at the same fixed offsets:
//   ethertype  frame[12..13]                      (kernel.c:427)
//   L3 proto   frame[23] (iphdr.protocol) / frame[20] (ipv6hdr.nexthdr)  (:108,:115)
//   saddr      frame[26..29] / frame[22..37]      (:204, :291)
//   L4 word    frame[34..37] / frame[54..57]      (:125,:135,:145,:155,:166 — dest
//              port at +2, ICMP type/code at +0/+1; L4 offset is fixed: IHL and
//              IPv6 extension headers are not consulted, :104, :111)
//   linear length, clamped to 255, for the truncation checks (:105-173, :423)
//   bpf_xdp_get_buff_len for the byte counters (:446, :450)
// Usable from host C++ and from HIP device code.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define INFW_HD __host__ __device__ __forceinline__
#else
#define INFW_HD static inline
#endif

#define INFW_HDR_SNAP 80  // bytes of a frame any consumer of the path ever reads (< 74 used)

struct infw_tuple {
    uint32_t saddr[4];  // frame bytes in memory order (little-endian words)
    uint32_t ifindex;
    uint32_t pkt_len;
    uint32_t meta;
    uint32_t l4word;
};

// hdr: the first min(caplen, INFW_HDR_SNAP) bytes of the frame.
// caplen: linear length (xdp data_end - data); pkt_len: full frame length.
INFW_HD void infw_pack_header(const uint8_t *hdr, uint32_t caplen, uint32_t pkt_len,
                              uint32_t ifindex, struct infw_tuple *t) {
    uint32_t ethertype = 0, proto = 0, l4off = 0, soff = 0, slen = 0;
    if (caplen >= 14) {
        ethertype = (uint32_t)hdr[12] << 8 | hdr[13];
        if (ethertype == 0x0800) {
            if (caplen > 23) proto = hdr[23];
            l4off = 34;
            soff = 26;
            slen = 4;
        } else if (ethertype == 0x86DD) {
            if (caplen > 20) proto = hdr[20];
            l4off = 54;
            soff = 22;
            slen = 16;
        }
    }
    uint8_t sb[16];
    for (int i = 0; i < 16; i++) sb[i] = 0;
    for (uint32_t i = 0; i < slen; i++)
        if (soff + i < caplen && soff + i < INFW_HDR_SNAP) sb[i] = hdr[soff + i];
    for (int w = 0; w < 4; w++)
        t->saddr[w] = (uint32_t)sb[4 * w] | (uint32_t)sb[4 * w + 1] << 8 |
                      (uint32_t)sb[4 * w + 2] << 16 | (uint32_t)sb[4 * w + 3] << 24;
    uint32_t l4 = 0;
    if (l4off)
        for (uint32_t i = 0; i < 4; i++)
            if (l4off + i < caplen && l4off + i < INFW_HDR_SNAP) l4 |= (uint32_t)hdr[l4off + i] << (8 * i);
    t->ifindex = ifindex;
    t->pkt_len = pkt_len;
    t->meta = ethertype | proto << 16 | (caplen > 255u ? 255u : caplen) << 24;
    t->l4word = l4;
}
