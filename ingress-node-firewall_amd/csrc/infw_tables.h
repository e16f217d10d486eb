// infw_tables.h — GPU table layout of one committed table epoch, and the
// per-packet walk over it (parse -> LPM -> class-filtered first-match scan).
//
// What the reference does per frame (bpf/ingress_node_firewall_kernel.c):
//   LPM lookup of {prefixLen, ifindex, ip_data} in an LPM trie (:204-219,
//   :291-302), then a first-match scan of the 100-slot rule array (:222-258,
//   :306-340).  The key space is unified: IPv4 lookups use prefixLen 64 with
//   the address in ip_data[0..3], IPv6 lookups prefixLen 160, so an IPv4
//   packet considers every entry of <= 32 address bits (whichever family wrote
//   it) and an IPv6 packet every entry of <= 128 bits.
//
// How the epoch lays that out in HBM (built on the host, tables.cpp):
//   ifindex -> slot      open-addressed u32 table
//   short (<= /32)       DIR-24-8 per slot: tbl24[slot][2^24] u32 + tbl8 groups
//                        of 256 u32; value = list+1 (0 = no entry), bit 31 of a
//                        tbl24 word = "tbl8 group index"
//   long  (/33../128)    one open-addressed table of 32-B records keyed by
//                        (slot, length, masked address), searched by binary
//                        search over the distinct lengths with markers
//                        (Waldvogel et al.); bmp = best real long prefix
//   rule lists           interned per distinct 1200-B value; per list and
//                        packet class c, the applicable rules in slot order as
//                        u64 {lo16, hi16, result32}; desc[list*8+c] = off|cnt<<32
// An IPv6 packet takes the long answer if any, else the short table on its
// top 32 bits — exactly the unified longest-prefix order.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define INFW_TD __host__ __device__ __forceinline__
#else
#define INFW_TD static inline
#endif

#define INFW_NCLS 7
#define INFW_DESC_STRIDE 8
#define INFW_TBL8_FLAG 0x80000000u
#define INFW_IF_EMPTY 0xFFFFFFFFu
#define INFW_MAX_LEVELS 96

// Packet classes (rule applicability): which protocol the scan honours.
enum {
    INFW_CLS_TCP = 0,       // proto 6, either family
    INFW_CLS_UDP = 1,       // proto 17
    INFW_CLS_SCTP = 2,      // proto 132
    INFW_CLS_ICMP4 = 3,     // proto 1 on the IPv4 path   (kernel.c:247)
    INFW_CLS_ICMP6 = 4,     // proto 58 on the IPv6 path  (kernel.c:329)
    INFW_CLS_58_ON_V4 = 5,  // proto 58 on IPv4: only protocol-0 rules can match
    INFW_CLS_1_ON_V6 = 6,   // proto 1 on IPv6: only protocol-0 rules can match
};

struct infw_long_entry {    // 32 B
    uint64_t hi, lo;        // masked address, big-endian halves
    uint32_t tag;           // slot << 8 | length (length >= 33, so never 0)
    uint32_t bmp;           // list+1 of the best real long prefix at or above this level, 0 = none
    uint32_t pad[2];
};

struct infw_dev_tables {
    const uint32_t *if_keys;
    const uint32_t *if_slot;   // INFW_IF_EMPTY = free
    uint32_t if_mask;
    uint32_t n_slots;
    const uint32_t *tbl24;
    const uint32_t *tbl8;
    const struct infw_long_entry *ltab;
    uint64_t lmask;
    const uint64_t *desc;
    const uint64_t *rules;
    uint32_t n_levels;
    uint8_t levels[INFW_MAX_LEVELS];
};

INFW_TD uint32_t infw_bswap32(uint32_t x) {
    return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}
INFW_TD uint64_t infw_be64(uint32_t w0, uint32_t w1) {  // bytes w0[0..3] w1[0..3] as a BE u64
    return (uint64_t)infw_bswap32(w0) << 32 | infw_bswap32(w1);
}

INFW_TD uint32_t infw_if_hash(uint32_t ifindex) { return ifindex * 0x9E3779B1u; }

INFW_TD uint64_t infw_long_hash(uint32_t tag, uint64_t hi, uint64_t lo) {
    uint64_t h = hi * 0x9E3779B97F4A7C15ull;
    h ^= (lo + 0x632BE59BD9B4E019ull) * 0xC2B2AE3D27D4EB4Full;
    h ^= (uint64_t)tag * 0x165667B19E3779F9ull;
    h ^= h >> 29;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 32;
    return h;
}

INFW_TD void infw_mask128(uint32_t len, uint64_t *hi, uint64_t *lo) {
    if (len >= 128) return;
    if (len > 64) {
        *lo &= ~0ull << (128 - len);
    } else {
        *lo = 0;
        *hi = len == 0 ? 0 : (*hi & (~0ull << (64 - len)));
    }
}

// Parse result of one tuple (ingress_node_firewall_main + ip_extract_l4info).
enum { INFW_PK_DROP_SHORT = 0, INFW_PK_PASS_NONIP = 1, INFW_PK_UNDEF = 2, INFW_PK_V4 = 3, INFW_PK_V6 = 4 };

INFW_TD int infw_parse(uint32_t meta, uint32_t l4word, int *cls, uint32_t *val) {
    uint32_t et = meta & 0xFFFFu, proto = (meta >> 16) & 0xFFu, cap = meta >> 24;
    if (cap < 14) return INFW_PK_DROP_SHORT;                      // kernel.c:423-426
    int v4;
    if (et == 0x0800) v4 = 1;                                     // :428
    else if (et == 0x86DD) v4 = 0;                                // :432
    else return INFW_PK_PASS_NONIP;                               // :436-438
    uint32_t l4 = v4 ? 34u : 54u;                                 // :104, :111
    uint32_t need;
    int c;
    switch (proto) {                                              // :117-172
    case 6: need = 20; c = INFW_CLS_TCP; break;
    case 17: need = 8; c = INFW_CLS_UDP; break;
    case 132: need = 12; c = INFW_CLS_SCTP; break;
    case 1: need = 8; c = v4 ? INFW_CLS_ICMP4 : INFW_CLS_1_ON_V6; break;
    case 58: need = 8; c = v4 ? INFW_CLS_58_ON_V4 : INFW_CLS_ICMP6; break;
    default: return INFW_PK_UNDEF;
    }
    if (cap < l4 + need) return INFW_PK_UNDEF;                    // truncated header
    if (c <= INFW_CLS_SCTP) *val = (l4word >> 8 & 0xFF00u) | (l4word >> 24);  // ntohs(dest)
    else *val = (l4word << 8 & 0xFF00u) | (l4word >> 8 & 0xFFu);              // type << 8 | code
    *cls = c;
    return v4 ? INFW_PK_V4 : INFW_PK_V6;
}

// Table pointers are read through T so host and device share the walk.
template <class T>
INFW_TD int infw_if_slot(const T &t, uint32_t ifindex) {
    uint32_t h = infw_if_hash(ifindex) & t.if_mask;
    for (;;) {
        uint32_t s = t.if_slot[h];
        if (s == INFW_IF_EMPTY) return -1;
        if (t.if_keys[h] == ifindex) return (int)s;
        h = (h + 1) & t.if_mask;
    }
}

template <class T>
INFW_TD uint32_t infw_dir_lookup(const T &t, uint32_t slot, uint32_t a32) {
    uint32_t e = t.tbl24[((uint64_t)slot << 24) | (a32 >> 8)];
    if (e & INFW_TBL8_FLAG) e = t.tbl8[((uint64_t)(e & ~INFW_TBL8_FLAG) << 8) | (a32 & 0xFFu)];
    return e;
}

template <class T>
INFW_TD uint32_t infw_long_lookup(const T &t, uint32_t slot, uint64_t hi, uint64_t lo) {
    int L = 0, R = (int)t.n_levels - 1;
    uint32_t best = 0;
    while (L <= R) {
        int mid = (L + R) >> 1;
        uint32_t len = t.levels[mid];
        uint64_t h = hi, l = lo;
        infw_mask128(len, &h, &l);
        uint32_t tag = slot << 8 | len;
        uint64_t i = infw_long_hash(tag, h, l) & t.lmask;
        bool hit = false;
        for (;;) {
            const struct infw_long_entry *e = &t.ltab[i];
            uint32_t etag = e->tag;
            if (etag == 0) break;
            if (etag == tag && e->hi == h && e->lo == l) {
                hit = true;
                best = e->bmp;
                break;
            }
            i = (i + 1) & t.lmask;
        }
        if (hit) L = mid + 1;
        else R = mid - 1;
    }
    return best;
}

// list+1 of the longest matching entry, 0 if none.
template <class T>
INFW_TD uint32_t infw_lpm(const T &t, int pk, uint32_t ifindex, const uint32_t sa[4]) {
    int slot = infw_if_slot(t, ifindex);
    if (slot < 0) return 0;
    uint32_t a32 = infw_bswap32(sa[0]);
    if (pk == INFW_PK_V6 && t.n_levels) {
        uint32_t r = infw_long_lookup(t, (uint32_t)slot, infw_be64(sa[0], sa[1]), infw_be64(sa[2], sa[3]));
        if (r) return r;
    }
    return infw_dir_lookup(t, (uint32_t)slot, a32);
}

// First match of class list (off, cnt) against value v (serial form).
template <class T>
INFW_TD uint32_t infw_scan_serial(const T &t, uint64_t d, uint32_t v) {
    uint32_t off = (uint32_t)d, cnt = (uint32_t)(d >> 32);
    for (uint32_t k = 0; k < cnt; k++) {
        uint64_t r = t.rules[off + k];
        uint32_t lo = (uint32_t)r & 0xFFFFu, hi = (uint32_t)(r >> 16) & 0xFFFFu;
        if (lo <= v && v <= hi) return (uint32_t)(r >> 32);
    }
    return 0;
}
