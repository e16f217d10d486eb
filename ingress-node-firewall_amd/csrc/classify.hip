// classify.hip — gfx950 kernel for the batched XDP classification
// (bpf/ingress_node_firewall_kernel.c:412-457 over one SoA batch).
//
// A persistent grid of kBlock-thread workgroups strides over the batch one
// tile (kBlock packets, one per lane) at a time.  Per tile:
//   1. each lane loads one 32-B tuple (five coalesced non-temporal streams; the
//      next tile's tuple is in flight while this one walks the tables), parses
//      it (infw_parse) and walks the LPM (ifindex map in LDS -> IPv6 /32-group
//      bucket -> DIR-24-8);
//   2. first match (default, G == 0): the LPM answer addresses the 64-B
//      decision-table entry line of (list, class) directly; an entry with more
//      than 10 segments selects one 64-B leaf line — at most two table lines per
//      packet after the LPM (infw_tables.h).  G > 0 keeps the one-lane-per-rule
//      ballot scan of the class list (the reference's in-order scan,
//      kernel.c:222-258, one wave step per 64 rules, G packets in flight);
//   3. result words / verdicts are stored coalesced; allow/deny counters are
//      summed per wavefront for the leading counter slot, the rest go to LDS
//      atomics (u32 packets, u64 bytes per rule id), flushed with one u64
//      atomic per touched counter when the workgroup retires.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/infw.h"
#include "infw_tables.h"
#include "infw_launch.h"

namespace {

constexpr int kStatKeys = INFW_MAX_TARGETS;
// rule ids with a workgroup counter in LDS (the Go loader writes 1..99, loader.go:437); higher ids (< 1024) add
// straight to the device counters
constexpr int kLdsStatKeys = 128;
constexpr uint32_t kBigLen = 1u << 20;                      // frames this long skip the packed LDS counters
constexpr unsigned long long kBytesMask = (1ull << 40) - 1;  // bytes field of a packed LDS counter
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kIfLds = 256;  // ifindex map entries mirrored in LDS
// word tags of the IPv6 group cache: tag ^ C_j in word j (distinct, so an all-zero entry never validates)
constexpr uint32_t kB6C0 = 0x00000001u, kB6C1 = 0x5bd1e995u, kB6C2 = 0x9e3779b9u, kB6C3 = 0xc2b2ae35u;

// Short-table lookup through the workgroup's LDS cache of DIR-24-8 words.  Traffic
// is heavy-tailed (at configs[2] the top 500 of 1M prefixes carry ~65 % of the hits),
// so a 1024-entry direct-mapped cache answers about half of the IPv4 lookups
// without an L2 request.  An entry is one 64-bit word {valid, slot << 24 | /24,
// list+1} written and read whole, so lanes racing on a slot can only replace
// one complete entry by another: a hit is always the table's own word.  Only
// plain words are cached; inline /24s and tbl8 groups take the table path.
// Decode a DIR-24-8 word for address a32 (tbl8 only for a /24 with > 3 runs).
__device__ __forceinline__ uint32_t d24_value(const infw_dev_tables &T, uint64_t w, uint32_t a32) {
    // plain and inline words decode as selects; only a tbl8 group (a /24 of > 3 runs) branches to its load
    const uint32_t inl = infw_d24_inline(w, a32 & 0xFFu);
    uint32_t v = (w & INFW_D24_GROUP) ? inl : (uint32_t)w;
    if ((w & (INFW_D24_GROUP | INFW_D24_INLINE)) == INFW_D24_GROUP) v = T.tbl8[((uint64_t)(uint32_t)w << 8) | (a32 & 0xFFu)];
    return v;
}

// kLean: the epoch has no compressed short table (DIR-24-8 or none), no overflowed IPv6 group and no
// partial-ifindex prefix (infw_dev_tables.lean), so those paths are compiled out.
// kD16: the LDS word cache holds /16 words instead of /24 answers: entry i = two 8-B halves {tag ^ C, half of
// the word}, tag = slot << 16 | /16 with bit 31 set; a torn pair fails the tag check.
constexpr uint32_t kD16C0 = 0x5bd1e995u, kD16C1 = 0x9e3779b9u;
template <int kLog>
__device__ __forceinline__ uint32_t d16c_idx(uint32_t key16) { return (key16 * 0x9E3779B1u) >> (32 - (kLog - 1)); }
__device__ __forceinline__ bool d16c_get(const unsigned long long *s, uint32_t idx, uint32_t key16, uint64_t &w) {
    const unsigned long long e0 = s[2 * idx], e1 = s[2 * idx + 1];
    const uint32_t tag = key16 | 0x80000000u;
    w = (e1 << 32) | (e0 & 0xFFFFFFFFull);
    return (uint32_t)(e0 >> 32) == (tag ^ kD16C0) && (uint32_t)(e1 >> 32) == (tag ^ kD16C1);
}
__device__ __forceinline__ void d16c_put(unsigned long long *s, uint32_t idx, uint32_t key16, uint64_t w) {
    const uint32_t tag = key16 | 0x80000000u;
    s[2 * idx] = (unsigned long long)(tag ^ kD16C0) << 32 | (uint32_t)w;
    s[2 * idx + 1] = (unsigned long long)(tag ^ kD16C1) << 32 | (uint32_t)(w >> 32);
}

// kD16: the epoch has /16 words in front of DIR-24-8 (infw_tables.h); a /16 they answer needs no tbl24 word.
template <bool kCache, int kLog, bool kLean = false, bool kD16 = false>
__device__ __forceinline__ uint32_t short_lookup_cached(const infw_dev_tables &T, uint32_t slot, uint32_t a32,
                                                        unsigned long long *s_c24) {
    if (!kCache || T.short_mode != INFW_SHORT_DIR24 || slot >= 256u)
        return kLean ? (T.short_mode == INFW_SHORT_DIR24 ? (kD16 ? infw_d16_lookup(T, slot, a32) : infw_dir24_lookup(T, slot, a32))
                        : 0u)
                     : infw_short_lookup(T, slot, a32);
    if (kD16) {  // the LDS cache holds /16 words: a cached or fetched inline word answers, else the tbl24 word
        const uint32_t key16 = slot << 16 | a32 >> 16, di = d16c_idx<kLog>(key16);
        uint64_t d;
        if (!d16c_get(s_c24, di, key16, d)) {
            d = T.d16[((uint64_t)slot << 16) | (a32 >> 16)];
            d16c_put(s_c24, di, key16, d);
        }
        if (d & INFW_D16_INLINE) return infw_d16_value(d, a32 & 0xFFFFu);
        return infw_dir24_lookup(T, slot, a32);
    }
    const uint32_t key = slot << 24 | a32 >> 8;
    const uint32_t idx = (key * 0x9E3779B1u) >> (32 - kLog);
    const unsigned long long e = s_c24[idx];
    if ((e >> 63) && (uint32_t)(e >> 31) == key) return (uint32_t)e & 0x7FFFFFFFu;
    const uint64_t w = T.tbl24[((uint64_t)slot << 24) | (a32 >> 8)];
    if (w & INFW_D24_GROUP) {
        if (w & INFW_D24_INLINE) return infw_d24_inline(w, a32 & 0xFFu);
        return T.tbl8[((uint64_t)(uint32_t)w << 8) | (a32 & 0xFFu)];
    }
    s_c24[idx] = 1ull << 63 | (unsigned long long)key << 31 | (uint32_t)w;  // list+1 < 2^25
    return (uint32_t)w;
}

__device__ __forceinline__ uint32_t readlane(uint32_t v, int lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}

// Sum over the 64 lanes of a wave with every lane active (DPP: row_shr 1/2/4/8 inside each 16-lane row,
// then row_bcast 15/31 across rows; lane 63 ends with the total).
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
    uint32_t v = x;
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return readlane(v, 63);
}

__device__ __forceinline__ bool rec_match(uint64_t rec, uint32_t v) {
    const uint32_t lo = (uint32_t)rec & 0xFFFFu, hi = (uint32_t)(rec >> 16) & 0xFFFFu;
    return lo <= v && v <= hi;
}

// First match of a class list (o, c) against v, starting at rule `from`, one lane per rule.
__device__ __forceinline__ uint32_t scan_tail(const uint64_t *__restrict__ rules, uint32_t o, uint32_t c,
                                              uint32_t v, uint32_t from, int lane) {
    for (uint32_t k0 = from; k0 < c; k0 += 64) {
        const uint32_t k = k0 + lane;
        uint64_t rec = 0;
        bool m = false;
        if (k < c) {
            rec = rules[(uint64_t)o + k];
            m = rec_match(rec, v);
        }
        const uint64_t mb = __ballot(m);
        if (mb) return readlane((uint32_t)(rec >> 32), __builtin_ctzll(mb));
    }
    return 0;
}

// First-match result from the decision-table lines of (list, cls) (infw_tables.h),
// one lane per packet: the entry line, and for S > 10 one leaf line, each read
// whole (four 16-B loads of one 64-B line, issued back to back).
// Keys below v in u16 pairs, two at a time in packed 16-bit math: v - key saturates to 0 unless key < v,
// min(., 1) makes it an indicator, and the two halves accumulate separately (1.5 VALU per key instead of
// a compare, a select and an add-with-carry per key).
struct KeyCount {
    uint32_t vv, acc = 0;
    __device__ __forceinline__ explicit KeyCount(uint32_t v) : vv(v | v << 16) {}
    __device__ __forceinline__ void add(uint32_t w) {
        // per half: sat(v - key) > 0 <=> key < v; min(., 1) -> 0/1.  The halves count at most 15 each, so
        // the indicators accumulate in one 32-bit add without a carry crossing between them.
        uint32_t d, r;
        asm("v_pk_sub_u16 %0, %1, %2 clamp" : "=v"(d) : "v"(vv), "v"(w));
        asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(d), "s"(0x00010001u));
        acc += r;
    }
    __device__ __forceinline__ uint32_t total() const { return (acc & 0xFFFFu) + (acc >> 16); }
};
__device__ __forceinline__ uint32_t dt_u32_leaf(u32x4 a, u32x4 b, u32x4 c, u32x4 d, uint32_t v) {
    KeyCount kc(v);
    kc.add(a[1]); kc.add(a[2]); kc.add(a[3]); kc.add(b[0]); kc.add(b[1]);
    const uint32_t k = kc.total();
    uint32_t r = b[2];
    r = k >= 1 ? b[3] : r;
    r = k >= 2 ? c[0] : r;
    r = k >= 3 ? c[1] : r;
    r = k >= 4 ? c[2] : r;
    r = k >= 5 ? c[3] : r;
    r = k >= 6 ? d[0] : r;
    r = k >= 7 ? d[1] : r;
    r = k >= 8 ? d[2] : r;
    r = k >= 9 ? d[3] : r;
    return r;
}
__device__ __forceinline__ uint32_t dt_root_index(u32x4 a, u32x4 b, u32x4 c, u32x4 d, uint32_t v) {
    KeyCount g(v);
    g.add(a[1]); g.add(a[2]); g.add(a[3]); g.add(b[0]); g.add(b[1]); g.add(b[2]); g.add(b[3]);
    g.add(c[0]); g.add(c[1]); g.add(c[2]); g.add(c[3]); g.add(d[0]); g.add(d[1]); g.add(d[2]); g.add(d[3]);
    return (a[0] & INFW_DT_INDEX) + g.total();
}
// The whole 64-B line at once (four 16-B loads issued back to back); the compact leaf decoded without branches.
__device__ __forceinline__ uint32_t dt_lookup_full(const infw_dt_line *__restrict__ dte,
                                                   const infw_dt_line *__restrict__ dtl, uint64_t slot, uint32_t v) {
    const u32x4 *e = reinterpret_cast<const u32x4 *>(dte + slot);
    u32x4 a = e[0], b = e[1], c = e[2], d = e[3];
    if (a[0] & INFW_DT_ROOT) {
        const u32x4 *l = reinterpret_cast<const u32x4 *>(dtl + dt_root_index(a, b, c, d, v));
        a = l[0];
        b = l[1];
        c = l[2];
        d = l[3];
    }
    if (a[0] & INFW_DT_COMPACT) {  // half-first layout (infw_tables.h): keys 0..7, codes 0..11, keys 8..19, codes 12..19
        KeyCount kc(v);
        kc.add(a[1]); kc.add(a[2]); kc.add(a[3]); kc.add(b[0]);
        kc.add(c[0]); kc.add(c[1]); kc.add(c[2]); kc.add(c[3]); kc.add(d[0]); kc.add(d[1]);
        const uint32_t k = kc.total();
        uint32_t w = b[1];
        w = k >= 4 ? b[2] : w;
        w = k >= 8 ? b[3] : w;
        w = k >= 12 ? d[2] : w;
        w = k >= 16 ? d[3] : w;
        return infw_dt_code_result(__builtin_amdgcn_ubfe(w, 8 * (k & 3u), 8));
    }
    return dt_u32_leaf(a, b, c, d, v);
}
// Half-first: the line's first 32 B; the second 32 B only where needed — a root's keys, a u32-form leaf, a compact
// leaf of > 9 segments whose value lies past its key 8.  For epochs of short step functions (choose_dt_half).
__device__ __forceinline__ uint32_t dt_lookup_half(const infw_dt_line *__restrict__ dte,
                                                   const infw_dt_line *__restrict__ dtl, uint64_t slot, uint32_t v) {
    const u32x4 *L = reinterpret_cast<const u32x4 *>(dte + slot);
    u32x4 a = L[0], b = L[1];
    if (a[0] & INFW_DT_ROOT) {
        const u32x4 c = L[2], d = L[3];
        L = reinterpret_cast<const u32x4 *>(dtl + dt_root_index(a, b, c, d, v));
        a = L[0];
        b = L[1];
    }
    if (a[0] & INFW_DT_COMPACT) {
        KeyCount kc(v);
        kc.add(a[1]); kc.add(a[2]); kc.add(a[3]); kc.add(b[0]);  // keys 0..7
        uint32_t k = kc.total();
        if (k == 8 && (a[0] & 0xFFu) > 9) {
            const u32x4 c = L[2], d = L[3];
            KeyCount k2(v);
            k2.add(c[0]); k2.add(c[1]); k2.add(c[2]); k2.add(c[3]); k2.add(d[0]); k2.add(d[1]);  // keys 8..19
            k += k2.total();
            if (k >= 12) return infw_dt_code_result(__builtin_amdgcn_ubfe(k >= 16 ? d[3] : d[2], 8 * (k & 3u), 8));
        }
        const uint32_t w = k < 4 ? b[1] : k < 8 ? b[2] : b[3];  // codes 0..11
        return infw_dt_code_result(__builtin_amdgcn_ubfe(w, 8 * (k & 3u), 8));
    }
    return dt_u32_leaf(a, b, L[2], L[3], v);
}
template <bool kHalf = false>
__device__ __forceinline__ uint32_t dt_lookup_at(const infw_dt_line *__restrict__ dte, const infw_dt_line *__restrict__ dtl,
                                                 uint64_t slot, uint32_t v) {
    return kHalf ? dt_lookup_half(dte, dtl, slot, v) : dt_lookup_full(dte, dtl, slot, v);
}
template <bool kHalf = false>
__device__ __forceinline__ uint32_t dt_lookup(const infw_dt_line *__restrict__ dte, const infw_dt_line *__restrict__ dtl,
                                              uint32_t list, int cls, uint32_t v, uint32_t plog2, uint32_t p) {
    return dt_lookup_at<kHalf>(dte, dtl, infw_dt_slot_p(list, cls, v, plog2, p), v);
}

// Longest /33../128 prefix covering an IPv6 address (infw_v6_long, device form):
// each probe reads the whole 64-B bucket — header and the three records — in one
// round of loads, so a lane's probe costs one dependent L2 round trip, not one
// for the header and one per record examined.
// Finish a first bucket probe whose header h and first record r0 are already loaded:
// most groups hold one record, so records 1..2 (and further probes) load on demand.
template <bool kLean = false>
__device__ __forceinline__ uint32_t v6_finish(const infw_dev_tables &T, uint32_t slot, uint32_t a32,
                                             const uint32_t sa[4], uint64_t i, u32x4 h, u32x4 r0) {
    const uint32_t mid = infw_bswap32(sa[1]);
    const uint64_t lo = infw_be64(sa[2], sa[3]);
    for (;;) {
        if (h[0] == 0) return 0;
        if (h[0] == slot + 1 && h[1] == a32) {
            const uint32_t nb = h[2];
            if (nb == INFW_BUCKET_OVERFLOW) return kLean ? 0u : infw_long_lookup(T, slot, (uint64_t)a32 << 32 | mid, lo);
            if (nb >= 1 && infw_rec_match(r0[2], (uint64_t)r0[1] << 32 | r0[0], r0[3], mid, lo)) return r0[3] & 0x1FFFFFFu;
            if (nb >= 2) {
                const u32x4 *b = reinterpret_cast<const u32x4 *>(T.btab + i);
                const u32x4 r1 = b[2], r2 = b[3];
                if (infw_rec_match(r1[2], (uint64_t)r1[1] << 32 | r1[0], r1[3], mid, lo)) return r1[3] & 0x1FFFFFFu;
                if (nb >= 3 && infw_rec_match(r2[2], (uint64_t)r2[1] << 32 | r2[0], r2[3], mid, lo))
                    return r2[3] & 0x1FFFFFFu;
            }
            return 0;
        }
        i = (i + 1) & T.bmask;
        const u32x4 *b = reinterpret_cast<const u32x4 *>(T.btab + i);
        h = b[0];
        r0 = b[1];
    }
}

// The batch as the kernel reads it: the 16-B address layout (infw_batch_soa) or the
// family-compact one (infw_batch_soa_c: 4 address bytes per packet + the IPv6 packets'
// remaining 12 bytes packed at the front of a 768-B block per 64-packet group).
struct BatchIn {
    const uint8_t *saddr;    // 16 B per packet (standard layout)
    const uint32_t *saddr4;  // compact layout
    const uint8_t *v6tail;
    const uint32_t *ifindex, *pkt_len, *meta, *l4word;
    // raw frames (kF, infw_frame_batch): pkt_len may be null (= linear length); offsets null = fixed stride
    const uint8_t *frames;
    const uint64_t *offsets;
    uint64_t fstride;
    const uint32_t *linear_len;
    // or AF_XDP RX descriptors (infw_classify_xdp): {addr, len, options} per frame into `frames` (the umem), one
    // ifindex for the ring; addr's bits 48..63 carry the unaligned-mode offset (XSK_UNALIGNED_BUF_OFFSET_SHIFT)
    const u32x4 *xdp;
    uint32_t xdp_ifindex;
    // kSplit (the two-phase form): phase 1 writes one word per packet here (split_word), phase 2 reads it
    uint64_t *mid;
};

// ---- raw frames (kF): the tuple of infw_pack_header() (infw_pack.h) built in the kernel from the frame's
// header window, bytes [10, 58) — every byte kernel.c reads (ethertype :427, protocol :108/:115, saddr :204/:291,
// the first L4 word at the fixed offset 34/54 :125-166).  A wave stages its 64 frames 16 at a time through a
// 1-KiB LDS buffer of its own: lanes 4j..4j+3 load the four 16-B aligned chunks covering frame j's window (one
// instruction moves 16 whole 64-B windows), then frame j's owner lane picks its fields out of LDS.  A chunk is
// read only when it starts before min(linear length, 58), so frames packed back to back are never read past
// their end; bytes at or past the linear length read as zero, as the packer's do.
constexpr uint32_t kFrameWinWords = 17;  // 64-B window + 4 B: the 16 owners' reads spread over the banks
__device__ __forceinline__ uint32_t bperm(uint32_t v, uint32_t src_lane) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)v);
}
// Frame bytes [o, o + 4) from a staged window w whose byte 10 sits at position d, bytes >= cap as zero.
__device__ __forceinline__ uint32_t frame_word(const uint32_t *w, uint32_t d, uint32_t o, uint32_t cap) {
    const uint32_t p = o - 10u + d, q = p >> 2;
    const uint32_t x = __builtin_amdgcn_alignbyte(w[q + 1], w[q], p & 3u);
    const int keep = (int)cap - (int)o;
    return keep >= 4 ? x : keep <= 0 ? 0u : x & ((1u << (8 * keep)) - 1u);
}

// G > 0: one-lane-per-rule ballot scan with G packets in flight; G == 0: decision tables.
struct EventSink {
    infw_event_rec *rec;
    uint64_t cap;
    unsigned long long *count;
};

// Debug lookup capture (kernel.c:214-216, :297-299): an open-addressed set of
// 2 * INFW_DBG_MAX_ENTRIES slots, a 64-bit key fingerprint per slot (0 = free)
// claimed by CAS, the 24-B key beside it, and the number of keys held.
struct DebugSink {
    unsigned long long *fp;
    uint32_t *keys;      // 6 words per slot
    unsigned int *count;
    uint32_t mask;
};

struct Sideband {
    EventSink ev;
    DebugSink dbg;
};

__device__ __forceinline__ uint64_t dbg_fingerprint(const uint32_t k[6]) {
    uint64_t h = 0x243F6A8885A308D3ull;
    for (int j = 0; j < 6; j++) {
        h = (h ^ k[j]) * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
    }
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 32;
    return h | 1;
}

// bpf_map_update_elem(&dbg_map, &key, &key, BPF_NOEXIST): present -> no-op, full -> dropped.
// Slots are claimed by CAS (global atomics are performed at the memory side, so all XCDs agree),
// then counted; a claim that finds the set full turns its slot into a tombstone, which probes
// step over like any other key, so no probe chain ever breaks.  A plain read first lets repeats of
// a held key return without an atomic (it can only be stale towards "free" or "tombstoned").
constexpr unsigned long long kDbgTomb = 2ull;  // fingerprints are odd
__device__ __noinline__ void dbg_insert(const DebugSink &d, const uint32_t k[6]) {
    const uint64_t fp = dbg_fingerprint(k);
    uint32_t i = (uint32_t)(fp >> 32) & d.mask;
    for (uint32_t probe = 0; probe <= d.mask; probe++) {
        if (__hip_atomic_load(&d.fp[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == fp) return;
        const uint64_t old = atomicCAS(&d.fp[i], 0ull, (unsigned long long)fp);
        if (old == fp) return;  // held
        if (old == 0) {         // claimed: count it, or give the slot up as a tombstone when full
            if (atomicAdd(d.count, 1u) < INFW_DBG_MAX_ENTRIES) {
                uint32_t *dst = d.keys + 6ull * i;
                for (int j = 0; j < 6; j++) dst[j] = k[j];
            } else {
                atomicSub(d.count, 1u);
                atomicExch(&d.fp[i], kDbgTomb);
            }
            return;
        }
        i = (i + 1) & d.mask;
    }
}

// ---- the two-phase form (infw_dev_tables.split; chosen at commit for epochs with many distinct rule lists,
// abi.cpp bind_view).  In the fused kernel every decision-line read depends on the packet's LPM answer; when the
// entry lines span GiBs (one list per key, random update order) each such dependent read pays for the span (DESIGN.md
// §7: dependent read pairs 27 -> 19 G/s from a 1- to a 12-GiB span, independent reads 53-57 G/s at any span).  Phase 1
// (classify_kernel<..., kSplit>) walks the LPM and writes one word per packet; phase 2 (decide_kernel) reads those
// words as a stream and the entry lines as independent gathers, then does the counters, results and verdicts.
// Word: bit 63 = a decision line to read: entry-line index in bits 0..30, the packet value (dport or type << 8 |
// code) in bits 31..46, min(frame length, 0xFFFF) in bits 47..62 (0xFFFF: read pkt_len); else 0 (no list: result 0)
// or 1 (too short: XDP_DROP, kernel.c:423-426).
__device__ __forceinline__ uint64_t split_word(uint64_t slot, uint32_t val, uint32_t plen) {
    return 1ull << 63 | (uint64_t)(plen < 0xFFFFu ? plen : 0xFFFFu) << 47 | (uint64_t)val << 31 | slot;
}

template <int kBlock>
__global__ __launch_bounds__(kBlock) void decide_kernel(const infw_dev_tables T, const uint64_t *__restrict__ mid,
                                                        const uint32_t *__restrict__ pkt_len, uint64_t n,
                                                        uint32_t *__restrict__ results, uint8_t *__restrict__ verdicts,
                                                        unsigned long long *__restrict__ stats) {
    __shared__ unsigned long long s_c[2 * kLdsStatKeys];  // as classify_kernel's: packets << 40 | bytes
    for (int i = threadIdx.x; i < 2 * kLdsStatKeys; i += kBlock) s_c[i] = 0;
    auto flush_counters = [&]() {
        for (int s = threadIdx.x; s < 2 * kLdsStatKeys; s += kBlock) {
            const unsigned long long c = s_c[s];
            if (c) {
                unsigned long long *dst = stats + (s >> 1) * 4 + (s & 1) * 2;
                atomicAdd(dst, c >> 40);
                atomicAdd(dst + 1, c & kBytesMask);
                s_c[s] = 0;
            }
        }
    };
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    uint32_t tiles_since_flush = 0;
    uint64_t nw = 0;  // the next tile's word, loaded a tile ahead
    {
        const uint64_t i0 = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
        if (i0 < n) nw = __builtin_nontemporal_load(&mid[i0]);
    }
    for (uint64_t base = (uint64_t)blockIdx.x * kBlock; base < n; base += stride) {
        const uint64_t i = base + threadIdx.x;
        const bool valid = i < n;
        const uint64_t w = valid ? nw : 0;
        if (i + stride < n) nw = __builtin_nontemporal_load(&mid[i + stride]);
        uint32_t result = 0, plen = 0;
        if (w >> 63) {
            plen = (uint32_t)(w >> 47) & 0xFFFFu;
            if (plen == 0xFFFFu) plen = pkt_len[i];
            result = dt_lookup_at(T.dte, T.dtl, w & 0x7FFFFFFFull, (uint32_t)(w >> 31) & 0xFFFFu);
        }
        // ---- verdict (kernel.c:444-456) and statistics (kernel.c:376-387), as in classify_kernel
        const uint32_t action = result & 0xFFu;
        const uint32_t key = (result >> 8) & 0xFFFFu;
        const int s0_ = ((action == INFW_XDP_DROP || action == INFW_XDP_PASS) && key < kStatKeys)
                            ? (int)key * 2 + (action == INFW_XDP_DROP) : -1;
        const bool lds = plen < kBigLen && key < (uint32_t)kLdsStatKeys;
        if (s0_ >= 0 && !lds) {
            unsigned long long *dst = stats + (s0_ >> 1) * 4 + (s0_ & 1) * 2;
            atomicAdd(dst, 1ull);
            atomicAdd(dst + 1, (unsigned long long)plen);
        }
        const int s = lds ? s0_ : -1;
        const uint64_t elig = __ballot(s >= 0);
        if (elig) {
            const int lead = __builtin_ctzll(elig);
            const int s0 = __builtin_amdgcn_readlane(s, lead);
            const bool mine = s == s0;
            const uint64_t grp = __ballot(mine);
            const uint32_t by = wave_sum(mine ? plen : 0u);
            if (lane == lead) atomicAdd(&s_c[s0], (unsigned long long)__popcll(grp) << 40 | by);
            if (s >= 0 && !mine) atomicAdd(&s_c[s], 1ull << 40 | plen);
        }
        if (valid) {
            if (results) __builtin_nontemporal_store(result, &results[i]);
            if (verdicts) verdicts[i] = (w == 1u || action == INFW_XDP_DROP) ? INFW_XDP_DROP : INFW_XDP_PASS;
        }
        if (++tiles_since_flush == T.stat_flush_tiles) {  // every workgroup runs the same number of tiles
            __syncthreads();
            flush_counters();
            __syncthreads();
            tiles_since_flush = 0;
        }
    }
    __syncthreads();
    flush_counters();
}

// One instantiation per selectable variant (the registry below):
//   kWaves   minimum waves per SIMD the register allocation must allow (8 = four 512-thread workgroups per CU;
//            6 leaves room for 104 SGPRs, no spills);
//   kIn      batch form: 0 SoA tuples (infw_batch_soa), 1 family-compact (infw_batch_soa_c), 2 raw frames,
//            3 raw frames named by AF_XDP descriptors (its own instantiation: the frames kernel keeps no branch);
//   kC24Log  LDS word cache of 1 << kC24Log entries (workgroups of >= 384 threads), kB6Log the IPv6 group cache
//            (0: none);
//   kEvents / kDebug  the deny-event and debug-lookup sidebands;
//   kLean    the epoch has no compressed short table, overflowed IPv6 group or partial-ifindex prefix;
//   kPl      per-list part counts mirrored in LDS; kD16 /16 words in front of DIR-24-8; kHalf half-first
//            decision-line reads; kSplit phase 1 of the two-phase form.
template <int kBlock, int G, int kWaves, int kIn, int kC24Log, int kB6Log, bool kEvents, bool kDebug, bool kLean,
          bool kPl, bool kD16, bool kSplit, bool kHalf>
__global__ __launch_bounds__(kBlock, kWaves) void classify_kernel(const infw_dev_tables T, const BatchIn in,
                                                          uint64_t n, uint32_t *__restrict__ results,
                                                          uint8_t *__restrict__ verdicts,
                                                          unsigned long long *__restrict__ stats,
                                                          const Sideband sb) {
    constexpr bool kC = kIn == 1, kF = kIn == 2 || kIn == 3, kX = kIn == 3;
    const EventSink &ev = sb.ev;
    // per-workgroup counters [rule][allow=0, deny=1], packets << 40 | bytes in one u64 (one LDS atomic per update):
    // only frames shorter than kBigLen take this path and the workgroup flushes every kFlushTiles tiles, so
    // neither field can carry into the other (kFlushTiles * kBlock * kBigLen < 2^40)
    __shared__ unsigned long long s_c[2 * kLdsStatKeys];
    __shared__ uint32_t s_ifk[kIfLds], s_ifs[kIfLds];  // ifindex -> slot map, when it fits
    // the 256-thread shapes (6 blocks per CU) have no LDS room for the word cache
    constexpr bool kCache = kBlock >= 384;
    constexpr uint32_t kC24 = 1u << kC24Log;
    __shared__ unsigned long long s_c24[kCache ? kC24 : 1];
    if (kCache)
        for (int i = threadIdx.x; i < (int)kC24; i += kBlock) s_c24[i] = 0;
    // per-workgroup LDS cache of single-record IPv6 groups of slots < 256: 1 << kB6Log entries of four
    // 8-B words {tag ^ C_j, payload_j}, payloads = the record {lo low, lo high, mid, meta}.  The entry
    // index and tag are the top bits and the low 32 bits of infw_b6_key(slot, top), a bijection of the
    // group key, so a word whose tag matches was written for the reader's own group: lanes racing on an
    // entry, torn at any 8-B granularity, can only leave words of several groups, which fail the check —
    // no access needs to be indivisible beyond 8 B.  The distinct C_j keep a zeroed entry from validating.
    constexpr bool kB6 = kB6Log > 0;
    __shared__ u32x4 s_b6[kB6 ? 2u << kB6Log : 1];
    __shared__ uint32_t s_fw[kF ? kBlock / 64 : 1][kF ? 16 * kFrameWinWords : 1];  // per-wave frame windows
    // kPl: the per-list part-count words (T.n_dt_pl == INFW_DT_PL_LISTS) mirrored in LDS
    __shared__ uint32_t s_pl[kPl ? INFW_DT_PL_LISTS : 1];
    if (kPl)
        for (uint32_t i = threadIdx.x; i < INFW_DT_PL_LISTS; i += kBlock) s_pl[i] = T.dt_pl[i];
    if (kB6)
        for (int i = threadIdx.x; i < (int)(2u << kB6Log); i += kBlock) s_b6[i] = u32x4{0u, 0u, 0u, 0u};
    for (int i = threadIdx.x; i < 2 * kLdsStatKeys; i += kBlock) s_c[i] = 0;
    // the workgroup's counters -> the device's (one u64 atomic per touched counter), zeroed for the next tiles
    auto flush_counters = [&]() {
        for (int s = threadIdx.x; s < 2 * kLdsStatKeys; s += kBlock) {
            const unsigned long long c = s_c[s];
            if (c) {
                unsigned long long *dst = stats + (s >> 1) * 4 + (s & 1) * 2;
                atomicAdd(dst, c >> 40);
                atomicAdd(dst + 1, c & kBytesMask);
                s_c[s] = 0;
            }
        }
    };
    uint32_t tiles_since_flush = 0;
    const bool if_in_lds = T.if_mask < kIfLds;
    if (if_in_lds)
        for (uint32_t i = threadIdx.x; i <= T.if_mask; i += kBlock) {
            s_ifk[i] = T.if_keys[i];
            s_ifs[i] = T.if_slot[i];
        }
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const uint4 *sa4 = reinterpret_cast<const uint4 *>(in.saddr);
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t *__restrict__ rules = T.rules;

    // the next tile's tuple is loaded while the current tile walks the tables:
    // the stream's latency overlaps the first table lookups instead of adding to them
    auto load_tuple = [&](uint64_t i, uint32_t &meta, uint32_t &l4w, uint32_t &ifx, uint32_t &plen, uint4 &sa,
                          bool with_meta = true) {
        if (kF) {  // frames: linear length (meta), frame byte offset (sa.x/sa.y), ifindex, frame length
            if (kX && i < n) {  // one 16-B descriptor per frame
                const u32x4 d = __builtin_nontemporal_load(&in.xdp[i]);
                const uint64_t a = (uint64_t)d[1] << 32 | d[0];
                const uint64_t off = (a & ((1ull << 48) - 1)) + (a >> 48);
                meta = d[2];
                plen = d[2];
                ifx = in.xdp_ifindex;
                sa.x = (uint32_t)off;
                sa.y = (uint32_t)(off >> 32);
            } else if (!kX && i < n) {
                meta = __builtin_nontemporal_load(&in.linear_len[i]);
                ifx = __builtin_nontemporal_load(&in.ifindex[i]);
                plen = in.pkt_len ? __builtin_nontemporal_load(&in.pkt_len[i]) : meta;
                const uint64_t off = in.offsets ? __builtin_nontemporal_load(&in.offsets[i]) : i * in.fstride;
                sa.x = (uint32_t)off;
                sa.y = (uint32_t)(off >> 32);
            }
            return;
        }
        if (i < n) {  // streamed once: non-temporal, keeps the tables resident in L2/MALL
            if (with_meta) meta = __builtin_nontemporal_load(&in.meta[i]);
            l4w = __builtin_nontemporal_load(&in.l4word[i]);
            ifx = __builtin_nontemporal_load(&in.ifindex[i]);
            plen = __builtin_nontemporal_load(&in.pkt_len[i]);
            if (kC) {
                sa = make_uint4(__builtin_nontemporal_load(&in.saddr4[i]), 0u, 0u, 0u);
            } else {
                const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(sa4) + i);
                sa = make_uint4(t[0], t[1], t[2], t[3]);
            }
        }
    };
    // compact layout: an IPv6 packet's address bytes 4..15 sit in its 64-packet group's block at its rank
    // among the group's IPv6 lanes (one ballot of the meta ethertype)
    auto load_tail = [&](uint64_t i, uint32_t meta, uint32_t &t0, uint32_t &t1, uint32_t &t2) {
        const bool is6 = i < n && (meta & 0xFFFFu) == 0x86DDu;
        const uint64_t m6 = __ballot(is6);
        if (is6) {
            const uint32_t rank = __popcll(m6 & ((1ull << lane) - 1));
            const uint32_t *t = reinterpret_cast<const uint32_t *>(in.v6tail + (i >> 6) * (INFW_V6_GROUP * 12ull)) + 3 * rank;
            t0 = __builtin_nontemporal_load(t);
            t1 = __builtin_nontemporal_load(t + 1);
            t2 = __builtin_nontemporal_load(t + 2);
        }
    };
    uint32_t n_meta = 0, n_l4w = 0, n_ifx = 0, n_plen = 0;
    uint4 n_sa = make_uint4(0, 0, 0, 0);
    // compact: the meta word runs two tiles ahead, so the next tile's tail loads can be issued a
    // whole tile early like the rest of its tuple (issued with the tile's own table loads, the tails' HBM
    // latency would hold back the in-order return of the bucket probes)
    uint32_t n_meta2 = 0, n_t0 = 0, n_t1 = 0, n_t2 = 0;
    {
        const uint64_t i0 = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
        load_tuple(i0, n_meta, n_l4w, n_ifx, n_plen, n_sa);
        if (kC) {
            if (i0 + stride < n) n_meta2 = __builtin_nontemporal_load(&in.meta[i0 + stride]);
            load_tail(i0, n_meta, n_t0, n_t1, n_t2);
        }
    }

    for (uint64_t base = (uint64_t)blockIdx.x * kBlock; base < n; base += stride) {
        const uint64_t i = base + threadIdx.x;
        const bool valid = i < n;
        uint32_t meta = valid ? n_meta : 0, l4w = n_l4w;
        const uint32_t ifx = n_ifx, plen = n_plen;
        uint4 sa = n_sa;
        if (kF) {
            const uint32_t cap = meta;  // linear length (0 past the batch: nothing is read)
            const uint64_t foff = (uint64_t)sa.y << 32 | sa.x;
            load_tuple(i + stride, n_meta, n_l4w, n_ifx, n_plen, n_sa);
            uint32_t *wb = s_fw[threadIdx.x >> 6];
            u32x4 ch[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {  // round r: chunk (lane & 3) of the wave's frame 16r + (lane >> 2)
                const uint32_t src = 16u * r + (lane >> 2);
                const uint32_t c_cap = bperm(cap, src);
                const uint64_t c_off = (uint64_t)bperm((uint32_t)(foff >> 32), src) << 32 | bperm((uint32_t)foff, src);
                const uintptr_t f = (uintptr_t)(in.frames + c_off);
                const uintptr_t at = ((f + 10u) & ~(uintptr_t)15) + 16u * (lane & 3u);
                ch[r] = u32x4{0u, 0u, 0u, 0u};
                if (c_cap > 10u && at < f + (c_cap < 58u ? c_cap : 58u))
                    ch[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(at));
            }
            const uint32_t d = (uint32_t)(((uintptr_t)(in.frames + foff) + 10u) & 15u);
            const uint32_t *w = wb + (lane & 15u) * kFrameWinWords;
            uint32_t et = 0, proto = 0, s0 = 0, s1 = 0, s2 = 0, s3 = 0, l4 = 0;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                uint32_t *dst = wb + (lane >> 2) * kFrameWinWords + 4u * (lane & 3u);
                dst[0] = ch[r][0];
                dst[1] = ch[r][1];
                dst[2] = ch[r][2];
                dst[3] = ch[r][3];
                // the owners read other lanes' LDS writes: a wave-scope release/acquire pair orders them (the
                // wave barrier alone is no memory fence to the compiler)
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if ((lane >> 4) == (uint32_t)r) {  // the round's 16 owners read their frames' fields
                    const uint32_t e = frame_word(w, d, 12, cap);
                    et = cap >= 14u ? (e & 0xFFu) << 8 | ((e >> 8) & 0xFFu) : 0u;
                    const bool v4 = et == 0x0800u, v6 = et == 0x86DDu;
                    const uint32_t f20 = frame_word(w, d, 20, cap);
                    proto = v4 ? f20 >> 24 : v6 ? f20 & 0xFFu : 0u;
                    s0 = v4 ? frame_word(w, d, 26, cap) : v6 ? frame_word(w, d, 22, cap) : 0u;
                    l4 = v4 ? frame_word(w, d, 34, cap) : v6 ? frame_word(w, d, 54, cap) : 0u;
                    if (v6) {
                        s1 = frame_word(w, d, 26, cap);
                        s2 = frame_word(w, d, 30, cap);
                        s3 = frame_word(w, d, 34, cap);
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();  // the next round rewrites the buffer
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            meta = et | proto << 16 | (cap > 255u ? 255u : cap) << 24;
            l4w = l4;
            sa = make_uint4(s0, s1, s2, s3);
        } else if (kC) {
            sa.y = n_t0;
            sa.z = n_t1;
            sa.w = n_t2;
        }
        if (!kF) {
            if (kC) {
                const uint32_t m1 = n_meta2;  // tile t+1's meta, loaded one tile ago
                load_tuple(i + stride, n_meta, n_l4w, n_ifx, n_plen, n_sa, false);
                if (i + 2 * stride < n) n_meta2 = __builtin_nontemporal_load(&in.meta[i + 2 * stride]);
                load_tail(i + stride, m1, n_t0, n_t1, n_t2);
                n_meta = m1;
            } else {
                load_tuple(i + stride, n_meta, n_l4w, n_ifx, n_plen, n_sa);
            }
        }
        int cls = 0;
        uint32_t val = 0;
        const int pk = valid ? infw_parse(meta, l4w, &cls, &val) : INFW_PK_PASS_NONIP;
        uint64_t d = 0;    // ballot mode: class-list descriptor
        uint32_t lst = 0;  // decision mode: list + 1 (0: no LPM entry)
        if (pk >= INFW_PK_V4) {
            const uint32_t sw[4] = {sa.x, sa.y, sa.z, sa.w};
            if (kDebug) {  // lookup key {prefixLen 64|160, ifindex, ip_data} (kernel.c:205-216, :292-299)
                // a full set stays as it is: skip the probe once INFW_DBG_MAX_ENTRIES keys are held
                if (__hip_atomic_load(sb.dbg.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < INFW_DBG_MAX_ENTRIES) {
                    const bool v6 = pk == INFW_PK_V6;
                    const uint32_t key[6] = {v6 ? 160u : 64u, ifx, sa.x, v6 ? sa.y : 0u, v6 ? sa.z : 0u, v6 ? sa.w : 0u};
                    dbg_insert(sb.dbg, key);
                }
            }
            uint32_t l1 = 0;
            {
                // ifindex -> slot (LDS copy of the open-addressed map)
                int slot;
                if (if_in_lds && T.if_mult) {  // collision-free placement: one probe, no loop
                    const uint32_t h = (ifx * T.if_mult) >> T.if_shift;
                    const uint32_t k = s_ifk[h], sl = s_ifs[h];
                    slot = k == ifx && sl != INFW_IF_EMPTY ? (int)sl : -1;
                } else if (if_in_lds) {
                    uint32_t h = infw_if_hash(ifx) & T.if_mask;
                    for (;;) {
                        const uint32_t sl = s_ifs[h];
                        if (sl == INFW_IF_EMPTY) { slot = -1; break; }
                        if (s_ifk[h] == ifx) { slot = (int)sl; break; }
                        h = (h + 1) & T.if_mask;
                    }
                } else {
                    slot = infw_if_slot(T, ifx);
                }
                l1 = 0;
                if (slot >= 0) {
                    // One round of table loads for the whole wave: IPv4 lanes' DIR-24-8 words
                    // and IPv6 lanes' first bucket probe are issued before either is waited
                    // for (a mixed wave would otherwise pay two dependent round trips).  IPv6:
                    // the /32 group's bucket; the short table only when no long prefix covers
                    // the address (2.8 % of them at configs[2]).
                    const uint32_t a32 = infw_bswap32(sa.x);
                    const bool v6 = pk == INFW_PK_V6 && T.n_levels;
                    const bool d24 = T.short_mode == INFW_SHORT_DIR24;
                    const uint32_t key = (uint32_t)slot << 24 | a32 >> 8;
                    const uint32_t cidx = (key * 0x9E3779B1u) >> (32 - kC24Log);
                    bool need24 = !v6 && d24;
                    uint32_t sh = 0;
                    bool d16known = false;  // kD16: the LDS cache held this /16's word and it does not answer
                    const uint32_t key16 = (uint32_t)slot << 16 | a32 >> 16;
                    const uint32_t d16i = kD16 ? d16c_idx<kC24Log>(key16) : 0u;
                    if (kCache && need24 && slot < 256) {
                        if (kD16) {
                            uint64_t dw;
                            if (d16c_get(s_c24, d16i, key16, dw)) {
                                if (dw & INFW_D16_INLINE) {
                                    sh = infw_d16_value(dw, a32 & 0xFFFFu);
                                    need24 = false;
                                } else {
                                    d16known = true;
                                }
                            }
                        } else {
                            const unsigned long long e = s_c24[cidx];
                            if ((e >> 63) && (uint32_t)(e >> 31) == key) {
                                sh = (uint32_t)e & 0x7FFFFFFFu;
                                need24 = false;
                            }
                        }
                    }
                    uint64_t w24 = 0, bi = 0;
                    u32x4 bh = {0, 0, 0, 0}, br0 = {0, 0, 0, 0};
                    uint32_t lng = 0, b6idx = 0, b6tag = 0;
                    bool need6 = v6;
                    uint64_t bhash = 0;
                    if (v6) bhash = infw_bucket_hash((uint32_t)slot, a32);
                    const bool b6ok = kB6 && v6 && slot < 256;
                    if (b6ok) {
                        const uint64_t bk = infw_b6_key((uint32_t)slot, a32);
                        b6idx = (uint32_t)(bk >> (40 - kB6Log));
                        b6tag = (uint32_t)bk;
                        const u32x4 A = s_b6[2 * b6idx], B = s_b6[2 * b6idx + 1];
                        if ((A[0] ^ kB6C0) == b6tag && (A[2] ^ kB6C1) == b6tag && (B[0] ^ kB6C2) == b6tag &&
                            (B[2] ^ kB6C3) == b6tag) {
                            need6 = false;  // the group's one record r0 = {A[1], A[3], B[1], B[3]}
                            if (infw_rec_match(B[1], (uint64_t)A[3] << 32 | A[1], B[3], infw_bswap32(sw[1]),
                                               infw_be64(sw[2], sw[3])))
                                lng = B[3] & 0x1FFFFFFu;
                        }
                    }
                    // /16 words (kD16): an IPv4 lane the LDS cache did not answer reads its /16 word in this round
                    // instead of the tbl24 word, and the tbl24 word only when the /16 word does not answer
                    const bool needd = kD16 && need24 && !d16known;
                    uint64_t wd = 0;
                    if (needd) {
                        need24 = false;
                        wd = T.d16[((uint64_t)slot << 16) | (a32 >> 16)];
                    }
                    if (need24) w24 = T.tbl24[((uint64_t)slot << 24) | (a32 >> 8)];
                    if (need6) {
                        bi = bhash & T.bmask;
                        const u32x4 *b = reinterpret_cast<const u32x4 *>(T.btab + bi);
                        bh = b[0];
                        br0 = b[1];
                    }
                    if (needd) {
                        if (kCache && slot < 256) d16c_put(s_c24, d16i, key16, wd);
                        if (wd & INFW_D16_INLINE) {
                            sh = infw_d16_value(wd, a32 & 0xFFFFu);
                        } else {
                            need24 = true;
                            w24 = T.tbl24[((uint64_t)slot << 24) | (a32 >> 8)];
                        }
                    }
                    if (need6) {
                        lng = v6_finish<kLean>(T, (uint32_t)slot, a32, sw, bi, bh, br0);
                        if (b6ok && bh[0] == (uint32_t)slot + 1 && bh[1] == a32 && bh[2] == 1u) {
                            s_b6[2 * b6idx] = u32x4{b6tag ^ kB6C0, br0[0], b6tag ^ kB6C1, br0[1]};
                            s_b6[2 * b6idx + 1] = u32x4{b6tag ^ kB6C2, br0[2], b6tag ^ kB6C3, br0[3]};
                        }
                    }
                    if (need24) {
                        sh = d24_value(T, w24, a32);
                        if (!kD16 && kCache && slot < 256 && !(w24 & INFW_D24_GROUP))
                            s_c24[cidx] = 1ull << 63 | (unsigned long long)key << 31 | (uint32_t)w24;
                    } else if (!v6 && !d24) {  // compressed / no short table
                        sh = kLean ? 0u : infw_short_lookup(T, (uint32_t)slot, a32);
                    }
                    if (v6 && !lng) sh = short_lookup_cached<kCache, kC24Log, kLean, kD16>(T, (uint32_t)slot, a32, s_c24);
                    l1 = lng ? lng : sh;
                }
                // an ifindex without entries of its own: prefixes shorter than the ifindex (prefixLen < 32)
                if (!kLean && slot < 0 && T.n_wild) l1 = infw_wild_match(T.wild, T.n_wild, ifx);
            }
            if (G == 0) lst = l1;
            else if (l1) d = T.desc[(uint64_t)(l1 - 1) * INFW_DESC_STRIDE + cls];
        }
        const uint32_t off = (uint32_t)d, cnt = (uint32_t)(d >> 32);
        if (kSplit) {  // phase 1 of the two-phase form: the packet's decision-line address instead of the decision
            if (valid) {
                uint64_t w = pk == INFW_PK_DROP_SHORT ? 1u : 0u;
                if (lst) {
                    uint32_t p = T.dt_plog2;
                    if (kPl) p = infw_dt_parts_of(s_pl[(lst - 1) & (INFW_DT_PL_LISTS - 1)], lst - 1, INFW_DT_PL_LISTS, cls, p);
                    else if (T.n_dt_pl && lst - 1 < T.n_dt_pl) p = (T.dt_pl[lst - 1] >> (3 * cls)) & 7u;
                    w = split_word(infw_dt_slot_p(lst - 1, cls, val, T.dt_plog2, p), val, plen);
                }
                __builtin_nontemporal_store(w, &in.mid[i]);
            }
            continue;  // no counters, results or verdicts in phase 1 (uniform over the workgroup: no barrier skipped)
        }

        uint32_t result = 0;
        if (G == 0 && lst) {
            // the (list, class)'s own part count when the epoch has them (infw_tables.h), else the uniform one
            uint32_t p = T.dt_plog2;
            if (kPl) p = infw_dt_parts_of(s_pl[(lst - 1) & (INFW_DT_PL_LISTS - 1)], lst - 1, INFW_DT_PL_LISTS, cls, p);
            else if (T.n_dt_pl && lst - 1 < T.n_dt_pl) p = (T.dt_pl[lst - 1] >> (3 * cls)) & 7u;
            result = dt_lookup<kHalf>(T.dte, T.dtl, lst - 1, cls, val, T.dt_plog2, p);
        }
        // ---- first match, one lane per rule, G packets in flight
        uint64_t pending = G == 0 ? 0 : __ballot(cnt != 0);
        while (G > 0 && pending) {
            constexpr int GG = G > 0 ? G : 1;
            int j[GG];
            uint32_t o[GG], c[GG], v[GG];
            uint64_t rec[GG];
#pragma unroll
            for (int g = 0; g < GG; g++) {
                if (pending) {
                    j[g] = __builtin_ctzll(pending);
                    pending &= pending - 1;
                    o[g] = readlane(off, j[g]);
                    c[g] = readlane(cnt, j[g]);
                    v[g] = readlane(val, j[g]);
                } else {
                    j[g] = -1;
                    o[g] = c[g] = v[g] = 0;
                }
            }
#pragma unroll
            for (int g = 0; g < GG; g++) rec[g] = (uint32_t)lane < c[g] ? rules[(uint64_t)o[g] + lane] : 0;
#pragma unroll
            for (int g = 0; g < GG; g++) {
                if (j[g] < 0) break;
                const uint64_t mb = __ballot((uint32_t)lane < c[g] && rec_match(rec[g], v[g]));
                uint32_t r;
                if (mb) r = readlane((uint32_t)(rec[g] >> 32), __builtin_ctzll(mb));
                else r = c[g] > 64 ? scan_tail(rules, o[g], c[g], v[g], 64, lane) : 0;
                if (lane == j[g]) result = r;
            }
        }

        // ---- verdict (kernel.c:444-456) and statistics (kernel.c:376-387)
        const uint32_t action = result & 0xFFu;
        const uint32_t key = (result >> 8) & 0xFFFFu;
        {
            // counter slot of this packet, or -1 (no stats: UNDEF, action outside {1,2}, key >= 1024)
            const int s0_ = (valid && (action == INFW_XDP_DROP || action == INFW_XDP_PASS) && key < kStatKeys)
                                ? (int)key * 2 + (action == INFW_XDP_DROP) : -1;
            // a frame of kBigLen bytes or more (never a real frame), or a rule id without an LDS counter, goes
            // straight to the device counters
            const bool lds = plen < kBigLen && key < (uint32_t)kLdsStatKeys;
            if (s0_ >= 0 && !lds) {
                unsigned long long *dst = stats + (s0_ >> 1) * 4 + (s0_ & 1) * 2;
                atomicAdd(dst, 1ull);
                atomicAdd(dst + 1, (unsigned long long)plen);
            }
            const int s = lds ? s0_ : -1;
            // per-wavefront aggregation of the most common slot (Zipf traffic: the first eligible
            // lane's slot): its lanes are summed in registers and added once; the rest go to LDS
            const uint64_t elig = __ballot(s >= 0);
            if (elig) {
                const int lead = __builtin_ctzll(elig);
                const int s0 = __builtin_amdgcn_readlane(s, lead);
                const bool mine = s == s0;
                const uint64_t grp = __ballot(mine);
                // the group's byte count: one 32-bit DPP reduction (64 frames shorter than 2^20 B sum below 2^26)
                const uint32_t by = wave_sum(mine ? plen : 0u);
                if (lane == lead) atomicAdd(&s_c[s0], (unsigned long long)__popcll(grp) << 40 | by);
                if (s >= 0 && !mine) atomicAdd(&s_c[s], 1ull << 40 | plen);
            }
        }
        if (kEvents) {  // deny events (kernel.c:392-399): one atomic per wave, lanes keep their order
            const bool deny = valid && action == INFW_XDP_DROP;
            const uint64_t m = __ballot(deny);
            if (m) {
                unsigned long long base = 0;
                if (lane == __builtin_ctzll(m)) base = atomicAdd(ev.count, (unsigned long long)__popcll(m));
                base = ((unsigned long long)readlane((uint32_t)(base >> 32), __builtin_ctzll(m)) << 32) |
                       readlane((uint32_t)base, __builtin_ctzll(m));
                const uint64_t slot = base + __popcll(m & ((1ull << lane) - 1));
                if (deny && slot < ev.cap) {
                    uint64_t *r = reinterpret_cast<uint64_t *>(ev.rec + slot);
                    // event_hdr_st {ifId, ruleId, action, pad, pktLength}: u16 truncations (kernel.c:370-373)
                    r[0] = (uint64_t)(ifx & 0xFFFFu) | (uint64_t)key << 16 | (uint64_t)INFW_XDP_DROP << 32 |
                           (uint64_t)(plen & 0xFFFFu) << 48;
                    r[1] = (uint64_t)(plen < INFW_MAX_EVENT_DATA ? plen : INFW_MAX_EVENT_DATA);
                    r[2] = i;
                }
            }
        }
        if (valid) {
            if (results) {
                __builtin_nontemporal_store(result, &results[i]);
            }
            if (verdicts)
                verdicts[i] = (pk == INFW_PK_DROP_SHORT || action == INFW_XDP_DROP) ? INFW_XDP_DROP : INFW_XDP_PASS;

        }
        // every workgroup runs the same number of tiles, so the barrier is uniform
        if (++tiles_since_flush == T.stat_flush_tiles) {
            __syncthreads();
            flush_counters();
            __syncthreads();
            tiles_since_flush = 0;
        }
    }

    __syncthreads();
    flush_counters();
}

// ---- the registry of instantiations and the selector ------------------------------------------------------------
// Every classify_kernel instantiation the library launches is one entry of kVariants; select() maps a launch (the
// epoch's kind, the batch form, the launch shape, the sidebands) onto exactly one key, and a key without an entry
// is an error, not a fallback.  tests/test_variants*.py enumerate the registry through the C ABI
// (infw_kernel_variant_name), reach each entry with a table and launch shape built for it and compare it with the
// oracle.
struct VKey {
    uint8_t in;      // INFW_INPUT_*
    uint16_t block;
    uint8_t waves, group, log, b6log;
    bool ev, dbg, lean, pl, d16, split, half;
    bool operator==(const VKey &o) const {
        return in == o.in && block == o.block && waves == o.waves && group == o.group && log == o.log &&
               b6log == o.b6log && ev == o.ev && dbg == o.dbg && lean == o.lean && pl == o.pl && d16 == o.d16 &&
               split == o.split && half == o.half;
    }
};

using RunFn = void (*)(uint32_t grid, const infw_dev_tables &T, const BatchIn &in, uint64_t n, uint32_t *results,
                       uint8_t *verdicts, unsigned long long *st, hipStream_t stream, const Sideband &sb);

template <int kBlock, int G, int kWaves, int kIn, int kLog, int kB6, bool kEv, bool kDbg, bool kLean, bool kPl,
          bool kD16, bool kSplit, bool kHalf>
void run(uint32_t grid, const infw_dev_tables &T, const BatchIn &in, uint64_t n, uint32_t *results, uint8_t *verdicts,
         unsigned long long *st, hipStream_t stream, const Sideband &sb) {
    hipLaunchKernelGGL((classify_kernel<kBlock, G, kWaves, kIn, kLog, kB6, kEv, kDbg, kLean, kPl, kD16, kSplit, kHalf>),
                       dim3(grid), dim3(kBlock), 0, stream, T, in, n, results, verdicts, st, sb);
}

struct Variant {
    VKey key;
    RunFn fn;
};
template <int kBlock, int G, int kWaves, int kIn, int kLog, int kB6, bool kEv, bool kDbg, bool kLean, bool kPl,
          bool kD16, bool kSplit, bool kHalf>
constexpr Variant V() {
    return Variant{VKey{(uint8_t)kIn, (uint16_t)kBlock, (uint8_t)kWaves, (uint8_t)G, (uint8_t)kLog, (uint8_t)kB6, kEv,
                        kDbg, kLean, kPl, kD16, kSplit, kHalf},
                   &run<kBlock, G, kWaves, kIn, kLog, kB6, kEv, kDbg, kLean, kPl, kD16, kSplit, kHalf>};
}
constexpr bool F = false, T_ = true;
constexpr int S = INFW_INPUT_SOA, C = INFW_INPUT_COMPACT, R = INFW_INPUT_FRAMES, X = INFW_INPUT_XDP;

// LDS per workgroup of the 768-thread shapes: the word cache (8 B x 2^log) and the IPv6 group cache (32 B x 2^b6)
// take what the counters (2 KiB), the ifindex map (2 KiB), the per-list part counts (16 KiB, pl) and the frame
// windows (frames) leave of 80 KiB (two workgroups per CU).  Measured choices: 4096 words + 512 groups at configs[2]
// (profiles/r03zc), 8192 /16 words + 256 groups for /16-word epochs without part counts (profiles/r04g).
static const Variant kVariants[] = {
    //   block G  W  in log b6  ev dbg lean pl  d16 split half
    // the default shape, 768 x 2 (24 waves per CU), per epoch kind
    V<768, 0, 6, S, 12, 9, F, F, F, F, F, F, F>(),
    V<768, 0, 6, S, 12, 9, F, F, T_, F, F, F, F>(),
    V<768, 0, 6, S, 12, 9, F, F, T_, T_, F, F, F>(),
    V<768, 0, 6, S, 12, 9, F, F, T_, T_, T_, F, F>(),
    V<768, 0, 6, S, 13, 8, F, F, T_, F, T_, F, F>(),
    V<768, 0, 6, S, 13, 8, F, F, T_, F, T_, F, T_>(),
    // phase 1 of the two-phase form (lean epochs with many distinct rule lists; phase 2 is decide_kernel)
    V<768, 0, 6, S, 12, 9, F, F, T_, F, F, T_, F>(),
    V<768, 0, 6, S, 12, 9, F, F, T_, T_, F, T_, F>(),
    V<768, 0, 6, S, 12, 9, F, F, T_, F, T_, T_, F>(),
    V<768, 0, 6, S, 11, 9, F, F, T_, T_, T_, T_, F>(),
    // the other decision-table shapes infw_set_launch accepts: any epoch
    V<512, 0, 4, S, 11, 0, F, F, F, F, F, F, F>(),
    V<512, 0, 6, S, 11, 8, F, F, F, F, F, F, F>(),
    V<512, 0, 8, S, 10, 0, F, F, F, F, F, F, F>(),
    V<256, 0, 6, S, 10, 0, F, F, F, F, F, F, F>(),
    // the one-lane-per-rule ballot scan (kernel.c:222-258 in rule order), G packets in flight
    V<512, 1, 8, S, 10, 0, F, F, F, F, F, F, F>(),
    V<512, 4, 8, S, 10, 0, F, F, F, F, F, F, F>(),
    V<512, 8, 8, S, 10, 0, F, F, F, F, F, F, F>(),
    V<256, 1, 6, S, 10, 0, F, F, F, F, F, F, F>(),
    V<256, 4, 6, S, 10, 0, F, F, F, F, F, F, F>(),
    V<256, 8, 6, S, 10, 0, F, F, F, F, F, F, F>(),
    // sidebands (deny events, debug lookup capture): 512 x 3 with them compiled in
    V<512, 0, 6, S, 10, 0, T_, F, F, F, F, F, F>(),
    V<512, 0, 6, S, 10, 0, F, T_, F, F, F, F, F>(),
    V<512, 0, 6, S, 10, 0, T_, T_, F, F, F, F, F>(),
    // the family-compact layout: the default shape per epoch kind, 512 x 3 for every other shape, debug capture
    V<768, 0, 6, C, 12, 9, F, F, F, F, F, F, F>(),
    V<768, 0, 6, C, 12, 9, F, F, T_, F, F, F, F>(),
    V<768, 0, 6, C, 12, 9, F, F, T_, T_, F, F, F>(),
    V<768, 0, 6, C, 12, 9, F, F, T_, T_, T_, F, F>(),
    V<768, 0, 6, C, 13, 8, F, F, T_, F, T_, F, F>(),
    V<768, 0, 6, C, 13, 8, F, F, T_, F, T_, F, T_>(),
    V<512, 0, 6, C, 11, 0, F, F, F, F, F, F, F>(),
    V<512, 0, 6, C, 10, 0, F, T_, F, F, F, F, F>(),
    // raw frames: 768 x 2, the word cache halved for the frame windows (and again beside the part counts)
    V<768, 0, 6, R, 11, 9, F, F, F, F, F, F, F>(),
    V<768, 0, 6, R, 10, 9, F, F, F, T_, F, F, F>(),
    V<768, 0, 6, R, 11, 9, F, F, T_, F, F, F, F>(),
    V<768, 0, 6, R, 10, 9, F, F, T_, T_, F, F, F>(),
    V<768, 0, 6, R, 11, 9, F, F, T_, F, T_, F, F>(),
    V<768, 0, 6, R, 10, 9, F, F, T_, T_, T_, F, F>(),
    V<512, 0, 6, R, 10, 0, T_, F, F, F, F, F, F>(),
    V<512, 0, 6, R, 10, 0, F, T_, F, F, F, F, F>(),
    V<512, 0, 6, R, 10, 0, T_, T_, F, F, F, F, F>(),
    // AF_XDP descriptors over a umem: as raw frames (no event stream: infw_classify_xdp has none)
    V<768, 0, 6, X, 11, 9, F, F, F, F, F, F, F>(),
    V<768, 0, 6, X, 10, 9, F, F, F, T_, F, F, F>(),
    V<768, 0, 6, X, 11, 9, F, F, T_, F, F, F, F>(),
    V<768, 0, 6, X, 10, 9, F, F, T_, T_, F, F, F>(),
    V<768, 0, 6, X, 11, 9, F, F, T_, F, T_, F, F>(),
    V<768, 0, 6, X, 10, 9, F, F, T_, T_, T_, F, F>(),
    V<512, 0, 6, X, 10, 0, F, T_, F, F, F, F, F>(),
};
constexpr int kNumVariants = (int)(sizeof(kVariants) / sizeof(kVariants[0]));
constexpr int kDecideBlock = 512, kDecideBpc = 2;  // decide_kernel: 2 x 512 per CU (profiles/r04e: 40.3 vs 39.1 Gpps at 4)

void variant_name(const VKey &k, char *buf, size_t cap) {
    static const char *const in[] = {"soa", "compact", "frames", "xdp"};
    snprintf(buf, cap, "%s.%u.w%u.g%u.c%u.b%u%s%s%s%s%s%s%s", in[k.in], k.block, k.waves, k.group, k.log, k.b6log,
             k.lean ? ".lean" : "", k.pl ? ".pl" : "", k.d16 ? ".d16" : "", k.half ? ".half" : "",
             k.split ? ".split" : "", k.ev ? ".ev" : "", k.dbg ? ".dbg" : "");
}

const Variant *find_variant(const VKey &k) {
    for (const Variant &v : kVariants)
        if (v.key == k) return &v;
    return nullptr;
}

bool dflt_shape(const infw_launch_args &a) { return a.block == 768 && a.blocks_per_cu == 2 && a.group == 0; }
bool has_sidebands(const infw_launch_args &a) { return a.ev_count != nullptr || a.dbg_fp != nullptr; }

// The one selector.  allow_split = false gives the fused kernel of a two-phase epoch (its scratch could not be had).
VKey select_variant(const infw_launch_args &a, bool allow_split, uint32_t *bpc) {
    const infw_dev_tables &T = *a.T;
    const bool lean = T.lean != 0, pl = T.n_dt_pl == INFW_DT_PL_LISTS, d16 = T.d16_on != 0;
    VKey k{};
    k.in = (uint8_t)a.input;
    if (has_sidebands(a)) {  // 512 x 3 with the sidebands compiled in
        k.block = 512, k.waves = 6, k.log = 10;
        k.ev = a.ev_count != nullptr, k.dbg = a.dbg_fp != nullptr;
        *bpc = 3;
        return k;
    }
    if (a.input == INFW_INPUT_FRAMES || a.input == INFW_INPUT_XDP) {  // any shape: 768 x 2
        k.block = 768, k.waves = 6, k.b6log = 9, k.log = pl ? 10 : 11;
        k.lean = lean, k.pl = pl, k.d16 = lean && d16;
        *bpc = 2;
        return k;
    }
    if (dflt_shape(a)) {
        k.block = 768, k.waves = 6, k.b6log = 9, k.log = 12;
        *bpc = 2;
        if (!lean) return k;
        k.lean = true;
        if (a.input == INFW_INPUT_SOA && T.split && allow_split) {
            k.split = true, k.pl = pl, k.d16 = d16;
            if (pl && d16) k.log = 11;
            return k;
        }
        if (d16 && !pl) {  // /16 words without part counts: 8192 /16 words, 256 IPv6 groups
            k.d16 = true, k.half = T.dt_half != 0, k.log = 13, k.b6log = 8;
            return k;
        }
        k.pl = pl, k.d16 = d16 && pl;
        return k;
    }
    if (a.input == INFW_INPUT_COMPACT) {  // every other shape: 512 x 3
        k.block = 512, k.waves = 6, k.log = 11;
        *bpc = 3;
        return k;
    }
    *bpc = (uint32_t)a.blocks_per_cu;
    k.block = (uint16_t)a.block, k.group = (uint8_t)a.group;
    if (a.group) {
        k.waves = a.block == 512 ? 8 : 6, k.log = 10;
        return k;
    }
    if (a.block == 256) k.waves = 6, k.log = 10;
    else if (a.blocks_per_cu == 2) k.waves = 4, k.log = 11;
    else if (a.blocks_per_cu == 3) k.waves = 6, k.log = 11, k.b6log = 8;
    else k.waves = 8, k.log = 10;
    return k;
}

BatchIn batch_of(const infw_launch_args &a) {
    BatchIn bi{};
    if (a.input == INFW_INPUT_COMPACT) {
        const infw_batch_soa_c *c = a.compact;
        bi.saddr4 = c->saddr4, bi.v6tail = c->v6tail, bi.ifindex = c->ifindex, bi.pkt_len = c->pkt_len;
        bi.meta = c->meta, bi.l4word = c->l4word;
    } else if (a.input == INFW_INPUT_XDP) {
        bi.frames = a.umem;
        bi.xdp = reinterpret_cast<const u32x4 *>(a.xdp);
        bi.xdp_ifindex = a.xdp_ifindex;
    } else if (a.input == INFW_INPUT_FRAMES) {
        const infw_frame_batch *f = a.frames;
        bi.ifindex = f->ifindex, bi.pkt_len = f->pkt_len, bi.frames = f->frames, bi.offsets = f->offsets;
        bi.fstride = f->stride, bi.linear_len = f->linear_len;
    } else {
        const infw_batch_soa *s = a.soa;
        bi.saddr = s->saddr, bi.ifindex = s->ifindex, bi.pkt_len = s->pkt_len, bi.meta = s->meta, bi.l4word = s->l4word;
    }
    return bi;
}

uint32_t grid_of(uint64_t n, int block, uint32_t bpc, uint32_t cus) {
    const uint64_t tiles = (n + block - 1) / block, grid = (uint64_t)bpc * cus;
    return (uint32_t)(tiles < grid ? tiles : grid);
}

}  // namespace

extern "C" int infw_launch_shape_ok(int block, int group, int bpc) {
    if (group == 0)
        return (block == 768 && bpc == 2) || (block == 512 && bpc >= 2 && bpc <= 4) || (block == 256 && bpc == 6);
    return (group == 1 || group == 4 || group == 8) && ((block == 512 && bpc == 3) || (block == 256 && bpc == 6));
}

extern "C" int infw_launch_variant_count(void) { return kNumVariants + 1; }

extern "C" const char *infw_launch_variant_name(int i) {
    static char names[kNumVariants + 1][96];
    static const bool init = [] {
        for (int j = 0; j < kNumVariants; j++) variant_name(kVariants[j].key, names[j], sizeof names[j]);
        snprintf(names[kNumVariants], sizeof names[kNumVariants], "decide.%d", kDecideBlock);
        return true;
    }();
    (void)init;
    return i >= 0 && i <= kNumVariants ? names[i] : nullptr;
}

extern "C" int infw_launch_variant(const infw_launch_args *a, char *name, size_t cap) {
    uint32_t bpc = 0;
    const VKey k = select_variant(*a, true, &bpc);
    char buf[128];
    variant_name(k, buf, sizeof buf);
    if (!find_variant(k)) snprintf(buf + strlen(buf), sizeof buf - strlen(buf), "(unregistered)");
    else if (k.split) snprintf(buf + strlen(buf), sizeof buf - strlen(buf), "+decide.%d", kDecideBlock);
    if (strlen(buf) + 1 > cap) return -ERANGE;
    memcpy(name, buf, strlen(buf) + 1);
    return 0;
}

// The two-phase form (see decide_kernel): the per-packet words live in stream-ordered scratch from the context's
// own pool (abi.cpp; trimmed before a full commit uploads), so concurrent classify calls on other streams never share
// it and no other allocator of the process is affected.  Returns 0, -EIO on a launch error, or 1 when the scratch
// cannot be allocated (the caller then runs the fused kernel).
static int launch_split(const infw_launch_args &a, const Variant &p1, BatchIn bi, unsigned long long *st) {
    uint64_t *mid = nullptr;
    if (!a.pool || hipMallocFromPoolAsync(reinterpret_cast<void **>(&mid), a.n * sizeof(uint64_t), a.pool, a.stream) !=
                       hipSuccess) {
        (void)hipGetLastError();
        return 1;
    }
    bi.mid = mid;
    p1.fn(grid_of(a.n, p1.key.block, 2, a.cus), *a.T, bi, a.n, nullptr, nullptr, st, a.stream, Sideband{});
    hipLaunchKernelGGL(decide_kernel<kDecideBlock>, dim3(grid_of(a.n, kDecideBlock, kDecideBpc, a.cus)),
                       dim3(kDecideBlock), 0, a.stream, *a.T, (const uint64_t *)mid, bi.pkt_len, a.n, a.results,
                       a.verdicts, st);
    const bool ok = hipGetLastError() == hipSuccess;
    (void)hipFreeAsync(mid, a.stream);
    return ok ? 0 : -EIO;
}

extern "C" int infw_launch_classify(const infw_launch_args *a) {
    if (a->n == 0) return 0;
    const BatchIn bi = batch_of(*a);
    auto *st = reinterpret_cast<unsigned long long *>(a->stats);
    const Sideband sb{EventSink{a->ev, a->ev_cap, reinterpret_cast<unsigned long long *>(a->ev_count)},
                      DebugSink{reinterpret_cast<unsigned long long *>(a->dbg_fp), a->dbg_keys, a->dbg_count,
                                a->dbg_slots ? a->dbg_slots - 1 : 0u}};
    uint32_t bpc = 0;
    VKey k = select_variant(*a, true, &bpc);
    const Variant *v = find_variant(k);
    if (v && k.split) {
        const int rc = launch_split(*a, *v, bi, st);
        if (a->split_counts && rc >= 0) __atomic_fetch_add(&a->split_counts[rc == 0 ? 0 : 1], 1, __ATOMIC_RELAXED);
        if (rc <= 0) return rc;
        k = select_variant(*a, false, &bpc);  // no scratch: the fused kernel
        v = find_variant(k);
    }
    if (!v) return -EIO;  // a selector result without a registry entry (tests/test_variants_cpu.py rules it out)
    v->fn(grid_of(a->n, k.block, bpc, a->cus), *a->T, bi, a->n, a->results, a->verdicts, st, a->stream, sb);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
