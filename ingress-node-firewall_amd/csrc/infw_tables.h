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
//   short (<= /32)       DIR-24-8 per slot: tbl24[slot][2^24] u64 + tbl8 groups
//                        of 256 u32; value = list+1 (0 = no entry); a /24 with
//                        longer entries is held inline in its tbl24 word when
//                        it has <= 3 runs (almost always), else in a tbl8 group
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

// IPv6 long prefixes grouped by (slot, address bits 0..31): one 64-B bucket
// holds up to 3 records of the group sorted longest first, so the first match
// is the longest; a larger group sets n = INFW_BUCKET_OVERFLOW and is looked
// up in the Waldvogel table instead.
#define INFW_BUCKET_INLINE 3
#define INFW_BUCKET_OVERFLOW 0xFFu
struct infw_v6_rec {        // 16 B
    uint64_t lo;            // address bits 64..127 (masked)
    uint32_t mid;           // address bits 32..63 (masked)
    uint32_t meta;          // (length - 32) << 25 | list+1
};
struct infw_v6_bucket {     // 64 B
    uint32_t tag;           // slot + 1, 0 = empty
    uint32_t top;           // address bits 0..31
    uint32_t n;             // records, or INFW_BUCKET_OVERFLOW
    uint32_t pad;
    struct infw_v6_rec rec[INFW_BUCKET_INLINE];
};

// First-match decision tables.  For one (rule list, packet class) the
// first-match result as a function of the 16-bit packet value (dport, or
// type << 8 | code) is a step function with S <= 2c + 1 <= 201 segments.  The
// value axis is cut into 2^dt_plog2 equal parts (16 by default, 1 when the
// table would exceed its memory budget), and each part's piece of the step
// function is stored from one 64-B line (one L2 request), so that a packet
// touches one line after the LPM answer, two when its part holds more
// segments than a leaf:
//   entry line   dte[((list * INFW_NCLS + cls) << dt_plog2) | v >> (16 - dt_plog2)]
//                — addressed directly from the LPM answer and the value, no
//                descriptor load in between;
//   leaf form    (w[0] bit 31 clear; S <= 10): u16 keys in w[1..5] (key j =
//                start of segment j+1 minus 1, so "key < v" <=> "start <= v";
//                pad 0xFFFF never counts) and the results in w[6..15]; the
//                result is w[6 + #keys below v];
//   compact leaf (w[0] bit 30; S <= 20): used when every result of the step
//                function is 0 or SET_ACTIONRULE_RESPONSE(1|2, ruleId 1..127) —
//                everything makeIngressFwRulesMap writes (loader.go:429-515):
//                n = w[0] & 0xFF segments, u16 keys and one result code per
//                segment (bytes), half-first (infw_dt_ckey_word / _ccode_word):
//                keys 0..7 and codes 0..11 in the first 32 B, the rest in the
//                second, so the kernel reads the second half only for a value
//                past key 8 of a leaf of > 9 segments; code 0 = no match, else
//                ruleId = code >> 1 and action = 1 + (code & 1).  Twice the
//                segments of a u32 leaf, so half the leaf lines;
//   root form    (bit 31 set): 30 u16 group keys in w[1..15] select one of
//                <= 31 leaf lines dtl[(w[0] & 0x3FFFFFFF) + #keys below v], each
//                a leaf over 10 (u32) or 20 (compact) consecutive segments.
// No applicable rule is the all-pad leaf with result 0.
#define INFW_DT_LEAF_SEGS 10u
#define INFW_DT_CLEAF_SEGS 20u
#define INFW_DT_ROOT_KEYS 30u
#define INFW_DT_ROOT 0x80000000u
#define INFW_DT_COMPACT 0x40000000u
#define INFW_DT_INDEX 0x3FFFFFFFu
struct infw_dt_line {       // 64 B
    uint32_t w[16];
};

// Compressed short table (the <= /32 key space), per slot: l16[slot][2^16]
// words indexed by address bits 0..15; a word is list+1 (0 = none) or, with
// bit 31 set, the index of a 64-B node resolving the next 8 bits.  A node
// keeps a 256-bit run bitmap (bit i set: child i differs from child i-1; bit 0
// always set) and the run values, inline when there are at most 6, else in
// vpool[base ..].  Child i's value is run popcount(bm[0..i]) - 1; values have
// the same encoding (bits 24..31 via a second node level).
#define INFW_NODE_FLAG 0x80000000u
#define INFW_NODE_INLINE 6
struct infw_bnode {         // 64 B
    uint32_t bm[8];
    uint32_t nv;            // runs
    uint32_t base;          // vpool index when nv > INFW_NODE_INLINE
    uint32_t v[INFW_NODE_INLINE];
};

struct infw_dev_tables {
    const uint32_t *if_keys;
    const uint32_t *if_slot;   // INFW_IF_EMPTY = free
    uint32_t if_mask;
    uint32_t n_slots;
    uint32_t if_mult, if_shift;  // != 0: ifindex i sits at (i * if_mult) >> if_shift (no probing)
    const uint32_t *l16;       // n_slots << 16
    const struct infw_bnode *nodes;
    const uint32_t *vpool;
    const uint64_t *tbl24;     // DIR-24-8 form: n_slots << 24 words (INFW_D24_*) + tbl8 groups
    const uint32_t *tbl8;
    uint32_t short_mode;       // INFW_SHORT_DIR24 or INFW_SHORT_COMPRESSED
    const struct infw_long_entry *ltab;
    uint64_t lmask;
    const struct infw_v6_bucket *btab;
    uint64_t bmask;
    const uint64_t *desc;      // ballot mode: off | cnt << 32 into rules
    const uint64_t *rules;
    const struct infw_dt_line *dte;  // decision mode: entry lines, n_lists * INFW_NCLS
    const struct infw_dt_line *dtl;  // decision mode: leaf lines
    const uint8_t *levels;     // n_levels distinct long lengths, ascending
    uint32_t n_levels;
    uint32_t dt_plog2;         // decision-table parts per (list, class): 1 << dt_plog2 (0 or 4)
    const uint32_t *wild;      // entries with prefixLen < 32 (a partial ifindex): {plen, key bits, list+1} x n_wild,
    uint32_t n_wild;           // longest first; consulted for ifindexes without a slot (their own entries)
    uint32_t lean;             // 1: no compressed short table, no overflowed IPv6 group, no partial-ifindex prefix —
                               // the kernel may launch without those code paths (fewer live registers)
    const uint32_t *dt_pl;     // n_dt_pl != 0: per-list part counts, 3 bits per class (see infw_dt_slot_p)
    uint32_t n_dt_pl;
    uint32_t stat_flush_tiles;  // classify: a workgroup flushes its LDS counters every this many tiles (<= 1024)
    const uint64_t *d16;       // d16_on: n_slots << 16 words in front of DIR-24-8 (INFW_D16_*)
    uint32_t d16_on;
    uint32_t dt_half;          // read decision lines half-first (the second 32 B only where needed; choose_dt_half)
    uint32_t split;            // classify in two phases (LPM -> per-packet decision-line address; then the decision
                               // lines as independent gathers): epochs whose entry lines span GiBs (classify.hip)
    uint64_t n_dte;            // entry lines (host-side: the split decision)
};

INFW_TD uint32_t infw_bswap32(uint32_t x) {
    return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}
INFW_TD uint64_t infw_be64(uint32_t w0, uint32_t w1) {  // bytes w0[0..3] w1[0..3] as a BE u64
    return (uint64_t)infw_bswap32(w0) << 32 | infw_bswap32(w1);
}

INFW_TD uint32_t infw_if_hash(uint32_t ifindex) { return ifindex * 0x9E3779B1u; }

INFW_TD uint64_t infw_bucket_hash(uint32_t slot, uint32_t top) {
    uint64_t h = ((uint64_t)slot << 32 | top) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    return h ^ (h >> 30);
}

// Key of an IPv6 /32 group in the kernel's per-workgroup LDS group cache (slot < 256): a bijection of
// the 40-bit (slot, top) onto itself.  The entry index is its top bits and every 8-B word of the entry
// carries its low 32 bits, so (index, word tag) names exactly one group: a word is accepted only when
// it was written for the reader's own group, whatever the interleaving of writers and readers.
INFW_TD uint64_t infw_b6_key(uint32_t slot, uint32_t top) {
    const uint64_t M = (1ull << 40) - 1;
    uint64_t k = ((uint64_t)slot << 32 | top) & M;
    k = (k * 0x9E3779B97Full) & M;  // odd multiplier: invertible mod 2^40
    k ^= k >> 20;                   // xorshift by half the width: invertible
    k = (k * 0xC2B2AE3D27ull) & M;
    return k ^ (k >> 23);
}

// Does record r cover address bits 32..127 (mid, lo)?
INFW_TD bool infw_rec_match(uint32_t rmid, uint64_t rlo, uint32_t meta, uint32_t mid, uint64_t lo) {
    const uint32_t L = (meta >> 25) + 32;  // 33..128
    if (L <= 64) {
        const uint32_t m = ~0u << (64 - L);  // L-32 in 1..32 leading bits of mid
        return ((mid ^ rmid) & m) == 0;
    }
    const uint64_t m = L >= 128 ? ~0ull : ~0ull << (128 - L);
    return mid == rmid && ((lo ^ rlo) & m) == 0;
}

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

// Written as bitwise ops and selects, not a switch or short-circuit tests: on the GPU every lane of a wave
// then takes the same path (a switch over the protocol compiles into a tree of divergent branches and
// exec-mask bookkeeping, ~120 instructions per wave).  *cls and *val are set on every path; they mean
// something only when V4 / V6 is returned.
INFW_TD int infw_parse(uint32_t meta, uint32_t l4word, int *cls, uint32_t *val) {
    const uint32_t et = meta & 0xFFFFu, proto = (meta >> 16) & 0xFFu, cap = meta >> 24;
    const uint32_t v4 = et == 0x0800, v6 = et == 0x86DD;                 // kernel.c:428, :432
    const uint32_t tcp = proto == 6, udp = proto == 17, sctp = proto == 132, ic1 = proto == 1, ic58 = proto == 58;
    const uint32_t known = tcp | udp | sctp | ic1 | ic58;                // :117-172, else UNDEF
    // fixed L4 offset 34 / 54 (:104, :111) plus the header the protocol's case reads: tcphdr 20, sctphdr 12,
    // udphdr / icmphdr / icmp6hdr 8 — a truncated header is UNDEF
    const uint32_t need = (v4 ? 34u : 54u) + 8u + tcp * 12u + sctp * 4u;
    // class: TCP 0, UDP 1, SCTP 2, proto 1 -> ICMP4 (3) on IPv4 / 1_ON_V6 (6), proto 58 -> 58_ON_V4 (5) / ICMP6 (4)
    const uint32_t c = udp * (uint32_t)INFW_CLS_UDP + sctp * (uint32_t)INFW_CLS_SCTP +
                       ic1 * (v4 ? (uint32_t)INFW_CLS_ICMP4 : (uint32_t)INFW_CLS_1_ON_V6) +
                       ic58 * (v4 ? (uint32_t)INFW_CLS_58_ON_V4 : (uint32_t)INFW_CLS_ICMP6);
    const uint32_t port = (l4word >> 8 & 0xFF00u) | (l4word >> 24);         // ntohs(dest)
    const uint32_t tc = (l4word << 8 & 0xFF00u) | (l4word >> 8 & 0xFFu);    // type << 8 | code
    *val = c <= (uint32_t)INFW_CLS_SCTP ? port : tc;
    *cls = (int)c;
    int pk = v4 ? INFW_PK_V4 : INFW_PK_V6;
    pk = (known & (uint32_t)(cap >= need)) ? pk : INFW_PK_UNDEF;
    pk = (v4 | v6) ? pk : INFW_PK_PASS_NONIP;                           // :436-438
    return cap < 14 ? INFW_PK_DROP_SHORT : pk;                          // :423-426
}

INFW_TD uint32_t infw_count_lt(uint32_t w, uint32_t v) {  // keys (two u16) below v
    return (uint32_t)((w & 0xFFFFu) < v) + (uint32_t)((w >> 16) < v);
}

// Keys (u16 halves of words w[a..b)) below v.
INFW_TD uint32_t infw_keys_below(const uint32_t *w, int a, int b, uint32_t v) {
    uint32_t c = 0;
    for (int k = a; k < b; k++) c += infw_count_lt(w[k], v);
    return c;
}

// Entry line of (list, cls) for value v.
INFW_TD uint64_t infw_dt_slot(uint32_t list, int cls, uint32_t v, uint32_t plog2) {
    return (((uint64_t)list * INFW_NCLS + (uint32_t)cls) << plog2) | (v >> (16u - plog2));
}
// Per-(list, class) part counts (n_dt_pl != 0, at most INFW_DT_PL_LISTS lists): (list, cls) keeps its region of
// 2^dt_plog2 entry lines but is cut into only 2^p parts, the fewest whose every part fits one line (p <=
// dt_plog2), so a packet's value lands on one of 2^p lines of the region, not 2^dt_plog2: fewer distinct lines
// per hot (list, class).  The list's word holds p in bits [3 cls, 3 cls + 3).  Lists appended by incremental
// commits past the table (id >= n_dt_pl) keep the uniform 2^dt_plog2 parts.
#define INFW_DT_PL_LISTS 4096u
INFW_TD uint32_t infw_dt_parts_of(uint32_t word, uint32_t list, uint32_t n_dt_pl, int cls, uint32_t plog2) {
    return list < n_dt_pl ? (word >> (3 * cls)) & 7u : plog2;
}
INFW_TD uint64_t infw_dt_slot_p(uint32_t list, int cls, uint32_t v, uint32_t plog2, uint32_t p) {
    return (((uint64_t)list * INFW_NCLS + (uint32_t)cls) << plog2) | (v >> (16u - p));
}

// Result word of a compact-leaf code (0 = no match).
INFW_TD uint32_t infw_dt_code_result(uint32_t code) {
    return code ? ((code >> 1) << 8 | (1u + (code & 1u))) : 0u;
}
// Compact-leaf code of a result word, or 0x100 when it has none.
INFW_TD uint32_t infw_dt_result_code(uint32_t r) {
    if (r == 0) return 0;
    const uint32_t a = r & 0xFFu, id = r >> 8;
    return (a == 1u || a == 2u) && id >= 1u && id <= 127u ? (id << 1 | (a - 1u)) : 0x100u;
}

// Compact leaf (<= 20 segments, u8 result codes), half-first: w[0] = COMPACT | n; keys 0..7 in w[1..4], codes
// 0..11 in w[5..7] — the first 32 B, which answer every value below key 8 and, when n <= 9, every value; keys 8..19
// in w[8..13], codes 12..19 in w[14..15].  Key j (u16 half j & 1 of its word) = start of segment j + 1, minus 1
// (0xFFFF past the last segment).
INFW_TD uint32_t infw_dt_ckey_word(uint32_t j) { return j < 8 ? 1 + (j >> 1) : 8 + ((j - 8) >> 1); }
INFW_TD uint32_t infw_dt_ccode_word(uint32_t j) { return j < 12 ? 5 + (j >> 2) : 14 + ((j - 12) >> 2); }

// Result of a leaf line (u32 or compact form) for v.
INFW_TD uint32_t infw_dt_leaf(const uint32_t *w, uint32_t v) {
    if (w[0] & INFW_DT_COMPACT) {
        uint32_t c = infw_keys_below(w, 1, 5, v);  // 0..8
        if (c == 8 && (w[0] & 0xFFu) > 9) c += infw_keys_below(w, 8, 14, v);  // 8..19
        return infw_dt_code_result((w[infw_dt_ccode_word(c)] >> (8 * (c & 3u))) & 0xFFu);
    }
    const uint32_t c = infw_keys_below(w, 1, 6, v);
    uint32_t r = w[6];
    for (uint32_t k = 1; k < INFW_DT_LEAF_SEGS; k++) r = c >= k ? w[6 + k] : r;
    return r;
}

// First-match result of (list, cls) for value v (host walk; the kernel has its own loads).
template <class T>
INFW_TD uint32_t infw_dt_eval(const T &t, uint32_t list, int cls, uint32_t v) {
    const uint32_t p = list < t.n_dt_pl ? (t.dt_pl[list] >> (3 * cls)) & 7u : t.dt_plog2;
    const uint32_t *w = t.dte[infw_dt_slot_p(list, cls, v, t.dt_plog2, p)].w;
    if (w[0] & INFW_DT_ROOT) w = t.dtl[(w[0] & INFW_DT_INDEX) + infw_keys_below(w, 1, 16, v)].w;
    return infw_dt_leaf(w, v);
}

// Table pointers are read through T so host and device share the walk.
template <class T>
INFW_TD int infw_if_slot(const T &t, uint32_t ifindex) {
    if (t.if_mult) {
        const uint32_t h = (ifindex * t.if_mult) >> t.if_shift;
        return t.if_keys[h] == ifindex && t.if_slot[h] != INFW_IF_EMPTY ? (int)t.if_slot[h] : -1;
    }
    uint32_t h = infw_if_hash(ifindex) & t.if_mask;
    for (;;) {
        uint32_t s = t.if_slot[h];
        if (s == INFW_IF_EMPTY) return -1;
        if (t.if_keys[h] == ifindex) return (int)s;
        h = (h + 1) & t.if_mask;
    }
}

INFW_TD uint32_t infw_popc(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__popc(x);
#else
    return (uint32_t)__builtin_popcount(x);
#endif
}

// Value of child i (0..255) of node n.
template <class T>
INFW_TD uint32_t infw_node_child(const T &t, const struct infw_bnode &n, uint32_t i) {
    const uint32_t w = i >> 5, b = i & 31;
    uint32_t r = infw_popc(n.bm[w] & (0xFFFFFFFFu >> (31 - b)));
    for (uint32_t k = 0; k < 8; k++) r += k < w ? infw_popc(n.bm[k]) : 0u;
    r -= 1;  // bit 0 is always set, so r >= 0
    if (n.nv <= INFW_NODE_INLINE) {
        uint32_t v = n.v[0];
        for (uint32_t k = 1; k < INFW_NODE_INLINE; k++) v = r == k ? n.v[k] : v;
        return v;
    }
    return t.vpool[n.base + r];
}

// Short-table form: DIR-24-8 (one 4-B gather, 64 MiB per ifindex) unless that
// exceeds the memory budget, then the compressed 16-8-8 form (~16 B per prefix).
#define INFW_SHORT_DIR24 0u
#define INFW_SHORT_COMPRESSED 1u
#define INFW_SHORT_NONE 2u        // DIR-24-8 build without any <= /32 entry
// DIR-24-8 word (8 B).  Bits 63..62:
//   00  plain: list+1 of the whole /24 in bits 0..31;
//   10  tbl8 group index in bits 0..31 (256 u32 values, one per last byte);
//   11  inline /24, one 8-B word instead of a second, dependent L2 request into
//       a tbl8 group.  Bit 61 picks the form:
//       0  <= 3 runs, values <= 0x7FFF: v0 bits 0..14, v1 15..29, v2 30..44, run
//          starts b1 bits 45..52 and b2 53..60 (b1 <= b2): last byte x ->
//          x < b1 ? v0 : x < b2 ? v1 : v2;
//       1  two values A, B <= 0x3FFFFF laid out A | B | A (a longer prefix inside
//          or at either end of its covering /24 — the usual shape): A bits 0..21,
//          B 22..43, b1 44..51, b2 52..60 (9 bits, 256 = to the end): x in
//          [b1, b2) ? B : A.  Keeps such /24s inline when list ids exceed 15 bits
//          (configs[2] with 1M distinct rule lists).
#define INFW_D24_GROUP (1ull << 63)
#define INFW_D24_INLINE (1ull << 62)
#define INFW_D24_ABA (1ull << 61)
#define INFW_D24_MAXV 0x7FFFu
#define INFW_D24_ABA_MAXV 0x3FFFFFu

// Word for a /24 whose 256 values are g (tbl8 group gidx): inline when it can be.
INFW_TD uint64_t infw_d24_encode(const uint32_t *g, uint32_t gidx) {
    uint32_t v[3] = {g[0], 0, 0}, b[2] = {0, 0}, runs = 1;
    bool ok = true;
    for (uint32_t x = 1; x < 256 && ok; x++) {
        if (g[x] == g[x - 1]) continue;
        if (runs == 3) ok = false;
        else {
            b[runs - 1] = x;
            v[runs++] = g[x];
        }
    }
    if (!ok) return INFW_D24_GROUP | gidx;
    if (runs == 1) return g[0];
    if (runs == 2) {
        v[2] = v[1];
        b[1] = b[0];
    }
    if (v[0] <= INFW_D24_MAXV && v[1] <= INFW_D24_MAXV && v[2] <= INFW_D24_MAXV)
        return INFW_D24_GROUP | INFW_D24_INLINE | (uint64_t)b[1] << 53 | (uint64_t)b[0] << 45 | (uint64_t)v[2] << 30 |
               (uint64_t)v[1] << 15 | v[0];
    // A | B | A form: two runs (B to the end: b2 = 256), or three whose first and last values agree
    uint32_t A = v[0], B = v[1], b1 = b[0], b2 = runs == 2 ? 256u : b[1];
    if (runs == 3 && v[2] != v[0]) return INFW_D24_GROUP | gidx;
    if (A > INFW_D24_ABA_MAXV || B > INFW_D24_ABA_MAXV) return INFW_D24_GROUP | gidx;
    return INFW_D24_GROUP | INFW_D24_INLINE | INFW_D24_ABA | (uint64_t)b2 << 52 | (uint64_t)b1 << 44 | (uint64_t)B << 22 |
           A;
}

INFW_TD uint32_t infw_d24_inline(uint64_t e, uint32_t x) {
    // both forms decoded, the word's form bit selects (no branch)
    const uint32_t a1 = (uint32_t)(e >> 44) & 0xFFu, a2 = (uint32_t)(e >> 52) & 0x1FFu;
    const uint32_t aba = (uint32_t)(e >> (x >= a1 && x < a2 ? 22 : 0)) & INFW_D24_ABA_MAXV;
    const uint32_t b1 = (uint32_t)(e >> 45) & 0xFFu, b2 = (uint32_t)(e >> 53) & 0xFFu;
    const uint32_t sh = x >= b2 ? 30u : x >= b1 ? 15u : 0u;
    const uint32_t three = (uint32_t)(e >> sh) & INFW_D24_MAXV;
    return (e & INFW_D24_ABA) ? aba : three;
}

template <class T>
INFW_TD uint32_t infw_dir24_lookup(const T &t, uint32_t slot, uint32_t a32) {
    const uint64_t e = t.tbl24[((uint64_t)slot << 24) | (a32 >> 8)];
    if (!(e & INFW_D24_GROUP)) return (uint32_t)e;
    if (e & INFW_D24_INLINE) return infw_d24_inline(e, a32 & 0xFFu);
    return t.tbl8[((uint64_t)(uint32_t)e << 8) | (a32 & 0xFFu)];
}

// /16 words in front of DIR-24-8 (d16_on; chosen per full compile when most /16s that hold any prefix longer
// than /16 are of the shape below, e.g. sparse tables of /16../32 prefixes).  One 8-B word per (slot, address
// bits 0..15), 512 KiB per slot — small enough to stay in L2 — where DIR-24-8 spreads a /16../23 prefix over
// up to 256 words on 16 lines of its 128 MiB per slot.  Bit 63 set: the /16 holds at most three runs of the
// shape A | B | A, values <= 0x7FFF: A bits 0..14, B 15..29, b bits 30..45, e 46..61, and address bits 16..31 x
// -> x in [b, e] ? B : A.  Bit 63 clear: the /16 is read from its DIR-24-8 word (which stays complete, so a
// reader that ignores the /16 words is still exact).
#define INFW_D16_INLINE (1ull << 63)
INFW_TD uint32_t infw_d16_value(uint64_t w, uint32_t lo16) {
    const uint32_t b = (uint32_t)(w >> 30) & 0xFFFFu, e = (uint32_t)(w >> 46) & 0xFFFFu;
    return (uint32_t)(w >> (lo16 >= b && lo16 <= e ? 15 : 0)) & 0x7FFFu;
}
INFW_TD uint64_t infw_d16_encode(uint32_t A, uint32_t B, uint32_t b, uint32_t e) {
    return INFW_D16_INLINE | (uint64_t)e << 46 | (uint64_t)b << 30 | (uint64_t)B << 15 | A;
}
template <class T>
INFW_TD uint32_t infw_d16_lookup(const T &t, uint32_t slot, uint32_t a32) {
    const uint64_t w = t.d16[((uint64_t)slot << 16) | (a32 >> 16)];
    return (w & INFW_D16_INLINE) ? infw_d16_value(w, a32 & 0xFFFFu) : infw_dir24_lookup(t, slot, a32);
}

template <class T>
INFW_TD uint32_t infw_dir_lookup(const T &t, uint32_t slot, uint32_t a32) {
    uint32_t e = t.l16[((uint64_t)slot << 16) | (a32 >> 16)];
    if (e & INFW_NODE_FLAG) {
        e = infw_node_child(t, t.nodes[e & ~INFW_NODE_FLAG], (a32 >> 8) & 0xFFu);
        if (e & INFW_NODE_FLAG) e = infw_node_child(t, t.nodes[e & ~INFW_NODE_FLAG], a32 & 0xFFu);
    }
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

// Longest long (/33../128) prefix covering an IPv6 address: its /32 group's
// bucket, or the Waldvogel table when the group overflowed.  list+1 or 0.
template <class T>
INFW_TD uint32_t infw_v6_long(const T &t, uint32_t slot, uint32_t a32, const uint32_t sa[4]) {
    const uint32_t mid = infw_bswap32(sa[1]);
    const uint64_t lo = infw_be64(sa[2], sa[3]);
    uint64_t i = infw_bucket_hash(slot, a32) & t.bmask;
    for (;;) {
        const struct infw_v6_bucket *b = &t.btab[i];
        const uint32_t tag = b->tag;
        if (tag == 0) return 0;
        if (tag == slot + 1 && b->top == a32) {
            const uint32_t nb = b->n;
            if (nb == INFW_BUCKET_OVERFLOW) return infw_long_lookup(t, slot, (uint64_t)a32 << 32 | mid, lo);
            for (uint32_t k = 0; k < nb; k++) {
                const struct infw_v6_rec r = b->rec[k];
                if (infw_rec_match(r.mid, r.lo, r.meta, mid, lo)) return r.meta & 0x1FFFFFFu;
            }
            return 0;
        }
        i = (i + 1) & t.bmask;
    }
}

template <class T>
INFW_TD uint32_t infw_short_lookup(const T &t, uint32_t slot, uint32_t a32) {
    if (t.short_mode == INFW_SHORT_DIR24) return t.d16_on ? infw_d16_lookup(t, slot, a32) : infw_dir24_lookup(t, slot, a32);
    return t.short_mode == INFW_SHORT_COMPRESSED ? infw_dir_lookup(t, slot, a32) : 0u;
}

// Longest entry shorter than the ifindex (prefixLen < 32) covering this ifindex: its first plen key bits are
// the ifindex's little-endian bytes read most significant bit first.  list+1 or 0.
INFW_TD uint32_t infw_wild_match(const uint32_t *w, uint32_t n, uint32_t ifindex) {
    const uint32_t k = infw_bswap32(ifindex);
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t plen = w[3 * i], m = plen ? ~0u << (32 - plen) : 0u;
        if (((k ^ w[3 * i + 1]) & m) == 0) return w[3 * i + 2];
    }
    return 0;
}

// list+1 of the longest matching entry, 0 if none.
template <class T>
INFW_TD uint32_t infw_lpm(const T &t, int pk, uint32_t ifindex, const uint32_t sa[4]) {
    int slot = infw_if_slot(t, ifindex);
    if (slot < 0) return infw_wild_match(t.wild, t.n_wild, ifindex);
    uint32_t a32 = infw_bswap32(sa[0]);
    if (pk == INFW_PK_V6 && t.n_levels) {
        uint32_t r = infw_v6_long(t, (uint32_t)slot, a32, sa);
        if (r) return r;
    }
    return infw_short_lookup(t, (uint32_t)slot, a32);
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
