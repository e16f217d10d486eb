// cachesim.cpp — L2 behaviour of the classify kernel's table walk, on the host.
//
// Builds the configs[2] tables with the product's compiler, generates packets
// with the workload generator, walks each packet the way the kernel does and
// feeds every table line it touches into a model of the MI355X L2: 8 XCDs x
// 4 MiB, 16-way, 128-B lines, LRU; packet i runs on XCD (i / 512) % 8 (tiles of
// 512 packets striped over workgroups, workgroups round-robin over XCDs).
// Reports L2 requests / misses per packet per structure, for the compiled layout
// ("current"; INFW_DT_PARTS / INFW_DT_FORM select it) and for candidate layouts
// expressed as alternative address maps over the single-part layout
// (INFW_DT_PARTS=1):
//   tbl24_u16   DIR-24-8 words of 2 bytes (no inline /24s)
//   entry32     decision entries of 32 B, a list's classes packed in 128-B lines
//   quartersQ / partsQxB   entry lines addressed by (list, class, value part)
//   d16         an 8-B word per (slot, /16) in front of DIR-24-8 answering /16s of <= 3 runs (A | B | A) alone
// CACHESIM_CFG / CACHESIM_PREFIXES / CACHESIM_TEMPLATES pick the workload and its table size.
// Build + run: make cachesim   (tools/cachesim [n_packets])
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <unordered_map>
#include <vector>

#include "../ingress-node-firewall_amd/csrc/infw_internal.h"
#include "../ingress-node-firewall_amd/csrc/workload.h"

namespace infw {
void set_error(const std::string &s) { fprintf(stderr, "set_error: %s\n", s.c_str()); }
}  // namespace infw
using namespace infw;

namespace {

struct L2 {
    static constexpr int kWays = 16, kLine = 128;
    uint32_t sets;
    std::vector<uint64_t> tag;  // sets x ways, most recent first
    explicit L2(uint64_t bytes) : sets((uint32_t)(bytes / kLine / kWays)), tag((size_t)sets * kWays, ~0ull) {}
    bool access(uint64_t addr) {  // true = hit
        const uint64_t line = addr / kLine;
        const uint64_t h = line * 0x9E3779B97F4A7C15ull;
        uint64_t *t = &tag[(size_t)((h >> 32) % sets) * kWays];
        for (int w = 0; w < kWays; w++)
            if (t[w] == line) {
                for (int k = w; k > 0; k--) t[k] = t[k - 1];
                t[0] = line;
                return true;
            }
        for (int k = kWays - 1; k > 0; k--) t[k] = t[k - 1];
        t[0] = line;
        return false;
    }
};

enum Struct { S_BUCKET, S_TBL24, S_TBL8, S_ENTRY, S_LEAF, S_D16, S_N };
const char *kName[S_N] = {"bucket", "tbl24", "tbl8", "entry", "leaf", "d16"};

struct Touch {
    int s;
    uint64_t addr;
};

// Separate virtual address spaces per structure (1 TiB apart).
constexpr uint64_t kSpace = 1ull << 40;

struct Variant {
    const char *name;
    bool tbl24_u16, entry32;
    int quarters;  // > 0: decision lines addressed by (list, class, value >> (16 - log2 quarters))
    int slot_bytes = 64;  // bytes per (list, class, part) slot: a compact leaf of 20 / 10 / 5 segments
    int entry_stride = 64;
    int dense_short = 0;  // 1: short-table lookups touch one 8-B word per matched prefix, prefixes sorted by (slot, address)
    int cuckoo = 0;   // 1: IPv6 groups in the two-choice table above (absent groups touch both buckets)
    int mini = 0;     // > 0: 16-B mini entry per (list, class, part) holding <= mini segments; others add the 64-B line
    int pairing = 0;  // 1: compiled parts, entry line at ((list * 16 + part) * 8 + cls) * 64 (classes of one part adjacent)
    int adapt = 0;    // 1: per-(list, class) part count — the fewest of 1..16 parts of <= 20 segments each — inside
                      // the compiled 16-line region (lines past the count are never touched)
    int cls_p = 0;    // 1: one part count per class (the fewest with <= 1/256 of its lines over 20 segments)
    int lp = 0;       // > 0: IPv6 groups placed in sets of lp 32-B slots (one per record) at lp_load slot load, linear
    double lp_load = 0.8;  // probing over sets with a per-set overflow flag; a lookup reads its home set and walks
                      // on only through flagged sets
    int set4 = 0;     // 1: IPv6 groups in 128-B sets of four 32-B slots at 0.8 slot load (a group takes 1..3 slots
                      // of its home set; the lookup reads the home set's line)
    int d16 = 0;      // 1: an 8-B word per (slot, /16) in front of DIR-24-8 answers /16s of <= 3 runs (A | B | A, values
                      // <= 15 bits) by itself; other /16s read their tbl24 word after it
    int mphf = 0;     // > 0: IPv6 groups in a dense array of mphf-byte records at their rank under a minimal perfect
                      // hash (a random permutation of the groups); an absent group reads one record at a hashed rank
};

// Does (slot, /16 hi) have at most three runs of the A | B | A shape with values <= 0x7FFF?
bool d16_inline(const infw_dev_tables &t, uint32_t slot, uint32_t hi) {
    uint32_t vals[4], nr = 0, prev = ~0u;
    for (uint32_t x = 0; x < 256; x++) {
        const uint64_t e = t.tbl24[((uint64_t)slot << 24) | hi << 8 | x];
        uint32_t seg[3], ns = 0;
        if (!(e & INFW_D24_GROUP)) seg[ns++] = (uint32_t)e;
        else {
            uint32_t last = ~0u;
            for (uint32_t y = 0; y < 256; y++) {
                const uint32_t v = infw_dir24_lookup(t, slot, hi << 16 | x << 8 | y);
                if (v != last) {
                    if (ns == 3) return false;
                    seg[ns++] = last = v;
                }
            }
        }
        for (uint32_t k = 0; k < ns; k++) {
            if (seg[k] == prev) continue;
            if (nr == 3 || seg[k] > 0x7FFFu) return false;
            vals[nr++] = prev = seg[k];
        }
    }
    return nr < 3 || vals[0] == vals[2];
}

}  // namespace

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : (4u << 20);
    infw_wl *wl = nullptr;
    const int cfg = getenv("CACHESIM_CFG") ? atoi(getenv("CACHESIM_CFG")) : INFW_WL_CFG2_MIXED_1M;
    const uint32_t npfx = getenv("CACHESIM_PREFIXES") ? (uint32_t)atoi(getenv("CACHESIM_PREFIXES")) : 0;
    const uint32_t ntpl = getenv("CACHESIM_TEMPLATES") ? (uint32_t)atoi(getenv("CACHESIM_TEMPLATES")) : 0;
    if (infw_wl_create(&wl, cfg, 0x1F000000ull + cfg, npfx, ntpl)) return 1;
    if (getenv("CACHESIM_UNIFORM") && atoi(getenv("CACHESIM_UNIFORM"))) infw_wl_uniform_sources(wl);  // bench --uniform
    PendingMap m;
    m.max_entries = 1u << 22;
    const uint64_t ne = infw_wl_n_entries(wl);
    const lpm_ip_key_st *keys = infw_wl_keys(wl);
    const uint32_t *vi = infw_wl_val_index(wl);
    const rulesVal_st *tv = infw_wl_templates(wl);
    // CACHESIM_SHUFFLE=1: the keys in a seeded random order, as bench.py's default --key-order shuffled (the
    // reference loader's Go map range): the last update of every entry, shuffled — the same map, other list ids
    std::vector<uint64_t> order(ne);
    for (uint64_t i = 0; i < ne; i++) order[i] = i;
    if (getenv("CACHESIM_SHUFFLE") && atoi(getenv("CACHESIM_SHUFFLE"))) {
        std::unordered_map<std::string, uint64_t> last;
        for (uint64_t i = 0; i < ne; i++) {
            NodeKey k;
            k.plen = keys[i].prefixLen;
            uint8_t md[20];
            memcpy(md, &keys[i].ingress_ifindex, 4);
            memcpy(md + 4, keys[i].ip_data, 16);
            mask_bits(md, k.plen, k.md, 20);
            last[std::string(reinterpret_cast<const char *>(&k), sizeof k)] = i;
        }
        order.clear();
        for (const auto &kv : last) order.push_back(kv.second);
        std::sort(order.begin(), order.end());
        uint64_t rs = 0x5EED;
        for (uint64_t i = order.size(); i > 1; i--) {  // Fisher-Yates with a fixed-seed generator
            rs = rs * 6364136223846793005ull + 1442695040888963407ull;
            std::swap(order[i - 1], order[(rs >> 33) % i]);
        }
    }
    for (uint64_t i : order) m.update(&keys[i], reinterpret_cast<const uint8_t *>(&tv[vi[i]]), 0);
    HostTables h;
    if (compile_tables(m, h, Options())) return 2;
    const infw_dev_tables t = h.view();
    std::vector<uint32_t> tup(n * 8);
    infw_wl_tuples(wl, 0, n, tup.data(), 8);

    // per (list, class): the step function, for the quartered variants
    std::vector<std::vector<uint32_t>> seg_starts((size_t)h.n_lists * INFW_NCLS);
    for (uint32_t l = 0; l < h.n_lists; l++)
        for (int c = 0; c < INFW_NCLS; c++) {
            const uint64_t d = h.desc[(size_t)l * INFW_DESC_STRIDE + c];
            std::vector<uint64_t> recs(h.rules.begin() + (uint32_t)d, h.rules.begin() + (uint32_t)d + (d >> 32));
            std::vector<uint32_t> st, rs;
            step_function(recs, st, rs);
            seg_starts[(size_t)l * INFW_NCLS + c] = st;
        }
    // short-table prefixes (<= 32 address bits) ranked by (slot, address, length)
    std::unordered_map<uint64_t, uint64_t> short_rank;
    {
        std::vector<std::pair<uint64_t, uint64_t>> v;  // ((slot, net), L) -> key
        for (uint64_t i = 0; i < ne; i++) {
            const uint32_t L = keys[i].prefixLen - 32;
            if (L > 32) continue;
            const int sl = infw_if_slot(t, keys[i].ingress_ifindex);
            if (sl < 0) continue;
            uint32_t a = (uint32_t)keys[i].ip_data[0] << 24 | keys[i].ip_data[1] << 16 | keys[i].ip_data[2] << 8 | keys[i].ip_data[3];
            a = L ? a & (~0u << (32 - L)) : 0;
            v.push_back({((uint64_t)sl << 32 | a) << 6 | L, ((uint64_t)sl << 40) | ((uint64_t)L << 32) | a});
        }
        std::sort(v.begin(), v.end());
        for (uint64_t r = 0; r < v.size(); r++) short_rank[v[r].second] = r;
    }
    const Variant vars[] = {{"current", false, false, 0}, {"tbl24_u16", true, false, 0}, {"entry32", false, true, 0},
                            {"quarters4", false, false, 4}, {"quarters8", false, false, 8},
                            {"quarters16", false, false, 16}, {"parts16x32B", false, false, 16, 32},
                            {"parts32x32B", false, false, 32, 32}, {"parts32x16B", false, false, 32, 16},
                            {"parts64x16B", false, false, 64, 16}, {"parts8x32B", false, false, 8, 32},
                            {"stride128", false, false, 0, 64, 128}, {"cls_paired", false, false, 0, 64, 64, 0, 0, 1},
                            {"dense_short", false, false, 0, 64, 64, 1}, {"cuckoo", false, false, 0, 64, 64, 0, 1},
                            {"list_minor", false, false, 0, 64, 64, 0, 0, 0, 2},
                            {"mini4", false, false, 0, 64, 64, 0, 0, 4}, {"mini3", false, false, 0, 64, 64, 0, 0, 3},
                            {"adaptP", false, false, 0, 64, 64, 0, 0, 0, 0, 1},
                            {"clsP", false, false, 0, 64, 64, 0, 0, 0, 0, 0, 1},
                            {"d16", false, false, 0, 64, 64, 0, 0, 0, 0, 0, 0, 0, 0.8, 0, 1},
                            {"set4", false, false, 0, 64, 64, 0, 0, 0, 0, 0, 0, 0, 0.8, 1, 0},
                            {"set4_d16", false, false, 0, 64, 64, 0, 0, 0, 0, 0, 0, 0, 0.8, 1, 1},
                            {"lp2_80", false, false, 0, 64, 64, 0, 0, 0, 0, 0, 0, 2, 0.8},
                            {"mphf32", false, false, 0, 64, 64, 0, 0, 0, 0, 0, 0, 0, 0.8, 0, 0, 32},
                            {"mphf64", false, false, 0, 64, 64, 0, 0, 0, 0, 0, 0, 0, 0.8, 0, 0, 64},
                            {"lp2_60", false, false, 0, 64, 64, 0, 0, 0, 0, 0, 0, 2, 0.6},
                            {"lp4_80", false, false, 0, 64, 64, 0, 0, 0, 0, 0, 0, 4, 0.8},
                            {"lp4_60", false, false, 0, 64, 64, 0, 0, 0, 0, 0, 0, 4, 0.6},
                            {"lp1_50", false, false, 0, 64, 64, 0, 0, 0, 0, 0, 0, 1, 0.5},
                            {"lp1_25", false, false, 0, 64, 64, 0, 0, 0, 0, 0, 0, 1, 0.25}};
    struct LpTab {
        uint64_t sets = 0;
        std::vector<uint8_t> used, flag;
        std::unordered_map<uint64_t, uint64_t> at;  // group -> set
    };
    std::unordered_map<std::string, LpTab> lptabs;
    auto lp_build = [&](const Variant &V) -> LpTab & {
        LpTab &L = lptabs[V.name];
        if (L.sets) return L;
        uint64_t slots = 0;
        std::vector<std::pair<uint64_t, uint32_t>> g;  // group key, slots
        for (const auto &b : h.btab)
            if (b.tag) {
                uint32_t k = b.n == INFW_BUCKET_OVERFLOW ? 1u : b.n;
                if (k > (uint32_t)V.lp) k = 1;  // more records than a set holds: an overflow marker (lp 1: one
                                                // group per 64-B bucket, as today, at a higher load)
                g.push_back({(uint64_t)(b.tag - 1) << 32 | b.top, k});
                slots += k;
            }
        L.sets = std::max<uint64_t>(1, (uint64_t)(slots / (V.lp * V.lp_load)) + 1);
        L.used.assign(L.sets, 0);
        L.flag.assign(L.sets, 0);
        uint64_t far = 0;
        for (const auto &x : g) {
            uint64_t s0 = infw_bucket_hash((uint32_t)(x.first >> 32), (uint32_t)x.first) % L.sets, s = s0;
            while (L.used[s] + x.second > (uint32_t)V.lp) {
                L.flag[s] = 1;
                s = (s + 1) % L.sets;
            }
            L.used[s] += x.second;
            L.at[x.first] = s;
            far += s != s0;
        }
        fprintf(stderr, "[lp %s] %zu groups, %llu slots, %llu sets, %.4f off home\n", V.name, g.size(),
                (unsigned long long)slots, (unsigned long long)L.sets, (double)far / std::max<size_t>(g.size(), 1));
        return L;
    };
    std::vector<int8_t> d16ok;
    const uint64_t tbl24_bytes = getenv("CACHESIM_TBL24_BYTES") ? atoi(getenv("CACHESIM_TBL24_BYTES")) : 8;  // word size  // per (slot, /16): -1 unknown, 0 tbl24, 1 inline
    // per-class part counts for clsP
    int cls_plog[INFW_NCLS];
    for (int c = 0; c < INFW_NCLS; c++) {
        cls_plog[c] = 4;
        for (int pp = 0; pp < 4; pp++) {
            uint64_t lines = 0, over = 0;
            for (uint32_t l = 0; l < h.n_lists; l++) {
                const auto &st = seg_starts[(size_t)l * INFW_NCLS + c];
                const uint32_t w = 65536u >> pp;
                for (uint32_t q = 0; q < (1u << pp); q++) {
                    uint32_t nseg = 1;
                    for (uint32_t x : st) nseg += x > q * w && x < (q + 1) * w;
                    lines++;
                    over += nseg > INFW_DT_CLEAF_SEGS;
                }
            }
            if (over * 256 <= lines) {
                cls_plog[c] = pp;
                break;
            }
        }
        printf("{\"class\": %d, \"plog2\": %d}\n", c, cls_plog[c]);
    }
    for (int Q : {4, 8, 16}) {  // how many (list, class, part) lines overflow 20 segments
        uint64_t parts = 0, over = 0;
        for (const auto &st : seg_starts)
            for (int q = 0; q < Q; q++) {
                const uint32_t lo = (uint32_t)q * (65536 / Q), hi = lo + 65536 / Q;
                uint32_t nseg = 1;
                for (uint32_t x : st) nseg += x > lo && x < hi;
                parts++;
                over += nseg > INFW_DT_CLEAF_SEGS;
            }
        printf("{\"parts\": %d, \"lines\": %llu, \"over_20_segments\": %llu}\n", Q, (unsigned long long)parts,
               (unsigned long long)over);
    }
    {  // path census (compiled layout): which lookups a packet needs
        uint64_t v4 = 0, v4_8 = 0, v6 = 0, v6_long = 0, v6_short = 0, v6_8 = 0, nolist = 0;
        std::vector<uint32_t> runs_hist(9, 0);
        for (uint64_t g = 0; g < (h.tbl8.size() >> 8); g++) {
            uint32_t r = 1;
            for (int j = 1; j < 256; j++) r += h.tbl8[g * 256 + j] != h.tbl8[g * 256 + j - 1];
            runs_hist[r < 8 ? r : 8]++;
        }
        for (uint64_t i = 0; i < n; i++) {
            const uint32_t *q = &tup[i * 8];
            int cls = 0;
            uint32_t val = 0;
            const int pk = infw_parse(q[6], q[7], &cls, &val);
            if (pk < INFW_PK_V4) continue;
            const int slot = infw_if_slot(t, q[4]);
            if (slot < 0) continue;
            const uint32_t a32 = infw_bswap32(q[0]);
            const uint64_t w = t.tbl24[((uint64_t)slot << 24) | (a32 >> 8)];
            const bool grp = (w & INFW_D24_GROUP) && !(w & INFW_D24_INLINE);
            if (pk == INFW_PK_V4) {
                v4++;
                v4_8 += grp;
            } else {
                v6++;
                if (infw_v6_long(t, (uint32_t)slot, a32, q)) v6_long++;
                else {
                    v6_short++;
                    v6_8 += grp;
                }
            }
            nolist += infw_lpm(t, pk, q[4], q) == 0;
        }
        printf("{\"census\": {\"v4\": %.4f, \"v4_tbl8\": %.4f, \"v6\": %.4f, \"v6_long_hit\": %.4f, "
               "\"v6_then_short\": %.4f, \"v6_tbl8\": %.4f, \"no_entry\": %.4f}, \"tbl8_runs_hist\": [",
               (double)v4 / n, (double)v4_8 / n, (double)v6 / n, (double)v6_long / n, (double)v6_short / n,
               (double)v6_8 / n, (double)nolist / n);
        for (int r = 0; r < 9; r++) printf("%s%u", r ? ", " : "", runs_hist[r]);
        printf("]}\n");
    }
    {  // IPv6 bucket probe lengths: per lookup, and the slowest lane of each 64-packet wave
        uint64_t looks = 0, probes = 0, waves = 0, wave_max_sum = 0;
        uint32_t hist[8] = {};
        uint32_t wmax = 0;
        for (uint64_t i = 0; i < n; i++) {
            if (i % 64 == 0 && i) {
                wave_max_sum += wmax;
                waves++;
                wmax = 0;
            }
            const uint32_t *q = &tup[i * 8];
            int cls = 0;
            uint32_t val = 0;
            if (infw_parse(q[6], q[7], &cls, &val) != INFW_PK_V6 || !t.n_levels) continue;
            const int slot = infw_if_slot(t, q[4]);
            if (slot < 0) continue;
            const uint32_t a32 = infw_bswap32(q[0]);
            uint64_t b = infw_bucket_hash((uint32_t)slot, a32) & t.bmask;
            uint32_t np = 1;
            for (;;) {
                const infw_v6_bucket &bk = t.btab[b];
                if (bk.tag == 0 || (bk.tag == (uint32_t)slot + 1 && bk.top == a32)) break;
                b = (b + 1) & t.bmask;
                np++;
            }
            looks++;
            probes += np;
            hist[np < 8 ? np : 7]++;
            wmax = np > wmax ? np : wmax;
        }
        printf("{\"v6_bucket_probes\": %.3f, \"wave_max_probes\": %.3f, \"load\": %.3f, \"hist\": [%u, %u, %u, %u, %u, %u, %u]}\n",
               (double)probes / looks, (double)wave_max_sum / waves, (double)h.n_buckets / h.btab.size(), hist[1],
               hist[2], hist[3], hist[4], hist[5], hist[6], hist[7]);
    }
    for (int lds_entries : {512, 1024, 2048}) {  // per-workgroup LDS cache of first-match results keyed by
        // (list, class, value): a hit needs no decision line (Zipf-hot lists with service ports repeat the key)
        const uint64_t per_wg = getenv("CACHESIM_WG_PACKETS") ? strtoull(getenv("CACHESIM_WG_PACKETS"), 0, 10) : 131072;
        const uint32_t wgs = (uint32_t)(n / per_wg) ? (uint32_t)(n / per_wg) : 1;
        std::vector<uint64_t> tag((size_t)wgs * lds_entries, ~0ull);
        uint64_t look = 0, hit = 0;
        for (uint64_t i = 0; i < n; i++) {
            const uint32_t *q = &tup[i * 8];
            int cls = 0;
            uint32_t val = 0;
            const int pk = infw_parse(q[6], q[7], &cls, &val);
            if (pk < INFW_PK_V4) continue;
            const uint32_t l1 = infw_lpm(t, pk, q[4], q);
            if (!l1) continue;
            const uint64_t key = (uint64_t)l1 << 19 | (uint64_t)cls << 16 | val;
            const uint32_t wg = (uint32_t)((i / 768) % wgs);
            const uint32_t idx = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 40) % (uint32_t)lds_entries;
            uint64_t &e = tag[(size_t)wg * lds_entries + idx];
            look++;
            hit += e == key;
            e = key;
        }
        printf("{\"lds_result_cache\": %d, \"decision_lookups_per_packet\": %.4f, \"hit_rate\": %.4f}\n", lds_entries,
               (double)look / n, (double)hit / std::max<uint64_t>(look, 1));
    }
    for (int lds_entries : {256, 1024, 2048}) {  // per-workgroup direct-mapped LDS cache of tbl24 words
        const uint64_t per_wg = getenv("CACHESIM_WG_PACKETS") ? strtoull(getenv("CACHESIM_WG_PACKETS"), 0, 10) : 131072;
        const uint32_t wgs = (uint32_t)(n / per_wg) ? (uint32_t)(n / per_wg) : 1;  // ~131k packets per workgroup, as at 128M packets over 1024 workgroups
        std::vector<uint64_t> tag((size_t)wgs * lds_entries, ~0ull);
        uint64_t look = 0, hit = 0;
        for (uint64_t i = 0; i < n; i++) {
            const uint32_t *q = &tup[i * 8];
            int cls = 0;
            uint32_t val = 0;
            const int pk = infw_parse(q[6], q[7], &cls, &val);
            if (pk != INFW_PK_V4) continue;
            const int slot = infw_if_slot(t, q[4]);
            if (slot < 0) continue;
            const uint64_t key = ((uint64_t)slot << 24) | (infw_bswap32(q[0]) >> 8);
            const uint32_t wg = (uint32_t)((i / 512) % wgs);
            uint64_t &e = tag[(size_t)wg * lds_entries + (key * 0x9E3779B1u >> 8) % lds_entries];
            look++;
            if (e == key) hit++;
            else e = key;
        }
        printf("{\"lds_tbl24_cache\": %d, \"v4_lookups_per_packet\": %.4f, \"hit_rate\": %.4f}\n", lds_entries,
               (double)look / n, (double)hit / look);
    }
    // per-workgroup direct-mapped LDS caches of whole 64-B lines: decision entry lines keyed by
    // (list, class, part) and IPv6 first-probe bucket lines keyed by (slot, /32)
    for (int lines : {64, 128, 256, 512}) {
        const uint64_t per_wg = getenv("CACHESIM_WG_PACKETS") ? strtoull(getenv("CACHESIM_WG_PACKETS"), 0, 10) : 131072;
        const uint32_t wgs = (uint32_t)(n / per_wg) ? (uint32_t)(n / per_wg) : 1;
        std::vector<uint64_t> etag((size_t)wgs * lines, ~0ull), btag((size_t)wgs * lines, ~0ull);
        uint64_t el = 0, eh = 0, bl = 0, bh = 0;
        for (uint64_t i = 0; i < n; i++) {
            const uint32_t *q = &tup[i * 8];
            int cls = 0;
            uint32_t val = 0;
            const int pk = infw_parse(q[6], q[7], &cls, &val);
            if (pk < INFW_PK_V4) continue;
            const int slot = infw_if_slot(t, q[4]);
            if (slot < 0) continue;
            const uint32_t wg = (uint32_t)((i / 512) % wgs);
            const uint32_t a32 = infw_bswap32(q[0]);
            if (pk == INFW_PK_V6 && t.n_levels) {
                const uint64_t key = ((uint64_t)slot << 32) | a32;
                uint64_t &e = btag[(size_t)wg * lines + ((key * 0x9E3779B97F4A7C15ull) >> 40) % lines];
                bl++;
                if (e == key) bh++;
                else e = key;
            }
            const uint32_t l1 = infw_lpm(t, pk, q[4], q);
            if (!l1) continue;
            const uint32_t pl = l1 - 1 < t.n_dt_pl ? (t.dt_pl[l1 - 1] >> (3 * cls)) & 7u : t.dt_plog2;
            const uint64_t key = infw_dt_slot_p(l1 - 1, cls, val, t.dt_plog2, pl);
            uint64_t &e = etag[(size_t)wg * lines + ((key * 0x9E3779B97F4A7C15ull) >> 40) % lines];
            el++;
            if (e == key) eh++;
            else e = key;
        }
        printf("{\"lds_line_cache\": %d, \"entry_lookups_per_packet\": %.4f, \"entry_hit_rate\": %.4f, "
               "\"bucket_lookups_per_packet\": %.4f, \"bucket_hit_rate\": %.4f}\n",
               lines, (double)el / n, (double)eh / el, (double)bl / n, (double)bh / bl);
        fflush(stdout);
    }
    // IPv6 group census (records per (slot, /32) group) and a what-if: the groups in a two-choice
    // table of 64-B buckets holding CUCKOO_SLOTS single-record groups each, at CUCKOO_LOAD
    std::unordered_map<uint64_t, uint64_t> cuckoo_at;  // group key -> bucket index (+ 1 << 62 if secondary)
    uint64_t cuckoo_buckets = 1;
    {
        uint64_t hist[6] = {}, ng = 0;
        std::vector<uint64_t> gk;
        for (const auto &b : h.btab)
            if (b.tag) {
                hist[b.n == INFW_BUCKET_OVERFLOW ? 5 : b.n < 4 ? b.n : 4]++;
                ng++;
                gk.push_back((uint64_t)(b.tag - 1) << 32 | b.top);
            }
        const double load = getenv("CUCKOO_LOAD") ? atof(getenv("CUCKOO_LOAD")) : 0.5;
        const uint32_t slots = getenv("CUCKOO_SLOTS") ? atoi(getenv("CUCKOO_SLOTS")) : 2;
        while ((double)cuckoo_buckets * slots * load < (double)ng) cuckoo_buckets <<= 1;
        std::vector<uint32_t> fill(cuckoo_buckets, 0);
        uint64_t sec = 0, fail = 0;
        for (uint64_t k : gk) {
            const uint64_t h1 = infw_bucket_hash((uint32_t)(k >> 32), (uint32_t)k) & (cuckoo_buckets - 1);
            const uint64_t h2 = (infw_bucket_hash((uint32_t)(k >> 32) ^ 0x5bd1e995u, (uint32_t)k) >> 7) & (cuckoo_buckets - 1);
            if (fill[h1] < slots) { fill[h1]++; cuckoo_at[k] = h1; }
            else if (fill[h2] < slots) { fill[h2]++; cuckoo_at[k] = h2 | 1ull << 62; sec++; }
            else fail++;
        }
        printf("{\"v6_groups\": %llu, \"records_hist\": [%llu, %llu, %llu, %llu, %llu, %llu], \"cuckoo\": {\"load\": %.2f, "
               "\"slots\": %u, \"buckets\": %llu, \"secondary\": %.4f, \"unplaced\": %llu}}\n",
               (unsigned long long)ng, (unsigned long long)hist[0], (unsigned long long)hist[1],
               (unsigned long long)hist[2], (unsigned long long)hist[3], (unsigned long long)hist[4],
               (unsigned long long)hist[5], load, slots, (unsigned long long)cuckoo_buckets, (double)sec / ng,
               (unsigned long long)fail);
    }
    if (getenv("CACHESIM_LDS_ONLY")) return 0;
    const char *only = getenv("CACHESIM_VARIANTS");
    const int xcd_mode = getenv("CACHESIM_XCD") ? atoi(getenv("CACHESIM_XCD")) : 0;
    for (const Variant &V : vars) {
        if (only && !strstr(only, V.name)) continue;
        std::vector<L2> l2(8, L2(4ull << 20));
        // CACHESIM_PHASES=1: a two-launch split (the whole batch's LPM, then its decision lookups) — the entry
        // and leaf lines get an L2 of their own instead of sharing it with the LPM lines
        const bool phases = getenv("CACHESIM_PHASES") && atoi(getenv("CACHESIM_PHASES"));
        std::vector<L2> l2b(phases ? 8 : 0, L2(4ull << 20));
        uint64_t req[S_N] = {}, miss[S_N] = {}, mmiss[S_N] = {};
        // CACHESIM_MALL=1: the 256-MB Infinity Cache behind the L2s (one shared LRU model, 128-B lines); with
        // CACHESIM_MALL_STREAM=1 the tuple stream's lines (32 B per packet) pass through it too
        const bool mall_on = getenv("CACHESIM_MALL") && atoi(getenv("CACHESIM_MALL"));
        const bool mall_stream = getenv("CACHESIM_MALL_STREAM") && atoi(getenv("CACHESIM_MALL_STREAM"));
        L2 mall(mall_on ? (256ull << 20) : 2048);
        for (uint64_t i = 0; i < n; i++) {
            const uint32_t *q = &tup[i * 8];
            int cls = 0;
            uint32_t val = 0;
            const int pk = infw_parse(q[6], q[7], &cls, &val);
            if (pk < INFW_PK_V4) continue;
            Touch tc[6];
            int nt = 0;
            const int slot = infw_if_slot(t, q[4]);
            uint32_t l1 = 0;
            if (slot >= 0) {
                const uint32_t a32 = infw_bswap32(q[0]);
                uint32_t lng = 0;
                if (pk == INFW_PK_V6 && t.n_levels) {
                    const uint64_t bi = infw_bucket_hash((uint32_t)slot, a32) & t.bmask;  // first probe only
                    tc[nt++] = {S_BUCKET, 0 * kSpace + bi * 64};
                    if (V.lp) {  // home set, then the flagged sets after it until the group's own
                        LpTab &L = lp_build(V);
                        const uint64_t gk = (uint64_t)slot << 32 | a32;
                        auto it = L.at.find(gk);
                        uint64_t s = infw_bucket_hash((uint32_t)slot, a32) % L.sets;
                        const uint32_t sb = V.lp == 1 ? 64 : V.lp * 32;
                        tc[nt - 1].addr = 8 * kSpace + s * sb;
                        for (int hop = 0; hop < 3; hop++) {  // (at most 6 touches per packet in the model)
                            if ((it != L.at.end() && it->second == s) || !L.flag[s]) break;
                            s = (s + 1) % L.sets;
                            tc[nt++] = {S_BUCKET, 8 * kSpace + s * sb};
                        }
                    }
                    if (V.set4) {  // slots needed: one per record of every group (n_buckets groups, ~1.3 records each)
                        const uint64_t sets = std::max<uint64_t>(1, (uint64_t)(h.n_buckets * 1.31 / (4 * 0.8)));
                        tc[nt - 1].addr = 7 * kSpace + (infw_bucket_hash((uint32_t)slot, a32) % sets) * 128;
                    }
                    if (V.mphf) {
                        static std::unordered_map<uint64_t, uint64_t> rank;
                        if (rank.empty()) {
                            std::vector<uint64_t> gk;
                            for (const infw_v6_bucket &b : h.btab)
                                if (b.tag) gk.push_back((uint64_t)(b.tag - 1) << 32 | b.top);
                            std::sort(gk.begin(), gk.end());
                            uint64_t r = 0x9E3779B97F4A7C15ull;
                            for (size_t j = gk.size(); j > 1; j--) {  // Fisher-Yates with a fixed seed
                                r = r * 6364136223846793005ull + 1442695040888963407ull;
                                std::swap(gk[j - 1], gk[(r >> 33) % j]);
                            }
                            for (size_t j = 0; j < gk.size(); j++) rank[gk[j]] = j;
                        }
                        const uint64_t gkey = (uint64_t)slot << 32 | a32;
                        auto it = rank.find(gkey);
                        const uint64_t rk = it != rank.end() ? it->second : infw_bucket_hash((uint32_t)slot, a32) % rank.size();
                        tc[nt - 1].addr = 10 * kSpace + rk * V.mphf;
                    }
                    if (V.cuckoo) {
                        const uint64_t gk = (uint64_t)slot << 32 | a32;
                        auto it = cuckoo_at.find(gk);
                        const uint64_t h1 = infw_bucket_hash((uint32_t)slot, a32) & (cuckoo_buckets - 1);
                        const uint64_t h2 = (infw_bucket_hash((uint32_t)slot ^ 0x5bd1e995u, a32) >> 7) & (cuckoo_buckets - 1);
                        tc[nt - 1].addr = 5 * kSpace + h1 * 64;
                        if (it == cuckoo_at.end() || (it->second >> 62)) tc[nt++] = {S_BUCKET, 5 * kSpace + h2 * 64};
                    }
                    lng = infw_v6_long(t, (uint32_t)slot, a32, q);
                }
                if (!lng) {
                    const uint64_t w = ((uint64_t)slot << 24) | (a32 >> 8);
                    bool skip24 = false;
                    if (V.d16) {
                        if (d16ok.empty()) d16ok.assign((size_t)t.n_slots << 16, -1);
                        int8_t &ok = d16ok[((size_t)slot << 16) | (a32 >> 16)];
                        if (ok < 0) ok = d16_inline(t, (uint32_t)slot, a32 >> 16);
                        tc[nt++] = {S_D16, 6 * kSpace + (((uint64_t)slot << 16) | (a32 >> 16)) * 8};
                        skip24 = ok;
                    }
                    if (!skip24) tc[nt++] = {S_TBL24, 1 * kSpace + w * (V.tbl24_u16 ? 2 : tbl24_bytes)};
                    if (V.dense_short) {  // the longest <= /32 prefix covering a32 in this slot
                        uint64_t r = ~0ull;
                        for (int L = 32; L >= 0 && r == ~0ull; L--) {
                            const uint32_t net = L ? a32 & (~0u << (32 - L)) : 0;
                            auto it = short_rank.find(((uint64_t)slot << 40) | ((uint64_t)L << 32) | net);
                            if (it != short_rank.end()) r = it->second;
                        }
                        tc[nt - 1].addr = 1 * kSpace + (r == ~0ull ? (1ull << 35) + w * 8 : r * 8);
                    }
                    const uint64_t e = t.tbl24[w];
                    if (!skip24 && (e & INFW_D24_GROUP) && !(e & INFW_D24_INLINE)) {
                        const uint64_t w8 = ((uint64_t)(uint32_t)e << 8) | (a32 & 0xFFu);
                        tc[nt++] = {S_TBL8, 2 * kSpace + w8 * 4};
                    }
                    l1 = infw_dir24_lookup(t, (uint32_t)slot, a32);
                } else {
                    l1 = lng;
                }
            }
            if (l1 && V.quarters) {
                const uint64_t ei = (uint64_t)(l1 - 1) * INFW_NCLS + cls;
                const uint32_t Q = (uint32_t)V.quarters, q = val / (65536 / Q);
                const uint32_t cap = V.slot_bytes == 64 ? 20 : V.slot_bytes == 32 ? 10 : 5;
                tc[nt++] = {S_ENTRY, 3 * kSpace + (ei * Q + q) * V.slot_bytes};
                const auto &st = seg_starts[ei];
                const uint32_t lo = q * (65536 / Q), hi = lo + 65536 / Q;
                uint32_t nseg = 1, below = 0;
                for (uint32_t x : st) {
                    nseg += x > lo && x < hi;
                    below += x > lo && x <= val;
                }
                if (nseg > cap)  // root in the slot, then one leaf of 20 segments
                    tc[nt++] = {S_LEAF, 4 * kSpace + ((ei * Q + q) * 16 + below / INFW_DT_CLEAF_SEGS) * 64};
            } else if (l1) {
                const uint64_t ei = (uint64_t)(l1 - 1) * INFW_NCLS + cls;
                // entry32: a list's 7 classes in 256 B (TCP, UDP, SCTP, ICMP4 | ICMP6, 58/v4, 1/v6)
                tc[nt++] = {S_ENTRY, 3 * kSpace + (V.entry32 ? (uint64_t)(l1 - 1) * 256 + cls * 32 : ei * V.entry_stride)};
                const uint32_t pl = l1 - 1 < t.n_dt_pl ? (t.dt_pl[l1 - 1] >> (3 * cls)) & 7u : t.dt_plog2;
                const uint64_t slot_i = infw_dt_slot_p(l1 - 1, cls, val, t.dt_plog2, pl);  // the compiled image's line
                if (t.dt_plog2) tc[nt - 1].addr = 3 * kSpace + slot_i * 64;  // the compiled layout's entry line
                if (t.dt_plog2 && V.pairing == 1)
                    tc[nt - 1].addr = 3 * kSpace + (((uint64_t)(l1 - 1) * 16 + (val >> 12)) * 8 + cls) * 64;
                if (t.dt_plog2 && V.pairing == 2)  // list-minor: (class, part) major, adjacent lists share a line
                    tc[nt - 1].addr = 3 * kSpace + (((uint64_t)cls * 16 + (val >> 12)) * h.n_lists + (l1 - 1)) * 64;
                if (t.dt_plog2 == 4 && V.adapt) {  // fewest parts (1 << p) whose every part holds <= 20 segments
                    static std::vector<int8_t> pbest;
                    if (pbest.empty()) pbest.assign((size_t)h.n_lists * INFW_NCLS, -1);
                    int8_t &pb = pbest[ei];
                    if (pb < 0) {
                        const auto &st = seg_starts[ei];
                        pb = 4;
                        for (int pp = 0; pp < 4; pp++) {
                            const uint32_t w = 65536u >> pp;
                            bool ok = true;
                            for (uint32_t q = 0; q < (1u << pp) && ok; q++) {
                                uint32_t nseg = 1;
                                for (uint32_t x : st) nseg += x > q * w && x < (q + 1) * w;
                                ok = nseg <= INFW_DT_CLEAF_SEGS;
                            }
                            if (ok) {
                                pb = (int8_t)pp;
                                break;
                            }
                        }
                    }
                    if (pb < 4) tc[nt - 1].addr = 3 * kSpace + (ei * 16 + (val >> (16 - pb))) * 64;
                }
                if (t.dt_plog2 == 4 && V.cls_p && cls_plog[cls] < 4)
                    tc[nt - 1].addr = 3 * kSpace + (ei * 16 + (val >> (16 - cls_plog[cls]))) * 64;
                if (t.dt_plog2 && V.mini) {  // mini entry first; the 64-B line only for parts with more segments
                    const auto &st = seg_starts[ei];
                    const uint32_t q = val >> 12, lo = q << 12, hi = lo + 4096;
                    uint32_t nseg = 1;
                    for (uint32_t x : st) nseg += x > lo && x < hi;
                    const uint64_t line_addr = tc[nt - 1].addr;
                    tc[nt - 1] = {S_ENTRY, 6 * kSpace + slot_i * 16};
                    if (nseg > (uint32_t)V.mini) tc[nt++] = {S_ENTRY, line_addr};
                }
                const uint32_t *w = t.dte[slot_i].w;
                if (w[0] & INFW_DT_ROOT) {
                    const uint64_t li = (w[0] & INFW_DT_INDEX) + infw_keys_below(w, 1, 16, val);
                    tc[nt++] = {S_LEAF, 4 * kSpace + li * 64};
                }
            }
            L2 &c = l2[(i / 512) % 8];
            if (mall_stream && (i & 3) == 0) mall.access(9 * kSpace + i * 32);
            for (int k = 0; k < nt; k++) {
                req[tc[k].s]++;
                L2 *cp = phases && (tc[k].s == S_ENTRY || tc[k].s == S_LEAF) ? &l2b[(i / 512) % 8] : &c;
                // CACHESIM_XCD=1: decision lines served by the XCD their list hashes to (packets binned by list
                // between an LPM phase and a decision phase); 2: every line by the XCD its address hashes to (the
                // eight L2s as one 32-MiB cache: the bound of any XCD-partitioned design)
                const bool dec = tc[k].s == S_ENTRY || tc[k].s == S_LEAF;
                // 3: packets grouped by a hash of their source /24 (IPv4) or /32 (IPv6) and the ifindex, one group
                // per XCD (an RSS-style queue split of the batch); 4: the same by the full source address
                if (xcd_mode >= 3) {
                    const uint32_t *q = &tup[i * 8];
                    const uint32_t a0 = infw_bswap32(q[0]);
                    uint64_t hk = xcd_mode == 3 ? (pk == INFW_PK_V4 ? (uint64_t)(a0 >> 8) : (uint64_t)a0 | 1ull << 40)
                                                : ((uint64_t)q[0] << 32 | q[1]) ^ ((uint64_t)q[2] << 32 | q[3]) * 31;
                    hk = hk * 0x9E3779B97F4A7C15ull + q[4];
                    cp = &l2[((hk * 0xD6E8FEB86659FD93ull) >> 61) & 7];
                } else if ((xcd_mode == 1 && dec) || xcd_mode == 2) {
                    const uint64_t hk = xcd_mode == 1 ? (uint64_t)l1 : tc[k].addr / 128;
                    cp = &l2[((hk * 0xD6E8FEB86659FD93ull) >> 61) & 7];
                }
                L2 &ck = *cp;
                if (!ck.access(tc[k].addr)) {
                    miss[tc[k].s]++;
                    if (mall_on && !mall.access(tc[k].addr)) mmiss[tc[k].s]++;
                }
            }
        }
        double tr = 0, tm = 0;
        printf("{\"variant\": \"%s\", \"packets\": %llu", V.name, (unsigned long long)n);
        for (int s = 0; s < S_N; s++) {
            printf(", \"%s\": [%.4f, %.4f]", kName[s], (double)req[s] / n, (double)miss[s] / n);
            tr += (double)req[s] / n;
            tm += (double)miss[s] / n;
        }
        printf(", \"requests\": %.4f, \"misses\": %.4f", tr, tm);
        if (mall_on) {
            double tmm = 0;
            printf(", \"mall_misses\": {");
            for (int s = 0; s < S_N; s++) {
                printf("%s\"%s\": %.4f", s ? ", " : "", kName[s], (double)mmiss[s] / n);
                tmm += (double)mmiss[s] / n;
            }
            printf("}, \"mall_misses_total\": %.4f", tmm);
        }
        printf("}\n");
        fflush(stdout);
    }
    infw_wl_destroy(wl);
    return 0;
}
