// incremental.cpp — patch the compiled table image with the keys edited since
// the last commit, instead of recompiling the whole epoch.
//
// The reference updates its LPM trie one key at a time (addOrUpdateRules,
// loader.go:200-208; purgeKeys, :633-649).  Here a commit turns the dirty keys
// into the smallest set of changed table bytes:
//   <= /32 entries   the DIR-24-8 words their prefix covers are recomputed
//                    (longest entry <= /24 per tbl24 word, <= /32 per tbl8
//                    entry); a /25../32 entry under a plain word gets a tbl8
//                    group (appended; groups are never freed);
//   IPv6 /33../128   the (slot, /32) group's 64-B bucket is rewritten (or
//                    inserted into a free probe position);
//   new rule values  their rule list is compiled and appended (decision lines,
//                    class records) — lists are only appended, never moved.
// Everything that would change the layout — a new ifindex, the compressed
// short table, a group crossing 3 records (the Waldvogel overflow table), the
// first long prefix, a bucket table past 1/4 load, too many edits, or half of
// the lists unreferenced — is left to a full compile.  Decisions are made
// before anything is modified, so "needs a full compile" leaves the image intact.
#include <errno.h>

#include <algorithm>
#include <array>
#include <cstring>
#include <chrono>
#include <stdio.h>
#include <stdlib.h>

#include <thread>

#include "infw_internal.h"

namespace infw {

namespace {

inline uint32_t rd_le32(const uint8_t *p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

struct Edit {
    const NodeKey *key;
    const NodeVal *now;  // nullptr: absent after the edits
    int64_t was;         // committed value id, or PendingMap::kAbsent
    uint32_t slot, P;    // address bits
    uint32_t a32;        // address bits 0..31 (masked)
    uint64_t hi, lo;     // full address (masked), big-endian halves
};

void mark(std::vector<DirtyRange> &r, int buf, uint64_t off, uint64_t len) {
    if (len) r.push_back(DirtyRange{(uint32_t)buf, off, len});
}

// Answers of the /P block at address a of one ifindex at resolution R (24: tbl24 words, 32: tbl8 entries):
// every unit starts from `base` (the longest entry of length <= P covering the block) and the entries longer
// than P inside the block are painted over it in ascending length, so each unit ends with its longest match.
// The entries come from the map's per-block short-key lists — no probe per unit and length.  ans[u] is the
// answer of unit u (2^(R - P) units).
void paint(const PendingMap &m, uint32_t ifx, uint32_t a, uint32_t P, uint32_t R, const NodeVal *base,
           std::vector<const NodeVal *> &ans, std::vector<PendingMap::ShortRef> &tmp) {
    ans.assign(1ull << (R - P), base);
    tmp.clear();
    for (uint32_t lv = 0; lv < R; lv += 8) {  // the level-lv lists hold lengths (lv, lv + 8]
        if (lv + 8 <= P) continue;
        if (lv <= P) {  // one block covers the /P block: keep its entries longer than P inside it
            if (const auto *v = m.sub_list(lv, ifx, a))
                for (const auto &r : *v)
                    if (r.L > P && r.L <= R && (P == 0 || (r.a32 >> (32 - P)) == (a >> (32 - P)))) tmp.push_back(r);
        } else {        // 2^(lv - P) blocks inside the /P block
            const uint64_t nb = 1ull << (lv - P);
            for (uint64_t k = 0; k < nb; k++)
                if (const auto *v = m.sub_list(lv, ifx, a + (uint32_t)(k << (32 - lv))))
                    for (const auto &r : *v)
                        if (r.L <= R) tmp.push_back(r);
        }
    }
    std::sort(tmp.begin(), tmp.end(), [](const PendingMap::ShortRef &x, const PendingMap::ShortRef &y) { return x.L < y.L; });
    for (const auto &r : tmp) {
        const uint64_t off = (uint64_t)(r.a32 - a) >> (32 - R);
        std::fill(ans.begin() + off, ans.begin() + off + (1ull << (R - r.L)), r.v);
    }
}

// The records of one IPv6 group while it is edited: at most INFW_BUCKET_INLINE, plus one before the check that
// refuses a fourth — inline, no allocation per group.
struct SmallRecs {
    infw_v6_rec r[INFW_BUCKET_INLINE + 1];
    uint32_t n = 0;
    infw_v6_rec *begin() { return r; }
    infw_v6_rec *end() { return r + n; }
    const infw_v6_rec *begin() const { return r; }
    const infw_v6_rec *end() const { return r + n; }
    size_t size() const { return n; }
    bool empty() const { return n == 0; }
    infw_v6_rec &operator[](size_t i) { return r[i]; }
    void push_back(const infw_v6_rec &x) { r[n++] = x; }
    void assign(const infw_v6_rec *a, const infw_v6_rec *b) {
        n = (uint32_t)(b - a);
        std::copy(a, b, r);
    }
    void erase(infw_v6_rec *from, infw_v6_rec *to) {
        std::copy(to, end(), from);
        n -= (uint32_t)(to - from);
    }
};

bool shorts_empty(const std::vector<Edit> &edits) {
    for (const Edit &e : edits)
        if (e.P <= 32) return false;
    return true;
}

void derive_lid_of_vid(IncState &inc) {
    uint32_t top = 0;
    for (const auto &kv : inc.list_of_vid) top = std::max(top, kv.first + 1);
    inc.lid_of_vid.assign(top, ~0u);
    for (const auto &kv : inc.list_of_vid) inc.lid_of_vid[kv.first] = kv.second;
}

void derive_g8bits(const HostTables &h, IncState &inc) {
    inc.g8bits.assign(((size_t)h.n_slots << 24) / 64, 0);
    for (const auto &kv : h.tbl8_of) inc.g8bits[kv.first >> 6] |= 1ull << (kv.first & 63);
}

}  // namespace

void patch_prepare(const HostTables &h, IncState &inc) {
    if (!inc.valid) return;
    derive_lid_of_vid(inc);
    if (h.short_mode == INFW_SHORT_DIR24) derive_g8bits(h, inc);
}

int patch_tables(const PendingMap &m, HostTables &h, IncState &inc, std::vector<DirtyRange> &ranges,
                 std::string *why, const Options &opt) {
    auto full = [&](const char *reason) {
        if (why) *why = reason;
        return 1;
    };
    if (!inc.valid) return full("no compiled image to patch");
    const size_t n_edits = m.n_dirty();
    if (n_edits == 0) return 0;
    if (n_edits > std::max<size_t>(65536, m.nodes.size() / 4)) return full("too many edits");
    // a partial-ifindex prefix (prefixLen < 32) sets slot defaults under every word of the short table
    if (h.n_wild) return full("partial-ifindex prefixes present");

    // ---- pass 1: classify the edits and check that the layout survives them
    const auto tpa = std::chrono::steady_clock::now();
    std::vector<Edit> edits;
    edits.reserve(n_edits);
    uint64_t short_words = 0;
    bool any_short = false;
    for (size_t di = 0; di < n_edits; di++) {
        if (di + 8 < n_edits) __builtin_prefetch(&m.nodes.node(m.dirty_ids[di + 8]));
        const MapNode &n = m.nodes.node(m.dirty_ids[di]);
        Edit e;
        e.key = &n.key;
        e.now = n.live ? &n.val : nullptr;
        e.was = n.was;
        if (!e.now && e.was == PendingMap::kAbsent) continue;  // added and removed again
        if (n.key.plen < 32) return full("partial-ifindex prefix edited");
        const uint32_t ifx = rd_le32(n.key.md);
        auto s = inc.slot_of.find(ifx);
        if (s == inc.slot_of.end()) return full("new ifindex");
        e.slot = s->second;
        e.P = n.key.plen - 32;
        const uint8_t *ip = n.key.md + 4;
        e.hi = e.lo = 0;
        for (int i = 0; i < 8; i++) e.hi = e.hi << 8 | ip[i];
        for (int i = 8; i < 16; i++) e.lo = e.lo << 8 | ip[i];
        e.a32 = (uint32_t)(e.hi >> 32);
        if (e.P <= 32) {
            any_short = true;
            short_words += e.P <= 24 ? (1ull << (24 - e.P)) : 256;
        }
        edits.push_back(e);
    }
    if (any_short && h.short_mode != INFW_SHORT_DIR24) return full("short table is not DIR-24-8");
    if (short_words > (1ull << 22)) return full("edits cover too much of the short table");

    const auto tpb = std::chrono::steady_clock::now();
    // IPv6 long prefixes: the final record set of every touched (slot, /32) group
    struct Group {
        uint64_t bucket;  // btab index (found or insert position)
        bool found;
        SmallRecs recs;
    };
    std::unordered_map<uint64_t, Group> groups;
    groups.reserve(edits.size());
    const uint64_t bmask = h.btab.size() - 1;
    uint64_t new_buckets = 0;
    // every long edit's first bucket line, requested before the groups are read (a few hundred lines: they
    // arrive while the loop below starts, instead of one miss after another)
    for (const Edit &e : edits) {
        if (e.P <= 32 || h.levels.empty()) continue;
        const uint64_t hh = infw_bucket_hash(e.slot, e.a32);
        __builtin_prefetch(&h.btab[hh & bmask]);
    }
    for (const Edit &e : edits) {
        if (e.P <= 32) continue;
        if (h.levels.empty()) return full("first long prefix");
        const uint64_t gk = (uint64_t)e.slot << 32 | e.a32;
        auto git = groups.find(gk);
        if (git == groups.end()) {
            Group g;
            uint64_t i = infw_bucket_hash(e.slot, e.a32) & bmask;
            for (;;) {
                const infw_v6_bucket &b = h.btab[i];
                if (b.tag == 0) {
                    g.found = false;
                    break;
                }
                if (b.tag == e.slot + 1 && b.top == e.a32) {
                    g.found = true;
                    break;
                }
                i = (i + 1) & bmask;
            }
            g.bucket = i;
            if (g.found) {
                const infw_v6_bucket &b = h.btab[i];
                if (b.n == INFW_BUCKET_OVERFLOW) return full("edit in an overflowed IPv6 group");
                g.recs.assign(b.rec, b.rec + b.n);
            } else {
                new_buckets++;
            }
            git = groups.emplace(gk, std::move(g)).first;
        }
        // replace this prefix's record (if any) by its current state
        auto &rv = git->second.recs;
        const uint32_t mid = (uint32_t)e.hi;
        rv.erase(std::remove_if(rv.begin(), rv.end(),
                                [&](const infw_v6_rec &r) { return (r.meta >> 25) == e.P - 32 && r.mid == mid && r.lo == e.lo; }),
                 rv.end());
        if (e.now) rv.push_back(infw_v6_rec{e.lo, mid, (e.P - 32) << 25});  // list filled in pass 2
        if (rv.size() > INFW_BUCKET_INLINE) return full("IPv6 group exceeds 3 prefixes");
    }
    // compiled at load <= 1/8; past 1/4 the probe chains a wave waits for grow: recompile
    if ((h.n_buckets + new_buckets) * 4 > h.btab.size()) return full("IPv6 bucket table past 1/4 load");
    // two new groups may share an insert position: they must not
    {
        std::vector<uint64_t> pos;
        for (auto &kv : groups)
            if (!kv.second.found && !kv.second.recs.empty()) pos.push_back(kv.second.bucket);
        std::sort(pos.begin(), pos.end());
        if (std::adjacent_find(pos.begin(), pos.end()) != pos.end()) return full("IPv6 bucket probe collision");
    }

    const auto tpc = std::chrono::steady_clock::now();
    // lists: values not compiled yet, and the reference counts after the edits
    if (inc.lid_of_vid.empty() && !inc.list_of_vid.empty()) derive_lid_of_vid(inc);
    auto lid_of = [&](uint32_t vid) -> uint32_t { return vid < inc.lid_of_vid.size() ? inc.lid_of_vid[vid] : ~0u; };
    std::vector<uint32_t> new_vids;
    {
        std::unordered_map<uint32_t, int> seen;
        for (const Edit &e : edits)
            if (e.now && lid_of(e.now->vid) == ~0u && seen.emplace(e.now->vid, 0).second)
                new_vids.push_back(e.now->vid);
    }
    const uint64_t n_lists_after = h.n_lists + new_vids.size();
    if (n_lists_after >= (1u << 25)) return full("more than 2^25-1 rule lists");
    std::unordered_map<uint32_t, int64_t> ref_delta;  // existing lists only
    ref_delta.reserve(2 * edits.size());
    for (const Edit &e : edits) {
        if (e.was != PendingMap::kAbsent) {
            const uint32_t l = lid_of((uint32_t)e.was);
            if (l == ~0u) return full("committed value without a rule list");  // cannot happen: recompile
            ref_delta[l]--;
        }
        if (e.now) {
            const uint32_t l = lid_of(e.now->vid);
            if (l != ~0u) ref_delta[l]++;
        }
    }
    int64_t dead_after = (int64_t)inc.dead_lists;
    for (const auto &d : ref_delta) {
        const int64_t before = (int64_t)inc.list_refs[d.first], after = before + d.second;
        dead_after += (after == 0) - (before == 0);
    }
    if (dead_after > 1024 && (uint64_t)dead_after * 2 > n_lists_after) return full("half of the rule lists are unreferenced");

    // ---- pass 2: modify the image (nothing below can refuse)
    const auto tp0 = std::chrono::steady_clock::now();
    const uint32_t n_lists_before = h.n_lists;
    for (uint32_t vid : new_vids) {
        const uint32_t lid = h.n_lists++;
        inc.list_of_vid[vid] = lid;
        if (vid >= inc.lid_of_vid.size()) inc.lid_of_vid.resize(std::max<size_t>(vid + 1, m.pool.vals.size()), ~0u);
        inc.lid_of_vid[vid] = lid;
        inc.list_refs.push_back(0);
        const size_t r0 = h.rules.size(), l0 = h.dtl.size();
        // the image always holds >= 1 list slot: list 0 may be the placeholder of an empty epoch
        if (h.desc.size() < (size_t)(lid + 1) * INFW_DESC_STRIDE) h.desc.resize((size_t)(lid + 1) * INFW_DESC_STRIDE, 0);
        const size_t per_list = (size_t)INFW_NCLS << h.dt_plog2;
        if (h.dte.size() < (lid + 1) * per_list) h.dte.resize((lid + 1) * per_list, infw_dt_line{});
        // a list past the part-count table keeps uniform parts (infw_dt_parts_of)
        const bool pl = lid < h.dt_pl.size();
        int rc = compile_rule_list(m.pool.vals[vid].data(), h.rules, &h.desc[(size_t)lid * INFW_DESC_STRIDE],
                                   &h.dte[lid * per_list], h.dtl, h.dt_plog2, pl ? &h.dt_pl[lid] : nullptr);
        if (pl) mark(ranges, TB_DTPL, (uint64_t)lid * 4, 4);
        if (rc) {
            inc.valid = false;  // the image is no longer trustworthy: the next commit recompiles
            set_error("incremental commit: decision-table leaf pool exhausted");
            return rc;
        }
        mark(ranges, TB_DESC, (uint64_t)lid * INFW_DESC_STRIDE * sizeof(uint64_t), INFW_DESC_STRIDE * sizeof(uint64_t));
        mark(ranges, TB_DTE, (uint64_t)lid * per_list * sizeof(infw_dt_line), per_list * sizeof(infw_dt_line));
        mark(ranges, TB_RULES, r0 * sizeof(uint64_t), (h.rules.size() - r0) * sizeof(uint64_t));
        mark(ranges, TB_DTL, l0 * sizeof(infw_dt_line), (h.dtl.size() - l0) * sizeof(infw_dt_line));
    }
    for (const Edit &e : edits)  // references of the lists just created (ref_delta holds the older ones)
        if (e.now && lid_of(e.now->vid) >= n_lists_before) inc.list_refs[lid_of(e.now->vid)]++;
    for (const auto &d : ref_delta) inc.list_refs[d.first] = (uint64_t)((int64_t)inc.list_refs[d.first] + d.second);
    inc.dead_lists = (uint64_t)dead_after;
    // list + 1 of a node's value: painted words repeat a few values, so a small direct-mapped memo in front of
    // the hash map answers almost every word
    struct Memo {
        uint32_t vid = ~0u, l1 = 0;
    };
    std::array<Memo, 256> memo{}, memo6{};  // one per phase (the IPv6 phase may run on a second thread)
    auto list1_in = [&](std::array<Memo, 256> &mm, const NodeVal *v) -> uint32_t {
        if (!v) return 0u;
        Memo &e = mm[(v->vid * 0x9E3779B1u) >> 24];
        if (e.vid != v->vid) e = Memo{v->vid, lid_of(v->vid) + 1};
        return e.l1;
    };
    auto list1 = [&](const NodeVal *v) { return list1_in(memo, v); };

    // IPv6 buckets.  Touches only btab, n_buckets and the groups (the short-table phase below only
    // the DIR-24-8 words, tbl8 groups and g8bits; both read the map), so with enough of both kinds of edits it
    // runs on a second thread beside the short-table phase.
    std::vector<uint32_t> ifx_of_slot(h.n_slots, 0);
    for (const auto &kv : inc.slot_of) ifx_of_slot[kv.second] = kv.first;
    std::vector<DirtyRange> ranges6;
    auto v6_phase = [&]() {
        auto list1 = [&](const NodeVal *v) { return list1_in(memo6, v); };
        auto &ranges = ranges6;
        // the entry of every record of the touched groups ({ifindex, address bits 0..127} at its length), looked up
        // with the index slot prefetched 16 records ahead and the node 8 ahead
        struct RecKey {
            NodeKey k;
            uint64_t h;
            infw_v6_rec *r;
        };
        std::vector<RecKey> rks;
        rks.reserve(groups.size() * 2);
        for (auto &kv : groups) {
            Group &g = kv.second;
            if (!g.found && g.recs.empty()) continue;
            const uint32_t slot = (uint32_t)(kv.first >> 32), top = (uint32_t)kv.first;
            for (infw_v6_rec &r : g.recs) {
                uint8_t kmd[20];
                const uint32_t L = (r.meta >> 25) + 32;
                memcpy(kmd, &ifx_of_slot[slot], 4);
                const uint64_t hi = (uint64_t)top << 32 | r.mid;
                for (int i = 0; i < 8; i++) kmd[4 + i] = (uint8_t)(hi >> (56 - 8 * i));
                for (int i = 0; i < 8; i++) kmd[12 + i] = (uint8_t)(r.lo >> (56 - 8 * i));
                RecKey rk;
                rk.k.plen = L + 32;
                mask_bits(kmd, L + 32, rk.k.md, 20);
                rk.h = NodeTable::hash(rk.k);
                rk.r = &r;
                rks.push_back(rk);
            }
        }
        for (size_t i = 0; i < rks.size(); i++) {
            if (i + 16 < rks.size()) m.nodes.prefetch_slot(rks[i + 16].h);
            if (i + 8 < rks.size()) m.nodes.prefetch_node(rks[i + 8].k, rks[i + 8].h);
            const MapNode *n = m.nodes.find(rks[i].k, rks[i].h);
            rks[i].r->meta = (rks[i].k.plen - 64) << 25 | list1(n && n->live ? &n->val : nullptr);
        }
        for (auto &kv : groups) {
            Group &g = kv.second;
            if (!g.found && g.recs.empty()) continue;
            const uint32_t slot = (uint32_t)(kv.first >> 32), top = (uint32_t)kv.first;
            std::sort(g.recs.begin(), g.recs.end(), [](const infw_v6_rec &a, const infw_v6_rec &c) { return a.meta > c.meta; });
            infw_v6_bucket &b = h.btab[g.bucket];
            if (!g.found) {
                b.tag = slot + 1;
                b.top = top;
                h.n_buckets++;
            }
            b.n = (uint32_t)g.recs.size();
            memset(b.rec, 0, sizeof(b.rec));
            for (size_t k = 0; k < g.recs.size(); k++) b.rec[k] = g.recs[k];
            mark(ranges, TB_BTAB, g.bucket * sizeof(infw_v6_bucket), sizeof(infw_v6_bucket));
        }
    };

    const auto tp1 = std::chrono::steady_clock::now();
    const bool split = !groups.empty() && !shorts_empty(edits) && edits.size() >= 256;
    std::thread t6;
    if (split) t6 = std::thread(v6_phase);
    if (!shorts_empty(edits) && inc.g8bits.size() != ((size_t)h.n_slots << 24) / 64) derive_g8bits(h, inc);
    auto has_group = [&](uint64_t w) { return (inc.g8bits[w >> 6] >> (w & 63)) & 1; };
    // <= /32: shorter prefixes first, so a /25../32 group starts from its final tbl24 word
    std::vector<const Edit *> shorts;
    for (const Edit &e : edits)
        if (e.P <= 32) shorts.push_back(&e);
    std::sort(shorts.begin(), shorts.end(), [](const Edit *a, const Edit *b) { return a->P < b->P; });
    std::vector<const NodeVal *> ans, ans8;
    std::vector<PendingMap::ShortRef> tmp;
    uint64_t n_refills = 0, n_words = 0;
    // tbl8 entries [j0, j0 + 2^(32 - P)) of group g under /24 i24: the /P block's answers at /32,
    // from base = the answer of the lengths <= P
    auto refill_group = [&](uint32_t ifx, uint32_t i24, uint32_t g, uint32_t j0, uint32_t P, const NodeVal *base) {
        uint32_t *t8 = &h.tbl8[(size_t)g << 8];
        n_refills++;
        paint(m, ifx, i24 << 8 | j0, P, 32, base, ans8, tmp);
        for (size_t u = 0; u < ans8.size(); u++) t8[j0 + u] = list1(ans8[u]);
        mark(ranges, TB_TBL8, (((uint64_t)g << 8) + j0) * 4, (4ull << (32 - P)));
    };
    for (const Edit *e : shorts) {
        const uint8_t *ifx_le = e->key->md;
        const uint32_t ifx = rd_le32(ifx_le);
        uint64_t *t24 = &h.tbl24[(size_t)e->slot << 24];
        const uint64_t gkey = (uint64_t)e->slot << 24;
        const uint32_t a = e->P ? e->a32 & (~0u << (32 - e->P)) : 0u;
        const NodeVal *below = e->P ? m.longest_short(ifx_le, a, e->P - 1) : nullptr;  // lengths < P
        const NodeVal *atP = e->now ? e->now : below;                                 // lengths <= P
        if (e->P <= 24) {
            const uint32_t i0 = a >> 8, cnt = 1u << (24 - e->P);
            n_words += cnt;
            paint(m, ifx, a, e->P, 24, atP, ans, tmp);  // the longest entry <= /24 of every word
            for (uint32_t k = 0; k < cnt; k++) {
                const uint32_t i = i0 + k;
                if (!has_group(gkey | i)) {
                    t24[i] = list1(ans[k]);
                    continue;
                }
                auto g = h.tbl8_of.find(gkey | i);
                if (g != h.tbl8_of.end()) {
                    refill_group(ifx, i, g->second, 0, 24, ans[k]);
                    t24[i] = infw_d24_encode(&h.tbl8[(size_t)g->second << 8], g->second);
                } else {
                    t24[i] = list1(ans[k]);
                }
            }
            mark(ranges, TB_TBL24, (((uint64_t)e->slot << 24) + i0) * 8, (uint64_t)cnt * 8);
        } else {
            const uint32_t i = a >> 8;
            auto it = h.tbl8_of.find(gkey | i);
            uint32_t g;
            if (it != h.tbl8_of.end()) {
                g = it->second;
            } else {
                if (!e->now) continue;  // nothing below /24 here, nothing to remove
                g = (uint32_t)(h.tbl8.size() >> 8);  // groups are never freed: a uniform one is harmless
                h.tbl8.resize(h.tbl8.size() + 256, 0);
                std::fill(h.tbl8.begin() + ((size_t)g << 8), h.tbl8.begin() + ((size_t)g << 8) + 256, (uint32_t)t24[i]);
                mark(ranges, TB_TBL8, ((uint64_t)g << 8) * 4, 256 * 4);
                h.tbl8_of[gkey | i] = g;
                inc.g8bits[(gkey | i) >> 6] |= 1ull << ((gkey | i) & 63);
                h.n_tbl8_groups++;
            }
            refill_group(ifx, i, g, a & 0xFFu, e->P, atP);
            t24[i] = infw_d24_encode(&h.tbl8[(size_t)g << 8], g);
            mark(ranges, TB_TBL24, (((uint64_t)e->slot << 24) + i) * 8, 8);
        }
    }

    // /16 words in front of DIR-24-8 (d16_on): re-derived for every /16 an edit covers, from the words just painted
    if (h.d16_on && !shorts.empty()) {
        std::vector<uint64_t> blocks;  // slot << 16 | /16
        for (const Edit *e : shorts) {
            const uint32_t a = e->P ? e->a32 & (~0u << (32 - e->P)) : 0u;
            const uint32_t cnt = e->P >= 16 ? 1u : 1u << (16 - e->P);
            for (uint32_t k = 0; k < cnt; k++) blocks.push_back((uint64_t)e->slot << 16 | ((a >> 16) + k));
        }
        std::sort(blocks.begin(), blocks.end());
        blocks.erase(std::unique(blocks.begin(), blocks.end()), blocks.end());
        for (size_t i = 0; i < blocks.size();) {
            size_t j = i;
            for (; j < blocks.size() && blocks[j] == blocks[i] + (j - i); j++)
                h.d16[blocks[j]] = d16_word(h, (uint32_t)(blocks[j] >> 16), (uint32_t)blocks[j] & 0xFFFFu);
            mark(ranges, TB_D16, blocks[i] * 8, (uint64_t)(j - i) * 8);
            i = j;
        }
    }

    const auto tp2 = std::chrono::steady_clock::now();
    if (split) {
        t6.join();
    } else {
        v6_phase();
    }
    ranges.insert(ranges.end(), ranges6.begin(), ranges6.end());
    h.n_entries = m.nodes.size();
    // half-first decision-line reads: the per-epoch choice follows the lines appended (choose_dt_half's rule over
    // the running count), so an epoch grown by incremental commits reads its lines the way a compile would choose
    if (h.n_lists != n_lists_before) {
        const size_t per_list = (size_t)INFW_NCLS << h.dt_plog2;
        for (size_t e = (size_t)n_lists_before * per_list; e < (size_t)h.n_lists * per_list && e < h.dte.size(); e++)
            h.dt_short_lines += infw_dt_line_short(h.dte[e]);
        h.dt_half = choose_dt_half(h, opt.dt_half);
    }
    if (opt.trace & 2) {
        uint32_t minP = 99;
        for (const Edit *e : shorts) minP = std::min(minP, e->P);
        const auto tp3 = std::chrono::steady_clock::now();
        auto ms = [](auto d) { return std::chrono::duration<double, std::milli>(d).count(); };
        fprintf(stderr, "[patch] checks: scan %.3f, groups %.3f, lists %.3f ms\n", ms(tpb - tpa), ms(tpc - tpb), ms(tp0 - tpc));
        fprintf(stderr, "[patch] %zu edits: checks %.2f ms, lists %.2f ms (%zu new), shorts %.2f ms (%zu, shortest /%u; %llu tbl24 words, %llu tbl8 refills), "
                "IPv6 groups %.2f ms (%zu)\n", edits.size(), ms(tp0 - tpa), ms(tp1 - tp0), new_vids.size(), ms(tp2 - tp1),
                shorts.size(), minP, (unsigned long long)n_words, (unsigned long long)n_refills, ms(tp3 - tp2), groups.size());
    }
    return 0;
}

}  // namespace infw
