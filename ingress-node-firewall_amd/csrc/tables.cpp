// tables.cpp — the pending LPM map (control-plane semantics of
// ingress_node_firewall_table_map) and its compilation into the GPU table
// layout described in infw_tables.h.
#include <errno.h>

#include <stdlib.h>

#include <algorithm>
#include <numeric>
#include <queue>
#include <thread>
#include <array>
#include <chrono>
#include <stdio.h>

#include "infw_internal.h"

namespace infw {

static inline uint32_t rd_le32(const uint8_t *p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

// 24-B node key -> 64-bit hash: three 8-B words folded through multiply-rotate steps, then a final avalanche.
uint64_t NodeTable::hash(const NodeKey &k) {
    static_assert(sizeof(NodeKey) == 24, "NodeKey is 3 words");
    uint64_t w[3];
    memcpy(w, &k, 24);
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < 3; i++) {
        h ^= w[i] * 0xBF58476D1CE4E5B9ull;
        h = (h << 31 | h >> 33) * 0x94D049BB133111EBull;
    }
    h ^= h >> 29;
    h *= 0xBF58476D1CE4E5B9ull;
    return h ^ (h >> 32);
}

size_t NodeKeyHash::operator()(const NodeKey &k) const { return (size_t)NodeTable::hash(k); }

MapNode *NodeTable::find(const NodeKey &k, uint64_t h) const {
    const uint64_t tag = h >> 32;
    for (uint64_t i = tag & mask_;; i = (i + 1) & mask_) {
        const uint64_t s = slots_[i];
        if (!s) return nullptr;
        if ((s >> 32) == tag) {
            MapNode &n = const_cast<MapNode &>(node((uint32_t)s - 1));
            if (n.key == k) return &n;
        }
    }
}

void NodeTable::prefetch_node(const NodeKey &k, uint64_t h) const {
    (void)k;
    const uint64_t tag = h >> 32;
    for (uint64_t i = tag & mask_;; i = (i + 1) & mask_) {
        const uint64_t s = slots_[i];
        if (!s) return;
        if ((s >> 32) == tag) {
            __builtin_prefetch(&node((uint32_t)s - 1));
            return;
        }
    }
}

void NodeTable::grow(size_t cap) {
    std::vector<uint64_t> old(cap, 0);
    old.swap(slots_);
    mask_ = cap - 1;
    for (uint64_t s : old) {
        if (!s) continue;
        uint64_t i = (s >> 32) & mask_;
        while (slots_[i]) i = (i + 1) & mask_;
        slots_[i] = s;
    }
}

void NodeTable::reserve(size_t n) {
    size_t cap = slots_.size();
    while (cap < 2 * n) cap <<= 1;
    if (cap != slots_.size()) grow(cap);
}

MapNode *NodeTable::insert(const NodeKey &k, uint64_t h) {
    if (2 * (n_indexed_ + 1) > slots_.size()) grow(slots_.size() * 2);
    uint32_t id;
    if (!free_.empty()) {
        id = free_.back();
        free_.pop_back();
    } else {
        id = hw_++;
        if ((id >> kChunkLog) >= chunks_.size()) chunks_.emplace_back(new MapNode[kChunk]());
    }
    MapNode &n = node(id);
    n = MapNode{};
    n.key = k;
    n.id = id;
    const uint64_t tag = h >> 32;
    uint64_t i = tag & mask_;
    while (slots_[i]) i = (i + 1) & mask_;
    slots_[i] = tag << 32 | (uint64_t)(id + 1);
    n_indexed_++;
    return &n;
}

void NodeTable::erase(MapNode *n) {
    const uint64_t tag = hash(n->key) >> 32;
    uint64_t i = tag & mask_;
    while ((uint32_t)slots_[i] != n->id + 1) i = (i + 1) & mask_;
    // backward-shift deletion: pull later members of the probe run into the hole while their home allows it
    for (uint64_t j = (i + 1) & mask_; slots_[j]; j = (j + 1) & mask_) {
        const uint64_t home = (slots_[j] >> 32) & mask_;
        const bool stays = i <= j ? (home > i && home <= j) : (home > i || home <= j);
        if (stays) continue;
        slots_[i] = slots_[j];
        i = j;
    }
    slots_[i] = 0;
    n_indexed_--;
    set_live(n, false);
    n->dirty = 0;
    free_.push_back(n->id);
}

void NodeTable::clear() {
    slots_.assign(1024, 0);
    mask_ = 1023;
    n_indexed_ = n_live_ = 0;
    chunks_.clear();
    hw_ = 0;
    free_.clear();
}

static inline int bit_at(const uint8_t *d, uint32_t i) { return (d[i >> 3] >> (7 - (i & 7))) & 1; }

bool PostOrderLess::operator()(const NodeKey &a, const NodeKey &b) const {
    uint32_t mn = a.plen < b.plen ? a.plen : b.plen;
    // first differing bit within the common length decides (0-branch first)
    uint32_t full = mn >> 3;
    for (uint32_t i = 0; i < full; i++) {
        if (a.md[i] != b.md[i]) {
            uint8_t x = a.md[i] ^ b.md[i];
            int msb = 7;
            while (!((x >> msb) & 1)) msb--;
            return ((a.md[i] >> msb) & 1) < ((b.md[i] >> msb) & 1);
        }
    }
    for (uint32_t i = full * 8; i < mn; i++) {
        int x = bit_at(a.md, i), y = bit_at(b.md, i);
        if (x != y) return x < y;
    }
    return a.plen > b.plen;  // descendant (longer) before ancestor; equal -> false
}

static inline void mask_key20(const uint8_t *in, uint32_t plen, uint8_t *out);

void mask_bits(const uint8_t *in, uint32_t plen, uint8_t *out, int nbytes) {
    if (nbytes == 20) return mask_key20(in, plen, out);
    for (int i = 0; i < nbytes; i++) {
        uint32_t b0 = 8u * (uint32_t)i;
        if (plen >= b0 + 8) out[i] = in[i];
        else if (plen <= b0) out[i] = 0;
        else out[i] = (uint8_t)(in[i] & (0xFFu << (8 - (plen - b0))));
    }
}

// mask_bits over the 20 key bytes as big-endian words: the first `plen` bits kept, the rest cleared.
static inline void mask_key20(const uint8_t *in, uint32_t plen, uint8_t *out) {
    auto keep = [](uint32_t plen, uint32_t from) -> uint64_t {  // the top (plen - from) bits of a word
        if (plen <= from) return 0;
        const uint32_t b = plen - from;
        return b >= 64 ? ~0ull : ~0ull << (64 - b);
    };
    uint64_t w0, w1;
    uint32_t w2;
    memcpy(&w0, in, 8);
    memcpy(&w1, in + 8, 8);
    memcpy(&w2, in + 16, 4);
    w0 = __builtin_bswap64(__builtin_bswap64(w0) & keep(plen, 0));
    w1 = __builtin_bswap64(__builtin_bswap64(w1) & keep(plen, 64));
    w2 = __builtin_bswap32(__builtin_bswap32(w2) & (uint32_t)(keep(plen, 128) >> 32));
    memcpy(out, &w0, 8);
    memcpy(out + 8, &w1, 8);
    memcpy(out + 16, &w2, 4);
}

// 1200-B value hash, 8 bytes per step (interning 1M distinct values hashes 1.2 GB).
static uint64_t value_hash(const uint8_t *v) {
    uint64_t h = 0x84222325CBF29CE4ull;
    for (size_t i = 0; i < 1200; i += 8) {
        uint64_t w;
        memcpy(&w, v + i, 8);
        h = (h ^ w) * 0x9E3779B97F4A7C15ull;
        h ^= h >> 32;
    }
    h *= 0xBF58476D1CE4E5B9ull;
    return h ^ (h >> 29);
}

uint32_t ValuePool::intern(const uint8_t *v) {
    uint64_t h = value_hash(v);
    auto range = index.equal_range(h);
    for (auto it = range.first; it != range.second; ++it)
        if (memcmp(vals[it->second].data(), v, 1200) == 0) return it->second;
    uint32_t id = (uint32_t)vals.size();
    vals.emplace_back();
    memcpy(vals.back().data(), v, 1200);
    index.emplace(h, id);
    return id;
}

uint32_t ValuePool::intern_at(const uint8_t *v) {
    AddrMemo &e = memo_[((uintptr_t)v >> 4) * 0x9E3779B97F4A7C15ull >> 54];
    if (e.addr == v && memcmp(vals[e.vid].data(), v, 1200) == 0) return e.vid;
    e.addr = v;
    e.vid = intern(v);
    return e.vid;
}

void ValuePool::clear() {
    vals.clear();
    index.clear();
    memo_.fill(AddrMemo{});
}

static NodeKey make_node(const lpm_ip_key_st *key) {
    NodeKey k;
    k.plen = key->prefixLen;
    uint8_t data[20];
    memcpy(data, &key->ingress_ifindex, 4);
    memcpy(data + 4, key->ip_data, 16);
    mask_key20(data, k.plen, k.md);
    return k;
}

void PendingMap::prefetch_slot(const lpm_ip_key_st *key) const {
    if (key->prefixLen <= INFW_MAX_PREFIXLEN) nodes.prefetch_slot(NodeTable::hash(make_node(key)));
}

void PendingMap::prefetch_node(const lpm_ip_key_st *key) const {
    if (key->prefixLen > INFW_MAX_PREFIXLEN) return;
    const NodeKey k = make_node(key);
    nodes.prefetch_node(k, NodeTable::hash(k));
}

// trie_update_elem (lpm_trie.c, Linux 6.18) order of checks.
int PendingMap::update(const lpm_ip_key_st *key, const uint8_t *val, uint64_t flags) {
    if (flags > INFW_BPF_EXIST || key->prefixLen > INFW_MAX_PREFIXLEN) return update_vid(key, 0, flags);  // errors
    return update_vid(key, ~0u, flags, val);
}

// The first edit of a key since the last commit records its committed value.
static inline void mark_dirty(PendingMap &m, MapNode *n, int32_t committed) {
    if (n->dirty) return;
    n->dirty = 1;
    n->was = committed;
    m.dirty_ids.push_back(n->id);
}

// update() with the value already interned (vid), or interned here from val when vid == ~0u (only once the
// checks have passed, so a refused update interns nothing).
int PendingMap::update_vid(const lpm_ip_key_st *key, uint32_t vid, uint64_t flags, const uint8_t *val) {
    if (flags > INFW_BPF_EXIST) {
        set_error("update: flags > BPF_EXIST");
        return -EINVAL;
    }
    if (key->prefixLen > INFW_MAX_PREFIXLEN) {
        set_error("update: prefixLen > 160");
        return -EINVAL;
    }
    const NodeKey k = make_node(key);
    const uint64_t h = NodeTable::hash(k);
    MapNode *n = nodes.find(k, h);
    if (n && n->live) {
        if (flags == INFW_BPF_NOEXIST) return -EEXIST;
        mark_dirty(*this, n, (int32_t)n->val.vid);
        memcpy(n->val.data, &key->ingress_ifindex, 4);  // the last writer's host bits
        memcpy(n->val.data + 4, key->ip_data, 16);
        n->val.vid = vid == ~0u ? pool.intern(val) : vid;
        generation++;
        return 0;
    }
    if (flags == INFW_BPF_EXIST) return -ENOENT;
    if (nodes.size() >= max_entries) {
        set_error("update: table map full");
        return -ENOSPC;
    }
    if (!n) {  // a tombstone (removed since the last commit) is revived instead, keeping its committed value
        n = nodes.insert(k, h);
        mark_dirty(*this, n, kAbsent);
    }
    memcpy(n->val.data, &key->ingress_ifindex, 4);
    memcpy(n->val.data + 4, key->ip_data, 16);
    n->val.vid = vid == ~0u ? pool.intern(val) : vid;
    nodes.set_live(n, true);
    index_short(k, &n->val);
    order_add.insert(k);
    if (order_add.size() > std::max<size_t>(4096, order_vec.size() / 8)) order_merge();
    len_count[k.plen]++;
    generation++;
    return 0;
}

void PendingMap::index_short(const NodeKey &k, const NodeVal *v) {
    if (k.plen <= 32 || k.plen > 64) return;  // only keys of the short (<= 32 address bits) table, L >= 1
    const uint32_t L = k.plen - 32, ifx = rd_le32(k.md);
    const uint32_t a32 = (uint32_t)k.md[4] << 24 | (uint32_t)k.md[5] << 16 | (uint32_t)k.md[6] << 8 | k.md[7];
    const uint64_t sk = sub_key((L - 1) & ~7u, ifx, a32);
    if (v) {
        sub[sk].push_back(ShortRef{a32, L, v});
        return;
    }
    auto it = sub.find(sk);
    if (it == sub.end()) return;
    auto &vec = it->second;
    for (size_t i = 0; i < vec.size(); i++)
        if (vec[i].L == L && vec[i].a32 == a32) {
            vec[i] = vec.back();
            vec.pop_back();
            break;
        }
    if (vec.empty()) sub.erase(it);
}

int PendingMap::remove(const lpm_ip_key_st *key) {
    if (key->prefixLen > INFW_MAX_PREFIXLEN) return -EINVAL;
    const NodeKey k = make_node(key);
    MapNode *n = nodes.find(k, NodeTable::hash(k));
    if (!n || !n->live) return -ENOENT;
    mark_dirty(*this, n, (int32_t)n->val.vid);
    index_short(n->key, nullptr);
    nodes.set_live(n, false);  // stays indexed until the commit (clear_dirty); order entries go stale
    len_count[k.plen]--;
    generation++;
    return 0;
}

void PendingMap::clear_dirty() {
    for (uint32_t id : dirty_ids) {
        MapNode &n = nodes.node(id);
        n.dirty = 0;
        if (!n.live) nodes.erase(&n);
    }
    dirty_ids.clear();
}

// Merge the inserted keys into the sorted vector and drop keys no longer live (and duplicates).  Liveness is
// checked with the index lookups pipelined (slot prefetched 16 keys ahead, node 8 ahead).
void PendingMap::order_merge() const {
    if (order_add.empty() && order_vec.size() <= nodes.size()) return;
    std::vector<NodeKey> add(order_add.begin(), order_add.end());
    order_add.clear();
    auto live_filter = [&](std::vector<NodeKey> &v) {
        const size_t n = v.size();
        std::vector<uint64_t> hs(n);
        for (size_t i = 0; i < n; i++) hs[i] = NodeTable::hash(v[i]);
        size_t o = 0;
        for (size_t i = 0; i < n; i++) {
            if (i + 16 < n) nodes.prefetch_slot(hs[i + 16]);
            if (i + 8 < n) nodes.prefetch_node(v[i + 8], hs[i + 8]);
            const MapNode *m = nodes.find(v[i], hs[i]);
            if (m && m->live && (o == 0 || !(v[o - 1] == v[i]))) v[o++] = v[i];
        }
        v.resize(o);
    };
    live_filter(order_vec);
    live_filter(add);
    std::vector<NodeKey> out;
    out.reserve(order_vec.size() + add.size());
    std::merge(order_vec.begin(), order_vec.end(), add.begin(), add.end(), std::back_inserter(out), PostOrderLess());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    order_vec.swap(out);
}

int PendingMap::lookup(const lpm_ip_key_st *key, uint8_t *val) const {
    uint32_t kp = key->prefixLen > INFW_MAX_PREFIXLEN ? INFW_MAX_PREFIXLEN : key->prefixLen;
    uint8_t data[20];
    memcpy(data, &key->ingress_ifindex, 4);
    memcpy(data + 4, key->ip_data, 16);
    for (int L = (int)kp; L >= 0; L--) {
        if (!len_count[L]) continue;
        NodeKey k;
        k.plen = (uint32_t)L;
        mask_bits(data, (uint32_t)L, k.md, 20);
        if (const MapNode *n = nodes.find_live(k)) {
            if (val) memcpy(val, pool.vals[n->val.vid].data(), 1200);
            return 0;
        }
    }
    return -ENOENT;
}

const NodeVal *PendingMap::longest(const uint8_t md[20], uint32_t minlen, uint32_t maxlen) const {
    for (int L = (int)maxlen; L >= (int)minlen; L--) {
        if (!len_count[L]) continue;
        NodeKey k;
        k.plen = (uint32_t)L;
        mask_bits(md, (uint32_t)L, k.md, 20);
        if (const MapNode *n = nodes.find_live(k)) return &n->val;
    }
    return nullptr;
}

// longest() over the short key space of one ifindex: the entry of length L <= maxL (address bits) covering a32,
// found through the per-block short-key lists (one list per 8 lengths, longest level first) instead of one hash
// probe per length; L = 0 (prefixLen 32, the whole ifindex) is probed last.
const NodeVal *PendingMap::longest_short(const uint8_t ifx_le[4], uint32_t a32, uint32_t maxL) const {
    if (maxL > 32) maxL = 32;
    const uint32_t ifx = rd_le32(ifx_le);
    for (int lv = maxL ? (int)((maxL - 1) & ~7u) : -8; lv >= 0; lv -= 8) {
        const std::vector<ShortRef> *v = sub_list((uint32_t)lv, ifx, a32);
        if (!v) continue;
        const NodeVal *best = nullptr;
        uint32_t best_l = 0;
        for (const ShortRef &r : *v)
            if (r.L <= maxL && r.L > best_l && ((r.a32 ^ a32) >> (32 - r.L)) == 0) {
                best = r.v;
                best_l = r.L;
            }
        if (best) return best;
    }
    if (!len_count[32]) return nullptr;
    NodeKey k;
    k.plen = 32;
    memset(k.md, 0, sizeof k.md);
    memcpy(k.md, ifx_le, 4);
    const MapNode *n = nodes.find_live(k);
    return n ? &n->val : nullptr;
}

// trie_get_next_key: the key after `key` in post-order, or the first key when `key` is absent (or NULL).
int PendingMap::next_key(const lpm_ip_key_st *key, lpm_ip_key_st *next) const {
    if (nodes.empty()) return -ENOENT;
    if (order_vec.size() > 2 * nodes.size() + 4096) order_merge();  // mostly removed keys: compact first
    bool after = false;
    NodeKey k{};
    if (key && key->prefixLen <= INFW_MAX_PREFIXLEN) {
        k = make_node(key);
        after = nodes.find_live(k) != nullptr;
    }
    const PostOrderLess less;
    const MapNode *best = nullptr;
    auto vi = after ? std::upper_bound(order_vec.begin(), order_vec.end(), k, less) : order_vec.begin();
    for (; vi != order_vec.end(); ++vi)
        if ((best = nodes.find_live(*vi))) break;
    auto ai = after ? order_add.upper_bound(k) : order_add.begin();
    for (; ai != order_add.end(); ++ai) {
        if (best && !less(*ai, best->key)) break;  // the vector's candidate comes first
        if (const MapNode *n = nodes.find_live(*ai)) {
            best = n;
            break;
        }
    }
    if (!best) return -ENOENT;
    next->prefixLen = best->key.plen;
    memcpy(&next->ingress_ifindex, best->val.data, 4);
    memcpy(next->ip_data, best->val.data + 4, 16);
    return 0;
}

// ------------------------------------------------------------------------
// Rule lists.  For one 1200-B value, the rules each packet class can match,
// in slot order (kernel.c:222-258 / :306-340), as {lo16, hi16, result32}:
//   ruleId == 0                      skipped (:225-227)
//   protocol 0                       every class, any value (:255-257)
//   TCP/UDP/SCTP                     that class; end == 0 -> [start, start],
//                                    else [start, end-1] (end-exclusive :241);
//                                    an empty range never matches: dropped
//   ICMP (1)                         IPv4 path only (:247): [type<<8|code]
//   ICMPv6 (58)                      IPv6 path only (:329)
//   any other protocol               can never match: dropped
// result32 = SET_ACTIONRULE_RESPONSE(action, ruleId) (ingress_node_firewall.h:22).
// ------------------------------------------------------------------------
// First-match step function of a class list: sweep the 16-bit value axis
// keeping the lowest-index rule covering it (min-heap with lazy deletion),
// merge equal neighbours, then lay the segment starts out as a 9-ary search
// tree (infw_tables.h) followed by the results.
// Lay one step function (segment starts ascending from 0, results) out as an
// entry line and, above INFW_DT_LEAF_SEGS segments, leaf lines (infw_tables.h).
// Leaf over n <= segs consecutive segments: u16 keys (start of the next segment
// minus 1, pad 0xFFFF) in the halves of w[1 ..], results after them.
static void fill_leaf(infw_dt_line &l, const uint32_t *starts, const uint32_t *res, uint32_t n, bool compact) {
    memset(&l, 0, sizeof(l));
    const uint32_t segs = compact ? INFW_DT_CLEAF_SEGS : INFW_DT_LEAF_SEGS, kw = segs / 2;  // key words
    auto key = [&](uint32_t j) -> uint32_t { return j + 1 < n ? (uint16_t)(starts[j + 1] - 1) : 0xFFFFu; };
    if (compact) {  // half-first: the first 32 B answer every value below key 8, and every value when n <= 9
        l.w[0] = INFW_DT_COMPACT | n;
        for (uint32_t j = 0; j < INFW_DT_CLEAF_SEGS; j++) {
            l.w[infw_dt_ckey_word(j)] |= key(j) << (16 * (j & 1u));
            l.w[infw_dt_ccode_word(j)] |= infw_dt_result_code(j < n ? res[j] : res[n - 1]) << (8 * (j & 3u));
        }
        return;
    }
    for (uint32_t k = 0; k < kw; k++) l.w[1 + k] = key(2 * k) | key(2 * k + 1) << 16;
    {
        l.w[0] = n;
        for (uint32_t j = 0; j < segs; j++) l.w[1 + kw + j] = j < n ? res[j] : res[n - 1];
    }
}

// Host threads for compiling rule lists (Options::compile_threads overrides; lists are independent, so a
// compile of 1M distinct 99-rule lists scales with cores).  Small sets stay on the calling thread.
static int compile_threads(size_t n_items, int req) {
    if (n_items < 4096) return 1;
    const int t = req > 0 ? req : (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(t, 16));
}

// f(thread, begin, end) over nt contiguous chunks of [0, n).
template <class F>
static void parallel_chunks(size_t n, int nt, F f) {
    if (nt <= 1) {
        f(0, 0, n);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++) th.emplace_back(f, t, n * (size_t)t / (size_t)nt, n * (size_t)(t + 1) / (size_t)nt);
    for (auto &x : th) x.join();
}

int emit_decision_lines(const std::vector<uint32_t> &starts, const std::vector<uint32_t> &res, infw_dt_line &entry,
                        std::vector<infw_dt_line> &leaves) {
    const uint32_t S = (uint32_t)starts.size();
    bool compact = true;
    for (uint32_t r : res) compact = compact && infw_dt_result_code(r) <= 0xFFu;
    const uint32_t segs = compact ? INFW_DT_CLEAF_SEGS : INFW_DT_LEAF_SEGS;
    memset(&entry, 0, sizeof(entry));
    if (S <= segs) {
        fill_leaf(entry, starts.data(), res.data(), S, compact);
        return 0;
    }
    const uint32_t G = (S + segs - 1) / segs;
    if (G > INFW_DT_ROOT_KEYS + 1 || leaves.size() + G > INFW_DT_INDEX) return -ENOSPC;
    entry.w[0] = INFW_DT_ROOT | (uint32_t)leaves.size();
    uint16_t key[2 * 15];
    for (uint32_t j = 0; j < INFW_DT_ROOT_KEYS; j++)
        key[j] = j + 1 < G ? (uint16_t)(starts[(j + 1) * segs] - 1) : (uint16_t)0xFFFF;
    for (uint32_t k = 0; k < 15; k++) entry.w[1 + k] = (uint32_t)key[2 * k] | (uint32_t)key[2 * k + 1] << 16;
    for (uint32_t g = 0; g < G; g++) {
        infw_dt_line l;
        const uint32_t a = g * segs, n = std::min(segs, S - a);
        fill_leaf(l, starts.data() + a, res.data() + a, n, compact);
        leaves.push_back(l);
    }
    return 0;
}

int build_decision_table(const std::vector<uint64_t> &recs, infw_dt_line *entry, std::vector<infw_dt_line> &leaves,
                         uint32_t plog2) {
    std::vector<uint32_t> starts, res;
    step_function(recs, starts, res);
    const uint32_t span = 65536u >> plog2;
    std::vector<uint32_t> ps, pr;
    size_t j = 0;  // segment holding the part's first value
    for (uint32_t q = 0; q < (1u << plog2); q++) {
        const uint32_t lo = q * span, hi = lo + span;
        while (j + 1 < starts.size() && starts[j + 1] <= lo) j++;
        ps.assign(1, lo);
        pr.assign(1, res[j]);
        for (size_t k = j + 1; k < starts.size() && starts[k] < hi; k++) {
            ps.push_back(starts[k]);
            pr.push_back(res[k]);
        }
        const int rc = emit_decision_lines(ps, pr, entry[q], leaves);
        if (rc) return rc;
    }
    return 0;
}

void step_function(const std::vector<uint64_t> &recs, std::vector<uint32_t> &starts, std::vector<uint32_t> &res) {
    starts.clear();
    res.clear();
    const size_t c = recs.size();
    if (c == 0) {
        starts.push_back(0);
        res.push_back(0);
        return;
    }
    std::vector<std::pair<uint32_t, uint32_t>> ev;  // (position, rule index) starts
    std::vector<std::pair<uint32_t, uint32_t>> en;  // (position, rule index) ends (hi + 1)
    std::vector<uint32_t> pts{0};
    for (uint32_t i = 0; i < c; i++) {
        uint32_t lo = (uint32_t)recs[i] & 0xFFFFu, hi = (uint32_t)(recs[i] >> 16) & 0xFFFFu;
        ev.emplace_back(lo, i);
        pts.push_back(lo);
        if (hi + 1 <= 0xFFFFu) {
            en.emplace_back(hi + 1, i);
            pts.push_back(hi + 1);
        }
    }
    std::sort(pts.begin(), pts.end());
    pts.erase(std::unique(pts.begin(), pts.end()), pts.end());
    std::sort(ev.begin(), ev.end());
    std::sort(en.begin(), en.end());
    std::vector<uint8_t> active(c, 0);
    std::priority_queue<uint32_t, std::vector<uint32_t>, std::greater<uint32_t>> heap;
    size_t ie = 0, in = 0;
    for (uint32_t p : pts) {
        while (in < en.size() && en[in].first == p) active[en[in++].second] = 0;
        while (ie < ev.size() && ev[ie].first == p) {
            active[ev[ie].second] = 1;
            heap.push(ev[ie++].second);
        }
        while (!heap.empty() && !active[heap.top()]) heap.pop();
        uint32_t r = heap.empty() ? 0u : (uint32_t)(recs[heap.top()] >> 32);
        if (res.empty() || res.back() != r) {
            starts.push_back(p);
            res.push_back(r);
        }
    }
}

// Per-class first-match records of one 100-slot rule list (kernel.c:222-258 / :306-340).
static void class_records(const uint8_t *val, std::vector<uint64_t> per[INFW_NCLS]) {
    for (int i = 0; i < INFW_MAX_RULES_PER_TARGET; i++) {
        const uint8_t *r = val + 12 * i;
        uint32_t rule_id = rd_le32(r);
        uint8_t proto = r[4];
        uint16_t ps = (uint16_t)(r[5] | r[6] << 8), pe = (uint16_t)(r[7] | r[8] << 8);
        uint8_t it = r[9], ic = r[10], action = r[11];
        if (rule_id == INFW_INVALID_RULE_ID) continue;
        uint64_t res = (uint64_t)INFW_RESULT(action, rule_id) << 32;
        auto rec = [&](uint32_t lo, uint32_t hi) { return (uint64_t)lo | (uint64_t)hi << 16 | res; };
        switch (proto) {
        case 0:
            for (int c = 0; c < INFW_NCLS; c++) per[c].push_back(rec(0, 0xFFFF));
            break;
        case 6:
        case 17:
        case 132: {
            int c = proto == 6 ? INFW_CLS_TCP : proto == 17 ? INFW_CLS_UDP : INFW_CLS_SCTP;
            if (pe == 0) per[c].push_back(rec(ps, ps));
            else if (ps < pe) per[c].push_back(rec(ps, (uint32_t)pe - 1));
            break;
        }
        case 1: {
            uint32_t v = (uint32_t)it << 8 | ic;
            per[INFW_CLS_ICMP4].push_back(rec(v, v));
            break;
        }
        case 58: {
            uint32_t v = (uint32_t)it << 8 | ic;
            per[INFW_CLS_ICMP6].push_back(rec(v, v));
            break;
        }
        default:
            break;
        }
    }
}

// Value parts per (list, class): the fewest (1, 2, 4, 8 or 16; as log2) for which at most
// 1/256 of the (list, class, part) lines need a root + leaf, i.e. a second dependent table
// line.  Fewer parts = fewer entry lines = more of them resident in L2: a rule set of short
// lists (configs[1]: 10 rules) fits one line per (list, class) — 1/16 of the footprint —
// while 99-rule lists (configs[2]) need 16 parts to stay at one line per packet.
static uint32_t choose_dt_plog2(const std::vector<const uint8_t *> &vals, const Options &opt) {
    const int nt = compile_threads(vals.size(), opt.compile_threads);
    std::vector<std::array<uint64_t, 10>> acc(nt);  // per thread: lines[5], over[5]
    parallel_chunks(vals.size(), nt, [&](int t, size_t a, size_t b) {
        uint64_t *lines = acc[t].data(), *over = lines + 5;
        std::fill(lines, lines + 10, 0ull);
        std::vector<uint64_t> per[INFW_NCLS];
        std::vector<uint32_t> starts, res;
        for (size_t x = a; x < b; x++) {
            for (auto &p : per) p.clear();
            class_records(vals[x], per);
            for (int c = 0; c < INFW_NCLS; c++) {
                step_function(per[c], starts, res);
                bool compact = true;
                for (uint32_t r : res) compact = compact && infw_dt_result_code(r) <= 0xFFu;
                const uint32_t segs = compact ? INFW_DT_CLEAF_SEGS : INFW_DT_LEAF_SEGS;
                for (uint32_t pl = 0; pl <= 4; pl++) {
                    const uint32_t span = 65536u >> pl;
                    uint32_t q = 0, nseg = 1;  // segments of part q: 1 + starts strictly inside it
                    for (size_t k = 1; k < starts.size(); k++) {
                        while (starts[k] >= (q + 1) * span) {
                            over[pl] += nseg > segs;
                            nseg = 1;
                            q++;
                        }
                        nseg += starts[k] > q * span;
                    }
                    for (; q < (1u << pl); q++, nseg = 1) over[pl] += nseg > segs;
                    lines[pl] += 1u << pl;
                }
            }
        }
    });
    uint64_t lines[5] = {}, over[5] = {};
    for (const auto &a : acc)
        for (int pl = 0; pl < 5; pl++) {
            lines[pl] += a[pl];
            over[pl] += a[5 + pl];
        }
    if (opt.trace & 1)
        for (uint32_t pl = 0; pl <= 4; pl++)
            fprintf(stderr, "[compile] %u parts: %llu (list, class, part) lines, %llu need a root + leaf\n", 1u << pl,
                    (unsigned long long)lines[pl], (unsigned long long)over[pl]);
    for (uint32_t pl = 0; pl < 4; pl++)
        if (over[pl] * 256 <= lines[pl]) return pl;
    return 4;
}

// Does every one of the 2^p parts of a step function fit one decision line (no root)?  Mirrors
// emit_decision_lines' forms: a compact leaf holds 20 segments when all of the part's results have a code.
static bool parts_fit_one_line(const std::vector<uint32_t> &starts, const std::vector<uint32_t> &res, uint32_t p) {
    const uint32_t span = 65536u >> p;
    size_t j = 0;
    for (uint32_t q = 0; q < (1u << p); q++) {
        const uint32_t lo = q * span, hi = lo + span;
        while (j + 1 < starts.size() && starts[j + 1] <= lo) j++;
        uint32_t S = 1;
        bool compact = infw_dt_result_code(res[j]) <= 0xFFu;
        for (size_t k = j + 1; k < starts.size() && starts[k] < hi; k++) {
            S++;
            compact = compact && infw_dt_result_code(res[k]) <= 0xFFu;
        }
        if (S > (compact ? INFW_DT_CLEAF_SEGS : INFW_DT_LEAF_SEGS)) return false;
    }
    return true;
}

// pl_out (per-list part counts, infw_tables.h): each class is cut into the fewest 2^p <= 2^plog2 parts that fit
// one line each, written at the start of its 2^plog2-line region; *pl_out gets p in bits [3c, 3c + 3).
int compile_rule_list(const uint8_t *val, std::vector<uint64_t> &rules,
                      uint64_t desc_out[INFW_DESC_STRIDE], infw_dt_line *entry_out,
                      std::vector<infw_dt_line> &leaves, uint32_t plog2, uint32_t *pl_out) {
    int rc = 0;
    std::vector<uint64_t> per[INFW_NCLS];
    class_records(val, per);
    uint32_t pl = 0;
    std::vector<uint32_t> st, rs;
    for (int c = 0; c < INFW_DESC_STRIDE; c++) {
        uint32_t p = plog2;
        if (c < INFW_NCLS && pl_out) {
            step_function(per[c], st, rs);
            for (uint32_t q = 0; q < plog2; q++)
                if (parts_fit_one_line(st, rs, q)) {
                    p = q;
                    break;
                }
            pl |= p << (3 * c);
        }
        if (c < INFW_NCLS && !rc) rc = build_decision_table(per[c], &entry_out[(size_t)c << plog2], leaves, p);
        if (c >= INFW_NCLS || per[c].empty()) {
            desc_out[c] = 0;
            continue;
        }
        uint64_t off = rules.size();
        rules.insert(rules.end(), per[c].begin(), per[c].end());
        desc_out[c] = off | (uint64_t)per[c].size() << 32;
    }
    if (pl_out) *pl_out = pl;
    return rc;
}

// ------------------------------------------------------------------------
// Host open-addressed table for long-prefix nodes while compiling.
// ------------------------------------------------------------------------
namespace {
struct LongNode {
    uint64_t hi, lo;
    uint32_t tag;
    uint32_t real;  // list+1 of a real prefix at exactly this node, 0 = marker only
};
struct LongSet {
    std::vector<LongNode> tab;
    uint64_t mask = 0, n = 0;
    void init(uint64_t expect) {
        uint64_t cap = 1024;
        while (cap < expect * 2) cap <<= 1;
        tab.assign(cap, LongNode{0, 0, 0, 0});
        mask = cap - 1;
        n = 0;
    }
    LongNode *find_or_insert(uint32_t tag, uint64_t hi, uint64_t lo) {
        uint64_t i = infw_long_hash(tag, hi, lo) & mask;
        for (;;) {
            LongNode &e = tab[i];
            if (e.tag == 0) {
                e.tag = tag; e.hi = hi; e.lo = lo; e.real = 0;
                n++;
                return &e;
            }
            if (e.tag == tag && e.hi == hi && e.lo == lo) return &e;
            i = (i + 1) & mask;
        }
    }
    const LongNode *find(uint32_t tag, uint64_t hi, uint64_t lo) const {
        uint64_t i = infw_long_hash(tag, hi, lo) & mask;
        for (;;) {
            const LongNode &e = tab[i];
            if (e.tag == 0) return nullptr;
            if (e.tag == tag && e.hi == hi && e.lo == lo) return &e;
            i = (i + 1) & mask;
        }
    }
};
struct ShortEnt {
    uint32_t slot, a32, plen, list1;
};
}  // namespace

// Capacity for n elements plus the 25 % slack incremental commits append into (compile_tables' inc
// path), reserved before the buffer is filled so that growing it later needs no copy.
template <class V>
static void reserve_slack(V &v, size_t n, bool inc) {
    v.reserve(inc ? n + std::max<size_t>(n / 4, 4096) : n);
}

int compile_tables(const PendingMap &m, HostTables &out, const Options &opt, IncState *inc) {
    // Options::trace & 1: wall time per phase on stderr
    const bool trace = (opt.trace & 1) != 0;
    auto tp = std::chrono::steady_clock::now();
    auto phase = [&](const char *what) {
        if (!trace) return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[compile] %-14s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(now - tp).count());
        tp = now;
    };
    out = HostTables();
    // --- slots: distinct ifindexes, ascending
    std::vector<uint32_t> ifs;
    ifs.reserve(64);
    {
        std::unordered_map<uint32_t, int> seen;
        m.nodes.for_each_live([&](const MapNode &n) {
            if (n.key.plen < 32) return;  // a partial-ifindex prefix names no interface (below)
            uint32_t ifx = rd_le32(n.key.md);
            if (seen.emplace(ifx, 0).second) ifs.push_back(ifx);
        });
        std::sort(ifs.begin(), ifs.end());
    }
    out.n_slots = (uint32_t)ifs.size();
    if (out.n_slots >= (1u << 23)) {
        set_error("compile: too many ifindexes");
        return -ENOSPC;
    }
    std::unordered_map<uint32_t, uint32_t> slot_of;
    for (uint32_t s = 0; s < out.n_slots; s++) slot_of[ifs[s]] = s;
    {
        uint32_t cap = 16;
        while (cap < 2 * out.n_slots) cap <<= 1;
        // a collision-free multiplier when one exists for up to 256 entries: ifindex i sits at
        // (i * if_mult) >> if_shift, so the kernel resolves an ifindex with one LDS probe and no loop
        // (infw_if_slot); otherwise open addressing from infw_if_hash
        out.if_mult = 0;
        out.if_shift = 0;
        for (uint32_t c = cap; c <= 256 && !out.if_mult; c <<= 1) {
            int lg = 0;
            while ((1u << lg) < c) lg++;
            for (uint32_t k = 0; k < 256 && !out.if_mult; k++) {
                const uint32_t m = (0x9E3779B1u + k * 0x6A09E668u) | 1u;
                std::vector<uint8_t> used(c, 0);
                bool ok = true;
                for (uint32_t s = 0; s < out.n_slots && ok; s++) {
                    const uint32_t h = (ifs[s] * m) >> (32 - lg);
                    ok = !used[h];
                    used[h] = 1;
                }
                if (ok) {
                    out.if_mult = m;
                    out.if_shift = 32 - lg;
                    cap = c;
                }
            }
        }
        out.if_keys.assign(cap, 0);
        out.if_slot.assign(cap, INFW_IF_EMPTY);
        for (uint32_t s = 0; s < out.n_slots; s++) {
            uint32_t h;
            if (out.if_mult) {
                h = (ifs[s] * out.if_mult) >> out.if_shift;
            } else {
                h = infw_if_hash(ifs[s]) & (cap - 1);
                while (out.if_slot[h] != INFW_IF_EMPTY) h = (h + 1) & (cap - 1);
            }
            out.if_keys[h] = ifs[s];
            out.if_slot[h] = s;
        }
    }

    // --- rule lists: one per distinct referenced value
    std::unordered_map<uint32_t, uint32_t> list_of_vid;
    m.nodes.for_each_live([&](const MapNode &n) {
        const uint32_t vid = n.val.vid;
        if (list_of_vid.count(vid)) return;
        uint32_t lid = (uint32_t)list_of_vid.size();
        list_of_vid[vid] = lid;
    });
    out.n_lists = (uint32_t)list_of_vid.size();
    phase("slots+lists");
    reserve_slack(out.desc, (size_t)std::max<uint32_t>(out.n_lists, 1) * INFW_DESC_STRIDE, inc);
    out.desc.assign((size_t)std::max<uint32_t>(out.n_lists, 1) * INFW_DESC_STRIDE, 0);
    // value parts per (list, class): the fewest that keep one table line per packet (choose_dt_plog2),
    // within a budget for the entry lines of one image — 2 GiB by default (INFW_DT_BUDGET_MB).  At 1M
    // distinct 99-rule lists 16 parts take 7.2 GB per image; with the keys loaded in random order (the
    // reference loader's Go map order) the hot lists' lines spread over all of it and every dependent
    // decision-line read pays for the span: 4 parts (1.8 GB, a leaf line for busy parts) 3.75 ms against
    // 5.03 at 16 (profiles/r03r; round 2's 16-part choice, profiles/r02b, was measured with the keys in
    // popularity order, where the hot lists sit together); the option dt_parts = 1|2|4|8|16 forces one form
    {
        std::vector<const uint8_t *> vals;
        vals.reserve(list_of_vid.size());
        for (const auto &p : list_of_vid) vals.push_back(m.pool.vals[p.first].data());
        out.dt_plog2 = choose_dt_plog2(vals, opt);
        const uint64_t budget = (uint64_t)opt.dt_budget_mb << 20;
        while (out.dt_plog2 && ((uint64_t)out.n_lists * INFW_NCLS * sizeof(infw_dt_line) << out.dt_plog2) > budget)
            out.dt_plog2--;
    }
    phase("choose parts");
    if (opt.dt_parts) {
        const int v = opt.dt_parts;
        out.dt_plog2 = v == 16 ? 4 : v == 8 ? 3 : v == 4 ? 2 : v == 2 ? 1 : v == 1 ? 0 : out.dt_plog2;
    }
    reserve_slack(out.dte, ((size_t)std::max<uint32_t>(out.n_lists, 1) * INFW_NCLS) << out.dt_plog2, inc);
    out.dte.assign(((size_t)std::max<uint32_t>(out.n_lists, 1) * INFW_NCLS) << out.dt_plog2, infw_dt_line{});
    out.dtl.clear();
    int dt_rc = 0;
    {
        // lists in id order, compiled in contiguous id ranges per thread into thread-local rule and leaf
        // pools; the pools are then concatenated and the chunk's offsets (class-list descriptors, root
        // entries' leaf index) rebased — the image is identical to a serial compile
        std::vector<uint32_t> vid_of_lid(out.n_lists);
        for (const auto &p : list_of_vid) vid_of_lid[p.second] = p.first;
        const int nt = compile_threads(out.n_lists, opt.compile_threads);
        std::vector<std::vector<uint64_t>> rules_t(nt);
        std::vector<std::vector<infw_dt_line>> leaves_t(nt);
        std::vector<int> rc_t(nt, 0);
        std::vector<std::pair<size_t, size_t>> range_t(nt);
        const size_t ents = (size_t)INFW_NCLS << out.dt_plog2;
        // per-list part counts when the list count fits the kernel's LDS copy (Options::dt_adapt 0 turns them off)
        const bool adapt = out.dt_plog2 > 0 && out.n_lists <= INFW_DT_PL_LISTS && opt.dt_adapt != 0;
        out.dt_pl.assign(adapt ? INFW_DT_PL_LISTS : 0, 0u);
        parallel_chunks(out.n_lists, nt, [&](int t, size_t a, size_t b) {
            range_t[t] = {a, b};
            for (size_t lid = a; lid < b && !rc_t[t]; lid++)
                rc_t[t] = compile_rule_list(m.pool.vals[vid_of_lid[lid]].data(), rules_t[t],
                                            &out.desc[lid * INFW_DESC_STRIDE], &out.dte[lid * ents], leaves_t[t],
                                            out.dt_plog2, adapt ? &out.dt_pl[lid] : nullptr);
        });
        size_t rbase = 0, lbase = 0;
        for (int t = 0; t < nt && !dt_rc; t++) {
            dt_rc = rc_t[t];
            if (lbase + leaves_t[t].size() > INFW_DT_INDEX) dt_rc = -ENOSPC;
            if (dt_rc) break;
            if (t > 0)
                for (size_t lid = range_t[t].first; lid < range_t[t].second; lid++) {
                    for (int c = 0; c < INFW_DESC_STRIDE; c++) {
                        uint64_t &d = out.desc[lid * INFW_DESC_STRIDE + c];
                        if (d) d += rbase;  // off in the low 32 bits, cnt above
                    }
                    for (size_t e = lid * ents; e < (lid + 1) * ents; e++)
                        if (out.dte[e].w[0] & INFW_DT_ROOT)
                            out.dte[e].w[0] = INFW_DT_ROOT | (uint32_t)((out.dte[e].w[0] & INFW_DT_INDEX) + lbase);
                }
            rbase += rules_t[t].size();
            lbase += leaves_t[t].size();
        }
        if (!dt_rc) {
            if (rbase >= (1ull << 32)) dt_rc = -ENOSPC;
            reserve_slack(out.rules, std::max<size_t>(rbase, 1), inc);
            reserve_slack(out.dtl, std::max<size_t>(lbase, 1), inc);
            for (int t = 0; t < nt; t++) {
                out.rules.insert(out.rules.end(), rules_t[t].begin(), rules_t[t].end());
                std::vector<uint64_t>().swap(rules_t[t]);
                out.dtl.insert(out.dtl.end(), leaves_t[t].begin(), leaves_t[t].end());
                std::vector<infw_dt_line>().swap(leaves_t[t]);
            }
        }
    }
    phase("rule lists");
    if (dt_rc) {
        set_error("compile: decision-table leaf pool exceeds 2^31 lines");
        return -ENOSPC;
    }
    if (out.rules.empty()) out.rules.push_back(0);
    if (out.dtl.empty()) out.dtl.push_back(infw_dt_line{});

    // --- split entries
    std::vector<ShortEnt> shorts;
    struct LongReal {
        uint32_t slot, len, list1;
        uint64_t hi, lo;
    };
    std::vector<LongReal> longs;
    shorts.reserve(m.nodes.size());
    // Entries shorter than the ifindex (prefixLen < 32: its first bits, in key byte order — the ifindex's
    // little-endian bytes — BuildEBPFKey never writes one, loader.go:543) cover every interface whose ifindex
    // bytes start that way, with any address, below every entry of the interface itself.  The longest one
    // covering an interface with entries becomes that slot's default answer (the short table's words start
    // from it instead of 0); an ifindex with no entries of its own takes the list of partial prefixes
    // (infw_wild_lookup), longest first.
    out.wild.clear();
    m.nodes.for_each_live([&](const MapNode &n) {
        if (n.key.plen < 32) {
            const uint8_t *d = n.key.md;  // masked to plen bits
            const uint32_t key = (uint32_t)d[0] << 24 | (uint32_t)d[1] << 16 | (uint32_t)d[2] << 8 | d[3];
            out.wild.push_back(n.key.plen);
            out.wild.push_back(key);
            out.wild.push_back(list_of_vid[n.val.vid] + 1);
        }
    });
    {
        std::vector<std::array<uint32_t, 3>> w;
        for (size_t i = 0; i < out.wild.size(); i += 3) w.push_back({out.wild[i], out.wild[i + 1], out.wild[i + 2]});
        std::sort(w.begin(), w.end(), [](const std::array<uint32_t, 3> &a, const std::array<uint32_t, 3> &b) {
            return a[0] != b[0] ? a[0] > b[0] : a[1] < b[1];
        });
        out.wild.clear();
        for (const auto &e : w) out.wild.insert(out.wild.end(), e.begin(), e.end());
    }
    out.n_wild = (uint32_t)(out.wild.size() / 3);
    if (out.wild.empty()) out.wild.assign(3, 0u);  // never an empty device buffer
    std::vector<uint32_t> slot_default(out.n_slots, 0);
    for (uint32_t sl = 0; sl < out.n_slots; sl++) slot_default[sl] = infw_wild_match(out.wild.data(), out.n_wild, ifs[sl]);
    m.nodes.for_each_live([&](const MapNode &n) {
        const NodeKey &k = n.key;
        if (k.plen < 32) return;
        uint32_t slot = slot_of[rd_le32(k.md)];
        uint32_t P = k.plen - 32;
        uint32_t list1 = list_of_vid[n.val.vid] + 1;
        const uint8_t *ip = k.md + 4;  // already masked to P bits
        if (P <= 32) {
            uint32_t a32 = (uint32_t)ip[0] << 24 | (uint32_t)ip[1] << 16 | (uint32_t)ip[2] << 8 | ip[3];
            shorts.push_back(ShortEnt{slot, a32, P, list1});
        } else {
            uint64_t hi = 0, lo = 0;
            for (int i = 0; i < 8; i++) hi = hi << 8 | ip[i];
            for (int i = 8; i < 16; i++) lo = lo << 8 | ip[i];
            longs.push_back(LongReal{slot, P, list1, hi, lo});
        }
    });
    out.n_entries = m.nodes.size();
    phase("split");

    // --- short table: per slot, a DIR-24-8 build image (shorter prefixes written
    // first, longer ones overwrite; /25-/32 in 256-entry tbl8 groups) compressed
    // into l16 words + 64-B run-bitmap nodes (infw_tables.h)
    std::sort(shorts.begin(), shorts.end(), [](const ShortEnt &a, const ShortEnt &b) {
        return a.slot != b.slot ? a.slot < b.slot : a.plen < b.plen;
    });
    // DIR-24-8 (128 MiB of words per ifindex) while the ifindexes' words fit 4 GiB, else the compressed form
    out.short_mode = opt.short_table == 1 ? INFW_SHORT_COMPRESSED
                     : opt.short_table == 0 || ((uint64_t)out.n_slots << 27) <= (4ull << 30) ? INFW_SHORT_DIR24
                                                                                          : INFW_SHORT_COMPRESSED;
    const bool dir24 = out.short_mode == INFW_SHORT_DIR24;
    out.l16.assign(dir24 ? 1 : (size_t)std::max<uint32_t>(out.n_slots, 1) << 16, 0u);
    {
        std::vector<uint32_t> t24, t8;
        // node for 256 values; returns the word for the parent (plain value or node ref)
        auto make_node = [&](const uint32_t *vals) -> uint32_t {
            bool uniform = true;
            for (int i = 1; i < 256 && uniform; i++) uniform = vals[i] == vals[0];
            if (uniform) return vals[0];
            infw_bnode n;
            memset(&n, 0, sizeof(n));
            std::vector<uint32_t> runs;
            for (int i = 0; i < 256; i++)
                if (i == 0 || vals[i] != vals[i - 1]) {
                    n.bm[i >> 5] |= 1u << (i & 31);
                    runs.push_back(vals[i]);
                }
            n.nv = (uint32_t)runs.size();
            if (n.nv <= INFW_NODE_INLINE) {
                for (uint32_t k = 0; k < n.nv; k++) n.v[k] = runs[k];
            } else {
                n.base = (uint32_t)out.vpool.size();
                out.vpool.insert(out.vpool.end(), runs.begin(), runs.end());
            }
            out.nodes.push_back(n);
            return INFW_NODE_FLAG | (uint32_t)(out.nodes.size() - 1);
        };
        size_t si = 0;
        for (uint32_t slot = 0; slot < out.n_slots; slot++) {
            size_t sj = si;
            while (sj < shorts.size() && shorts[sj].slot == slot) sj++;
            if (sj == si && !slot_default[slot]) continue;
            t24.assign((size_t)1 << 24, slot_default[slot]);
            t8.clear();
            for (size_t x = si; x < sj; x++) {
                const ShortEnt &e = shorts[x];
                if (e.plen <= 24) {
                    uint32_t start = e.a32 >> 8, cnt = 1u << (24 - e.plen);
                    std::fill(t24.begin() + start, t24.begin() + start + cnt, e.list1);
                } else {
                    uint32_t i24 = e.a32 >> 8, w = t24[i24], g;
                    if (w & INFW_TBL8_FLAG) {
                        g = w & ~INFW_TBL8_FLAG;
                    } else {
                        g = (uint32_t)(t8.size() >> 8);
                        t8.resize(t8.size() + 256, w);
                        t24[i24] = INFW_TBL8_FLAG | g;
                    }
                    uint32_t start = e.a32 & 0xFFu, cnt = 1u << (32 - e.plen);
                    std::fill(t8.begin() + ((size_t)g << 8) + start, t8.begin() + ((size_t)g << 8) + start + cnt,
                              e.list1);
                }
            }
            out.n_tbl8_groups += t8.size() >> 8;
            if (dir24) {  // keep the DIR-24-8 image as the device form
                if (out.tbl24.empty()) out.tbl24.assign((size_t)out.n_slots << 24, 0ull);
                const uint32_t gbase = (uint32_t)(out.tbl8.size() >> 8);
                for (size_t k = 0; k < ((size_t)1 << 24); k++) {
                    const uint32_t w = t24[k];
                    if (w & INFW_TBL8_FLAG) {
                        const uint32_t lg = w & ~INFW_TBL8_FLAG;
                        out.tbl24[((size_t)slot << 24) + k] = infw_d24_encode(&t8[(size_t)lg << 8], gbase + lg);
                        out.tbl8_of[(uint64_t)slot << 24 | k] = gbase + lg;
                    } else {
                        out.tbl24[((size_t)slot << 24) + k] = w;
                    }
                }
                out.tbl8.insert(out.tbl8.end(), t8.begin(), t8.end());
                si = sj;
                continue;
            }
            uint32_t *l16 = &out.l16[(size_t)slot << 16];
            uint32_t vals[256];
            for (uint32_t b = 0; b < 65536; b++) {
                const uint32_t *blk = &t24[(size_t)b << 8];
                for (int i = 0; i < 256; i++) {
                    uint32_t w = blk[i];
                    vals[i] = (w & INFW_TBL8_FLAG) ? make_node(&t8[(size_t)(w & ~INFW_TBL8_FLAG) << 8]) : w;
                }
                l16[b] = make_node(vals);
                if (out.nodes.size() >= INFW_NODE_FLAG) {
                    set_error("compile: short-table nodes exhausted");
                    return -ENOSPC;
                }
            }
            si = sj;
        }
    }
    if (out.tbl24.empty()) {  // no <= /32 entry on any interface: nothing to index
        out.tbl24.push_back(0);
        if (out.short_mode == INFW_SHORT_DIR24) out.short_mode = INFW_SHORT_NONE;
    }
    {
        uint64_t n_wide = 0;  // <= /32 prefixes of /20 or shorter
        for (const ShortEnt &e : shorts) n_wide += e.plen <= 20;
        build_d16(out, shorts.size(), n_wide, opt.d16);
    }
    if (out.tbl8.empty()) out.tbl8.assign(256, 0);
    if (out.nodes.empty()) out.nodes.push_back(infw_bnode{});
    if (out.vpool.empty()) out.vpool.push_back(0);

    phase("short table");
    // --- long prefixes: levels, markers, best-matching-prefix
    {
        std::vector<uint8_t> lv;
        bool present[129] = {};
        for (const auto &r : longs) present[r.len] = true;
        for (int l = 33; l <= 128; l++)
            if (present[l]) lv.push_back((uint8_t)l);
        if (lv.size() > INFW_MAX_LEVELS) {
            set_error("compile: too many IPv6 prefix lengths");
            return -ENOSPC;
        }
        out.levels = lv;
        int nl = (int)lv.size();
        int level_idx[129];
        for (int i = 0; i < 129; i++) level_idx[i] = -1;
        for (int i = 0; i < nl; i++) level_idx[lv[i]] = i;

        LongSet set;
        set.init(longs.size() * 6 + 16);
        for (const auto &r : longs) {
            int t = level_idx[r.len];
            int L = 0, R = nl - 1;
            while (L <= R) {
                int mid = (L + R) >> 1;
                uint32_t len = lv[mid];
                uint64_t h = r.hi, l = r.lo;
                infw_mask128(len, &h, &l);
                LongNode *n = set.find_or_insert(r.slot << 8 | len, h, l);
                if (mid == t) {
                    n->real = r.list1;
                    break;
                }
                if (mid < t) L = mid + 1;  // marker on the way to a longer level
                else R = mid - 1;
            }
        }
        // bmp: a real node is its own answer; a marker takes the longest real
        // prefix (of a level below it) covering its bits.
        uint64_t cap = 1024;
        while (cap < set.n * 2) cap <<= 1;
        out.ltab.assign(cap, infw_long_entry{0, 0, 0, 0, {0, 0}});
        uint64_t lmask = cap - 1;
        for (const LongNode &n : set.tab) {
            if (n.tag == 0) continue;
            uint32_t bmp = n.real;
            if (!bmp) {
                uint32_t slot = n.tag >> 8, len = n.tag & 0xFF;
                for (int i = level_idx[len] - 1; i >= 0 && !bmp; i--) {
                    uint64_t h = n.hi, l = n.lo;
                    infw_mask128(lv[i], &h, &l);
                    const LongNode *p = set.find(slot << 8 | lv[i], h, l);
                    if (p && p->real) bmp = p->real;
                }
            }
            uint64_t i = infw_long_hash(n.tag, n.hi, n.lo) & lmask;
            while (out.ltab[i].tag) i = (i + 1) & lmask;
            out.ltab[i] = infw_long_entry{n.hi, n.lo, n.tag, bmp, {0, 0}};
        }
        out.n_long_entries = set.n;
    }

    phase("long table");
    // --- /32-grouped buckets for IPv6 long prefixes (the fast path)
    {
        struct G {
            uint32_t slot, top;
            std::vector<infw_v6_rec> recs;
        };
        std::unordered_map<uint64_t, G> groups;
        for (const auto &r : longs) {
            uint32_t top = (uint32_t)(r.hi >> 32);
            G &g = groups[(uint64_t)r.slot << 32 | top];
            g.slot = r.slot;
            g.top = top;
            if (r.list1 >= (1u << 25)) {
                set_error("compile: more than 2^25-1 rule lists");
                return -ENOSPC;
            }
            g.recs.push_back(infw_v6_rec{r.lo, (uint32_t)r.hi, (r.len - 32) << 25 | r.list1});
        }
        // a wave waits for its slowest lane's probe chain: keep the load at or below 1/8 (the untouched capacity
        // costs no cache)
        const uint64_t spread = 8;
        uint64_t cap = 1024;
        while (cap < groups.size() * spread) cap <<= 1;
        out.btab.assign(cap, infw_v6_bucket{});
        memset(out.btab.data(), 0, cap * sizeof(infw_v6_bucket));
        const uint64_t bmask = cap - 1;
        for (auto &kv : groups) {
            G &g = kv.second;
            uint64_t i = infw_bucket_hash(g.slot, g.top) & bmask;
            while (out.btab[i].tag) i = (i + 1) & bmask;
            infw_v6_bucket &b = out.btab[i];
            b.tag = g.slot + 1;
            b.top = g.top;
            if (g.recs.size() > INFW_BUCKET_INLINE) {
                b.n = INFW_BUCKET_OVERFLOW;
                out.n_overflow_groups++;
            } else {
                // longest first: the first covering record is the longest match
                std::sort(g.recs.begin(), g.recs.end(),
                          [](const infw_v6_rec &a, const infw_v6_rec &c) { return a.meta > c.meta; });
                b.n = (uint32_t)g.recs.size();
                for (size_t k = 0; k < g.recs.size(); k++) b.rec[k] = g.recs[k];
            }
        }
        out.n_buckets = groups.size();
    }
    phase("buckets");
    out.dt_short_lines = count_dt_short_lines(out);
    out.dt_half = choose_dt_half(out, opt.dt_half);
    if (inc) {
        // the buffers incremental commits append to get the device images' 25 % slack on the host too, so
        // the first commits after a compile do not copy a 30-MB vector to grow it by one rule list
        // (touched once here: a first write into fresh pages can stall for milliseconds in the kernel's
        // huge-page allocation, which would land on a commit)
        auto slack = [](auto &v) {
            const size_t n = v.size();
            v.resize(n + std::max<size_t>(n / 4, 4096));
            v.resize(n);
        };
        slack(out.tbl8);
        slack(out.desc);
        slack(out.rules);
        slack(out.dte);
        slack(out.dtl);
        *inc = IncState();
        inc->slot_of = std::move(slot_of);
        inc->list_refs.assign(out.n_lists, 0);
        m.nodes.for_each_live([&](const MapNode &n) { inc->list_refs[list_of_vid[n.val.vid]]++; });
        inc->list_of_vid = std::move(list_of_vid);
        inc->valid = true;
    }
    phase("slack+inc");
    return 0;
}

uint32_t choose_dt_half(const HostTables &h, int req) {
    // the kernel's decision-line reads (infw_dev_tables.dt_half): the first 32 B, then the second half only where
    // needed, when nearly every entry line is a compact leaf of <= 9 segments (answered by its first half: configs[1],
    // same-box A/B 1.107 -> 1.020 ms); else the whole line at once (a wave waits for the dependent second half
    // whenever one of its lanes needs it: configs[2] and [4] 0.2-0.5 % slower reading halves, profiles/r04hf)
    if (req >= 0) return req ? 1u : 0u;
    return !h.dte.empty() && h.dt_short_lines * 100 >= (uint64_t)h.dte.size() * 95 ? 1u : 0u;
}

uint64_t count_dt_short_lines(const HostTables &h) {
    uint64_t n = 0;
    for (const infw_dt_line &l : h.dte) n += infw_dt_line_short(l);
    return n;
}

uint64_t d16_word(const HostTables &h, uint32_t slot, uint32_t hi, uint32_t *runs) {
    const uint64_t *w = &h.tbl24[((size_t)slot << 24) | (size_t)hi << 8];
    uint32_t v[3] = {0, 0, 0}, st[3] = {0, 0, 0}, nr = 0;
    bool fits = true;
    auto push = [&](uint32_t start, uint32_t val) {
        if (nr && v[nr - 1] == val) return;
        if (nr == 3) {
            fits = false;
            return;
        }
        st[nr] = start;
        v[nr++] = val;
    };
    for (uint32_t i = 0; i < 256 && fits; i++) {
        const uint64_t e = w[i];
        if (!(e & INFW_D24_GROUP)) {
            push(i << 8, (uint32_t)e);
        } else if (e & INFW_D24_INLINE) {  // the word's runs start at 0 and at its (at most two) boundaries
            const uint32_t b1 = (e & INFW_D24_ABA) ? (uint32_t)(e >> 44) & 0xFFu : (uint32_t)(e >> 45) & 0xFFu;
            const uint32_t b2 = (e & INFW_D24_ABA) ? (uint32_t)(e >> 52) & 0x1FFu : (uint32_t)(e >> 53) & 0xFFu;
            push(i << 8, infw_d24_inline(e, 0));
            if (b1 < 256) push(i << 8 | b1, infw_d24_inline(e, b1));
            if (b2 < 256) push(i << 8 | b2, infw_d24_inline(e, b2));
        } else {
            const uint32_t *g = &h.tbl8[(size_t)(uint32_t)e << 8];
            for (uint32_t x = 0; x < 256 && fits; x++) push(i << 8 | x, g[x]);
        }
    }
    if (runs) *runs = fits ? nr : 4u;
    if (!fits || v[0] > 0x7FFFu || v[1] > 0x7FFFu || (nr == 3 && v[2] != v[0])) return 0;
    if (nr == 1) return infw_d16_encode(v[0], v[0], 0, 0xFFFFu);
    return infw_d16_encode(v[0], v[1], st[1], nr == 3 ? st[2] - 1 : 0xFFFFu);
}

void build_d16(HostTables &h, uint64_t n_short, uint64_t n_short_wide, int req) {
    h.d16_on = 0;
    h.d16_permille = 0;
    h.d16.clear();
    if (h.short_mode == INFW_SHORT_DIR24 && h.tbl24.size() == ((size_t)h.n_slots << 24) && h.n_slots && req != 0) {
        std::vector<uint64_t> d((size_t)h.n_slots << 16);
        std::vector<uint64_t> cnt(2 * (size_t)h.n_slots, 0);  // per slot: /16s with structure, of them inline
        auto one = [&](uint32_t s) {
            for (uint32_t b = 0; b < 65536; b++) {
                uint32_t nr = 0;
                const uint64_t w = d16_word(h, s, b, &nr);
                d[((size_t)s << 16) | b] = w;
                cnt[2 * s] += nr > 1;
                cnt[2 * s + 1] += nr > 1 && w;
            }
        };
        const uint32_t nt = std::min<uint32_t>(h.n_slots, 16);
        std::vector<std::thread> th;
        for (uint32_t t = 1; t < nt; t++)
            th.emplace_back([&, t] {
                for (uint32_t s = t; s < h.n_slots; s += nt) one(s);
            });
        for (uint32_t s = 0; s < h.n_slots; s += nt) one(s);
        for (auto &x : th) x.join();
        uint64_t structured = 0, inl = 0;
        for (uint32_t s = 0; s < h.n_slots; s++) {
            structured += cnt[2 * s];
            inl += cnt[2 * s + 1];
        }
        h.d16_permille = structured ? (uint32_t)(inl * 1000 / structured) : 1000u;
        // Worth a word in front of DIR-24-8 when almost every /16 with structure inside is answered by it (a lookup
        // that falls through reads both: one more dependent L2 round trip) and prefixes of /20 or shorter — spread
        // over 2..16 lines of DIR-24-8 words each, where the /16 word is one — are common.  Measured on MI355X
        // (profiles/r03j, r03l): configs[1] (927 permille, 29 % of prefixes <= /20) +13 %, configs[4] (928, 33 %)
        // +10 %; configs[2]-shaped tables (BGP-like, 12 % <= /20) -2..-5 % at 100k / 300k prefixes (891 / 698
        // permille) and -9 % at 1M (262); configs[4] at 1M (451) even.
        const bool wide = n_short && n_short_wide * 5 >= n_short;
        if (req == 1 || (h.d16_permille >= 800 && wide)) {
            h.d16 = std::move(d);
            h.d16_on = 1;
        }
    }
    if (h.d16.empty()) h.d16.push_back(0);
}

void host_buffer(const HostTables &h, int b, const void **p, size_t *bytes) {
#define INFW_HB(v) \
    *p = h.v.data(); \
    *bytes = h.v.size() * sizeof(h.v[0]); \
    break
    switch (b) {
    case TB_IFK: INFW_HB(if_keys);
    case TB_IFS: INFW_HB(if_slot);
    case TB_L16: INFW_HB(l16);
    case TB_NODES: INFW_HB(nodes);
    case TB_VPOOL: INFW_HB(vpool);
    case TB_TBL24: INFW_HB(tbl24);
    case TB_TBL8: INFW_HB(tbl8);
    case TB_LTAB: INFW_HB(ltab);
    case TB_BTAB: INFW_HB(btab);
    case TB_DESC: INFW_HB(desc);
    case TB_RULES: INFW_HB(rules);
    case TB_DTE: INFW_HB(dte);
    case TB_DTL: INFW_HB(dtl);
    case TB_LEVELS: INFW_HB(levels);
    case TB_WILD: INFW_HB(wild);
    case TB_DTPL: INFW_HB(dt_pl);
    case TB_D16: INFW_HB(d16);
    default:
        *p = nullptr;
        *bytes = 0;
    }
#undef INFW_HB
}

infw_dev_tables view_of(const HostTables &h, void *const buf[TB_COUNT]) {
    infw_dev_tables t;
    memset(&t, 0, sizeof(t));
    t.if_keys = static_cast<const uint32_t *>(buf[TB_IFK]);
    t.if_slot = static_cast<const uint32_t *>(buf[TB_IFS]);
    t.l16 = static_cast<const uint32_t *>(buf[TB_L16]);
    t.nodes = static_cast<const infw_bnode *>(buf[TB_NODES]);
    t.vpool = static_cast<const uint32_t *>(buf[TB_VPOOL]);
    t.tbl24 = static_cast<const uint64_t *>(buf[TB_TBL24]);
    t.tbl8 = static_cast<const uint32_t *>(buf[TB_TBL8]);
    t.ltab = static_cast<const infw_long_entry *>(buf[TB_LTAB]);
    t.btab = static_cast<const infw_v6_bucket *>(buf[TB_BTAB]);
    t.desc = static_cast<const uint64_t *>(buf[TB_DESC]);
    t.rules = static_cast<const uint64_t *>(buf[TB_RULES]);
    t.dte = static_cast<const infw_dt_line *>(buf[TB_DTE]);
    t.dtl = static_cast<const infw_dt_line *>(buf[TB_DTL]);
    t.levels = static_cast<const uint8_t *>(buf[TB_LEVELS]);
    t.wild = static_cast<const uint32_t *>(buf[TB_WILD]);
    t.dt_pl = static_cast<const uint32_t *>(buf[TB_DTPL]);
    t.d16 = static_cast<const uint64_t *>(buf[TB_D16]);
    t.n_wild = h.n_wild;
    t.lean = (h.short_mode == INFW_SHORT_DIR24 || h.short_mode == INFW_SHORT_NONE) && h.n_overflow_groups == 0 &&
             h.n_wild == 0;
    t.if_mask = (uint32_t)h.if_keys.size() - 1;
    t.if_mult = h.if_mult;
    t.if_shift = h.if_shift;
    t.n_slots = h.n_slots;
    t.short_mode = h.short_mode;
    t.lmask = h.ltab.size() - 1;
    t.bmask = h.btab.size() - 1;
    t.n_levels = (uint32_t)h.levels.size();
    t.dt_plog2 = h.dt_plog2;
    t.n_dt_pl = (uint32_t)h.dt_pl.size();
    t.d16_on = h.d16_on;
    t.dt_half = h.dt_half;
    t.n_dte = h.dte.size();
    t.stat_flush_tiles = 1024;
    return t;
}

infw_dev_tables HostTables::view() const {
    void *buf[TB_COUNT];
    for (int b = 0; b < TB_COUNT; b++) {
        const void *p;
        size_t bytes;
        host_buffer(*this, b, &p, &bytes);
        buf[b] = const_cast<void *>(p);
    }
    return view_of(*this, buf);
}

}  // namespace infw
