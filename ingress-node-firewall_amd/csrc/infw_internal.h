// infw_internal.h — host-side types of libinfw (not part of the C ABI).
#pragma once
#include <stdint.h>
#include <string.h>

#include <array>
#include <deque>
#include <memory>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/infw.h"
#include "infw_tables.h"

namespace infw {

void set_error(const std::string &msg);

// ------------------------------------------------------------------------
// Pending LPM map with the kernel LPM-trie semantics (kernel.c:50-57 map,
// kernel/bpf/lpm_trie.c).  A node is identified by (prefixLen, data masked
// to prefixLen); the stored data keeps the last writer's host bits, which
// get_next_key returns (trie_get_next_key copies node->data).
// ------------------------------------------------------------------------
struct NodeKey {
    uint32_t plen;
    uint8_t md[20];  // [ifindex LE][ip_data], masked to plen bits
    bool operator==(const NodeKey &o) const { return plen == o.plen && memcmp(md, o.md, 20) == 0; }
};
struct NodeKeyHash {
    size_t operator()(const NodeKey &k) const;
};
// Trie post-order: descendants before ancestors, 0-branch before 1-branch.
struct PostOrderLess {
    bool operator()(const NodeKey &a, const NodeKey &b) const;
};
struct NodeVal {
    uint8_t data[20];
    uint32_t vid;  // interned value id
};

// The entry set of a table image (image.cpp): interned values (1200 B each, in id order) and the nodes.
struct ImageEntries {
    std::vector<uint8_t> vals;
    std::vector<std::pair<NodeKey, NodeVal>> nodes;
};

struct ValuePool {
    std::deque<std::array<uint8_t, 1200>> vals;  // deque: growing never copies the values held
    std::unordered_multimap<uint64_t, uint32_t> index;
    uint32_t intern(const uint8_t *v);
    // intern() with a memo of the caller's value addresses: a batch update names the same few template values
    // call after call, and comparing one against the value its address had last time is far cheaper than
    // hashing it (a stale address whose bytes changed fails the compare and is interned afresh).
    uint32_t intern_at(const uint8_t *v);
    void clear();

  private:
    struct AddrMemo {
        const uint8_t *addr = nullptr;
        uint32_t vid = 0;
    };
    std::array<AddrMemo, 1024> memo_{};
};

// One entry of the pending map, 64 B (one host cache line): key, value, and the commit bookkeeping.
struct alignas(64) MapNode {
    NodeKey key;
    NodeVal val;
    int32_t was;     // while dirty: the committed value id (PendingMap::kAbsent: not in the committed set)
    uint32_t id;     // index in the node pool
    uint8_t live;    // in the map (0: removed since the last commit, kept until the commit as a tombstone)
    uint8_t dirty;   // listed in PendingMap::dirty_ids
    uint8_t pad[6];
};
static_assert(sizeof(MapNode) == 64, "MapNode is one cache line");

// The pending map's storage: nodes in a chunked pool (addresses never change, so the short-key lists and the
// dirty list can point at them) and an open-addressed index of 8-B slots ((hash >> 32) << 32 | id + 1, linear
// probing, backward-shift deletion, load <= 1/2).  A lookup is one index line and one node line, and both can
// be prefetched ahead of a batch of keys (prefetch_slot, then prefetch_node).
class NodeTable {
  public:
    static uint64_t hash(const NodeKey &k);
    size_t size() const { return n_live_; }
    bool empty() const { return n_live_ == 0; }
    // The indexed node of key k (live or a tombstone), or nullptr.
    MapNode *find(const NodeKey &k, uint64_t h) const;
    const MapNode *find_live(const NodeKey &k) const {
        const MapNode *n = find(k, hash(k));
        return n && n->live ? n : nullptr;
    }
    // A new indexed node for key k (absent), not yet live.
    MapNode *insert(const NodeKey &k, uint64_t h);
    // Unindex node n and return it to the pool.
    void erase(MapNode *n);
    void set_live(MapNode *n, bool live) {
        if (n->live != (uint8_t)live) n_live_ += live ? 1 : -1;
        n->live = live;
    }
    void prefetch_slot(uint64_t h) const { __builtin_prefetch(&slots_[(h >> 32) & mask_]); }
    void prefetch_node(const NodeKey &k, uint64_t h) const;
    MapNode &node(uint32_t id) { return chunks_[id >> kChunkLog][id & (kChunk - 1)]; }
    const MapNode &node(uint32_t id) const { return chunks_[id >> kChunkLog][id & (kChunk - 1)]; }
    template <class F>
    void for_each_live(F f) const {
        for (uint32_t id = 0; id < hw_; id++) {
            const MapNode &n = node(id);
            if (n.live) f(n);
        }
    }
    void reserve(size_t n);
    void clear();

  private:
    static constexpr uint32_t kChunkLog = 12, kChunk = 1u << kChunkLog;
    std::vector<uint64_t> slots_ = std::vector<uint64_t>(1024, 0);
    uint64_t mask_ = 1023;
    size_t n_indexed_ = 0, n_live_ = 0;
    std::vector<std::unique_ptr<MapNode[]>> chunks_;
    uint32_t hw_ = 0;
    std::vector<uint32_t> free_;
    void grow(size_t cap);
};

struct PendingMap {
    uint32_t max_entries = 0;
    NodeTable nodes;
    uint64_t len_count[INFW_MAX_PREFIXLEN + 1] = {};
    ValuePool pool;
    uint64_t generation = 0;  // bumped on every successful edit
    // Keys edited since the last commit: their nodes (a removed key stays indexed as a tombstone until then), each
    // with its committed value id (kAbsent: the key was not in the committed set).  Drives the incremental commit.
    static constexpr int32_t kAbsent = -1;
    std::vector<uint32_t> dirty_ids;
    size_t n_dirty() const { return dirty_ids.size(); }
    // After a commit: the edits are the committed state; tombstones leave the index.
    void clear_dirty();
    // Key order for get_next_key (trie post-order), kept lazily: a sorted vector that may still hold removed keys
    // (and a key twice) plus the keys inserted since the last merge; next_key skips keys no longer live, and a
    // merge drops them.  A remove costs nothing here and an insert one small-set insert (a std::set over a
    // million keys cost ~5 us per insert or remove, in cache misses).
    mutable std::vector<NodeKey> order_vec;
    mutable std::set<NodeKey, PostOrderLess> order_add;
    void order_merge() const;
    // The live keys in post-order (merges first).
    const std::vector<NodeKey> &ordered() const {
        order_merge();
        return order_vec;
    }
    // Prefetch the index slot / the node of a key a few iterations ahead of update or remove.
    void prefetch_slot(const lpm_ip_key_st *key) const;
    void prefetch_node(const lpm_ip_key_st *key) const;
    // Short keys (1..32 address bits) listed under their enclosing block: (level, ifindex, the address's top
    // `level` bits) -> the entries with level < L <= level + 8, for level 0, 8, 16, 24.  An incremental commit
    // paints the DIR-24-8 words (and tbl8 entries) an edit covers from these lists — base answer, then the
    // longer entries inside the block in ascending length — instead of probing the map per word and length.
    // The NodeVal pointers stay valid: pool nodes never move, and a removed key leaves its list.
    struct ShortRef {
        uint32_t a32;       // address bits 0..31, masked to L
        uint32_t L;
        const NodeVal *v;
    };
    std::unordered_map<uint64_t, std::vector<ShortRef>> sub;
    static uint64_t sub_key(uint32_t level, uint32_t ifindex, uint32_t a32) {
        return (uint64_t)(level >> 3) << 62 | (uint64_t)ifindex << 24 | (level ? a32 >> (32 - level) : 0u);
    }
    const std::vector<ShortRef> *sub_list(uint32_t level, uint32_t ifindex, uint32_t a32) const {
        auto it = sub.find(sub_key(level, ifindex, a32));
        return it == sub.end() ? nullptr : &it->second;
    }
    void index_short(const NodeKey &k, const NodeVal *v);  // v == nullptr: remove
    PendingMap() = default;
    PendingMap(const PendingMap &) = delete;  // `sub` points into `nodes`
    PendingMap &operator=(const PendingMap &) = delete;

    int update(const lpm_ip_key_st *key, const uint8_t *val, uint64_t flags);
    int update_vid(const lpm_ip_key_st *key, uint32_t vid, uint64_t flags, const uint8_t *val = nullptr);
    // An imported committed set into an empty map (image.cpp); clear() empties the map.
    int install_committed(const ImageEntries &ent, std::string *why);
    void clear();
    int remove(const lpm_ip_key_st *key);
    int lookup(const lpm_ip_key_st *key, uint8_t *val) const;
    int next_key(const lpm_ip_key_st *key, lpm_ip_key_st *next) const;
    // Longest entry with minlen <= prefixLen <= maxlen covering md (20 bytes:
    // ifindex LE + address): its node, or nullptr.
    const NodeVal *longest(const uint8_t md[20], uint32_t minlen, uint32_t maxlen) const;
    // The same for prefixLen 32..32+maxL of one ifindex (the short table's keys), through `sub`.
    const NodeVal *longest_short(const uint8_t ifx_le[4], uint32_t a32, uint32_t maxL) const;
};

void mask_bits(const uint8_t *in, uint32_t plen, uint8_t *out, int nbytes);

// ------------------------------------------------------------------------
// One compiled epoch on the host (tables.cpp).
// ------------------------------------------------------------------------
struct HostTables {
    std::vector<uint32_t> if_keys, if_slot;
    uint32_t if_mult = 0, if_shift = 0;  // collision-free placement (0: open addressing)
    uint32_t n_slots = 0;
    std::vector<uint32_t> l16;    // n_slots << 16
    std::vector<infw_bnode> nodes;
    std::vector<uint32_t> vpool;
    uint64_t n_tbl8_groups = 0;   // DIR-24-8 second-level groups of the build image
    std::vector<uint64_t> tbl24;        // DIR-24-8 form (short_mode == INFW_SHORT_DIR24), INFW_D24_* words
    std::vector<uint32_t> tbl8;         // 256-value groups of every /24 with entries longer than /24
    std::unordered_map<uint64_t, uint32_t> tbl8_of;  // slot << 24 | /24 -> its group (inline words too)
    uint32_t short_mode = INFW_SHORT_DIR24;
    std::vector<infw_long_entry> ltab;
    std::vector<infw_v6_bucket> btab;
    uint64_t n_buckets = 0, n_overflow_groups = 0;
    std::vector<uint32_t> wild{0u, 0u, 0u};  // prefixLen < 32 entries: {plen, key bits, list+1}, longest first
    uint32_t n_wild = 0;
    std::vector<uint8_t> levels;
    std::vector<uint64_t> desc;
    std::vector<uint64_t> rules;
    std::vector<infw_dt_line> dte, dtl;  // decision-table entry and leaf lines
    uint32_t dt_plog2 = 0;               // value-axis parts per (list, class): 1 << dt_plog2
    std::vector<uint32_t> dt_pl;         // per-list part counts (INFW_DT_PL_LISTS words) or empty (infw_tables.h)
    std::vector<uint64_t> d16;           // d16_on: n_slots << 16 /16 words in front of DIR-24-8 (infw_tables.h)
    uint32_t d16_on = 0;
    uint32_t d16_permille = 0;           // of the /16s holding a prefix longer than /16, those with an inline word
    uint32_t dt_half = 0;                // the kernel reads decision lines half-first (choose_dt_half)
    uint64_t dt_short_lines = 0;         // entry lines a first half answers (infw_dt_line_short; not serialised)
    uint32_t n_lists = 0;
    uint64_t n_entries = 0;
    uint64_t n_long_entries = 0;
    // A host view with the same walk functions as the device (self-test only).
    infw_dev_tables view() const;
};

// The device-resident buffers of one image, in upload order.
enum TableBuf {
    TB_IFK, TB_IFS, TB_L16, TB_NODES, TB_VPOOL, TB_TBL24, TB_TBL8, TB_LTAB, TB_BTAB,
    TB_DESC, TB_RULES, TB_DTE, TB_DTL, TB_LEVELS, TB_WILD, TB_DTPL, TB_D16, TB_COUNT
};
// The kernel's view of image h whose buffer b lives at buf[b] (device buffers, or the host vectors for view()).
infw_dev_tables view_of(const HostTables &h, void *const buf[TB_COUNT]);

// Per-context options (infw_set_option, include/infw.h).  Each one selects among bit-exact forms of the same epoch,
// the host threads of a compile, how often the kernel flushes its counters, or tracing: none changes a result word,
// a verdict or a counter.  Defaults are the measured choices; -1 means "chosen per epoch".
struct Options {
    int32_t short_table = -1;       // full compiles: -1 DIR-24-8 while n_slots x 128 MiB <= 4 GiB, else compressed;
                                    // 0 DIR-24-8, 1 the compressed 16-8-8 form
    int32_t d16 = -1;               // /16 words in front of DIR-24-8: -1 per epoch (build_d16), 0 never, 1 always
    int32_t dt_half = -1;           // half-first decision-line reads: -1 per epoch (choose_dt_half), 0, 1
    int32_t dt_parts = 0;           // value parts per (list, class): 0 per epoch (choose_dt_plog2), else 1|2|4|8|16
    int32_t dt_adapt = 1;           // per-list part counts (<= INFW_DT_PL_LISTS lists): 1 on, 0 off
    int64_t dt_budget_mb = 2048;    // the entry lines of one image stay below this (fewer parts)
    int32_t compile_threads = 0;    // host threads of a full compile: 0 = hardware threads (<= 16)
    int32_t split = -1;             // two-phase classify: -1 when the entry lines exceed split_min_mb, 0 never, 1 always
    int64_t split_min_mb = 1024;
    int32_t stat_flush_tiles = 1024; // a workgroup flushes its LDS counters every this many tiles (1..1024)
    int32_t trace = 0;              // stderr: 1 compile phases, 2 incremental patch phases, 4 commit timing,
                                    // 8 classify_xdp_host pipeline timing
    int32_t host_threads = 0;       // packer threads of infw_classify_xdp_host: 0 = the CPUs the process may use (<= 16)
};
// Name, bounds and field of every option (abi.cpp infw_set_option / infw_get_option / infw_option_name).
struct OptionDef {
    const char *name;
    int64_t lo, hi;
    const char *doc;
};

// Bookkeeping of the compiled image that an incremental commit patches
// (incremental.cpp); filled by compile_tables.
struct IncState {
    bool valid = false;
    std::unordered_map<uint32_t, uint32_t> slot_of;      // ifindex -> slot
    std::unordered_map<uint32_t, uint32_t> list_of_vid;  // interned value -> rule list
    std::vector<uint64_t> list_refs;                     // entries referencing each list
    uint64_t dead_lists = 0;                             // lists no entry references any more
    // One bit per tbl24 word (slot << 24 | /24): a tbl8 group exists for it (tbl8_of has it).  Derived from
    // tbl8_of on the first patch after a compile or import, then kept up to date; lets a short edit skip the
    // hash lookup for the (most common) words without a group.
    std::vector<uint64_t> g8bits;
    // list_of_vid as a dense vector (vid -> list, ~0u: none), derived on the first patch after a compile or
    // import and kept up to date by the patch: a commit looks every edited key's old and new list up.
    std::vector<uint32_t> lid_of_vid;
};

// The /16 word of (slot, address bits 0..15) from the DIR-24-8 image: inline when its runs fit, else 0.
// *runs: 1 for a /16 of one answer throughout (either way).
uint64_t d16_word(const HostTables &h, uint32_t slot, uint32_t hi, uint32_t *runs = nullptr);
// Decide whether the epoch gets /16 words (req: Options::d16) and build them; n_short_wide of the n_short
// <= /32 prefixes are /20 or shorter.
void build_d16(HostTables &h, uint64_t n_short, uint64_t n_short_wide, int req = -1);
// An entry line whose first 32 B answer every value: a compact leaf of <= 9 segments.
inline uint32_t infw_dt_line_short(const infw_dt_line &l) {
    return (l.w[0] & INFW_DT_COMPACT) && !(l.w[0] & INFW_DT_ROOT) && (l.w[0] & 0xFFu) <= 9;
}
uint64_t count_dt_short_lines(const HostTables &h);
// Half-first decision-line reads for this image (req: Options::dt_half), from h.dt_short_lines.
uint32_t choose_dt_half(const HostTables &h, int req = -1);

int compile_tables(const PendingMap &m, HostTables &out, const Options &opt = Options(), IncState *inc = nullptr);
// Host bytes of buffer b (at least one element, like the upload).
void host_buffer(const HostTables &h, int b, const void **p, size_t *bytes);
struct DirtyRange {
    uint32_t buf;
    uint64_t off, len;  // bytes
};
// Table images (image.cpp): size, serialise, parse (nothing installed; ent/h/inc filled).
uint64_t image_bytes(const PendingMap &m, const HostTables &h, const IncState &inc, const char *build_id);
void image_write(const PendingMap &m, const HostTables &h, const IncState &inc, const char *build_id, uint8_t *out);
int image_read(const uint8_t *buf, uint64_t size, const char *build_id, ImageEntries &ent, HostTables &h,
               IncState &inc, std::string *why);

// Apply m.dirty to the compiled image in place (DIR-24-8 words and tbl8 groups,
// IPv6 buckets, appended rule lists), recording every byte range it changes.
// Returns 0 when patched, 1 when the edit needs a full compile (*why says why;
// nothing was modified), < 0 on error.
int patch_tables(const PendingMap &m, HostTables &h, IncState &inc, std::vector<DirtyRange> &ranges,
                 std::string *why, const Options &opt = Options());
// The patch's derived indexes (g8bits, lid_of_vid) of a freshly compiled or imported image, built up front so the
// first incremental commit after it does not pay for them (~5 ms at configs[2]).
void patch_prepare(const HostTables &h, IncState &inc);

// Class-filtered GPU rule records of one 1200-B value (appended to rules) and
// the per-class first-match decision-table entry lines, INFW_NCLS << plog2 of
// them (leaf lines appended to leaves).
int compile_rule_list(const uint8_t *val, std::vector<uint64_t> &rules, uint64_t desc_out[INFW_DESC_STRIDE],
                      infw_dt_line *entry_out, std::vector<infw_dt_line> &leaves, uint32_t plog2, uint32_t *pl_out = nullptr);
// First-match step function of one class list (records {lo16, hi16, result32} in
// scan order): segment starts ascending from 0 and the result of each segment.
void step_function(const std::vector<uint64_t> &recs, std::vector<uint32_t> &starts, std::vector<uint32_t> &res);
// Decision table of one class list (records {lo16, hi16, result32} in scan
// order): 1 << plog2 entry lines, one per part of the value axis.
int build_decision_table(const std::vector<uint64_t> &recs, infw_dt_line *entry, std::vector<infw_dt_line> &leaves,
                         uint32_t plog2);
// Entry (and leaf) lines of a step function: segment starts ascending from 0 and their results.
int emit_decision_lines(const std::vector<uint32_t> &starts, const std::vector<uint32_t> &res, infw_dt_line &entry,
                        std::vector<infw_dt_line> &leaves);

}  // namespace infw
