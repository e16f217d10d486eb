// image.cpp — serialised committed epochs (infw_table_export / infw_table_import, include/infw.h).
//
// One process per GPU each keeps a context; rather than every rank compiling the same 1M-entry set (seconds of
// host time and GiBs of peak RSS each), one rank exports its committed epoch and the others import it.  An image
// holds exactly what a context keeps after a commit:
//   - the committed entry set (PendingMap: the interned 1200-B values in id order, then every node — masked key,
//     stored key bytes, value id — in the map's post-order), so get_next_key / lookup / later edits behave as on
//     the exporter;
//   - the compiled host tables (HostTables: every buffer the devices get, plus the bookkeeping incremental commits
//     patch: tbl8 group index, counts, the chosen forms);
//   - the incremental-commit state (IncState).
// Layout: little-endian; a header (magic, format, ABI version, build id, element sizes) and then length-prefixed
// arrays.  An image is only accepted by a library of the same build id: the table layout is the compiler's.
#include <errno.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "infw_internal.h"

namespace infw {

namespace {

constexpr char kMagic[8] = {'I', 'N', 'F', 'W', 'I', 'M', 'G', '1'};
constexpr uint32_t kFormat = 1;

struct Writer {
    uint8_t *p;  // nullptr: count only
    uint64_t n = 0;
    void put(const void *src, size_t len) {
        if (p && len) memcpy(p + n, src, len);
        n += len;
    }
    template <class T>
    void pod(const T &v) {
        put(&v, sizeof v);
    }
    template <class T>
    void vec(const std::vector<T> &v) {
        pod((uint64_t)v.size());
        put(v.data(), v.size() * sizeof(T));
    }
};

struct Reader {
    const uint8_t *p;
    uint64_t size, n = 0;
    bool ok = true;
    bool get(void *dst, size_t len) {
        if (!ok || len > size - n) return ok = false;
        if (len) memcpy(dst, p + n, len);
        n += len;
        return true;
    }
    template <class T>
    bool pod(T &v) {
        return get(&v, sizeof v);
    }
    template <class T>
    bool vec(std::vector<T> &v) {
        uint64_t c = 0;
        if (!pod(c)) return false;
        if (c > (size - n) / sizeof(T)) return ok = false;
        v.resize(c);
        return get(v.data(), c * sizeof(T));
    }
};

struct Header {
    char magic[8];
    uint32_t format, abi;
    char build_id[32];
    uint32_t sz_bnode, sz_long, sz_bucket, sz_line;
};

Header make_header(const char *build_id) {
    Header h;
    memset(&h, 0, sizeof h);
    memcpy(h.magic, kMagic, 8);
    h.format = kFormat;
    h.abi = INFW_ABI_VERSION;
    strncpy(h.build_id, build_id, sizeof h.build_id - 1);
    h.sz_bnode = sizeof(infw_bnode);
    h.sz_long = sizeof(infw_long_entry);
    h.sz_bucket = sizeof(infw_v6_bucket);
    h.sz_line = sizeof(infw_dt_line);
    return h;
}

template <class IO, class M>
void tables_io(IO &io, M &h) {  // HostTables fields, in one order for both directions
    io.vec(h.if_keys);
    io.vec(h.if_slot);
    io.pod(h.if_mult);
    io.pod(h.if_shift);
    io.pod(h.n_slots);
    io.vec(h.l16);
    io.vec(h.nodes);
    io.vec(h.vpool);
    io.pod(h.n_tbl8_groups);
    io.vec(h.tbl24);
    io.vec(h.tbl8);
    io.pod(h.d24_inline);
    io.pod(h.short_mode);
    io.vec(h.ltab);
    io.vec(h.btab);
    io.pod(h.n_buckets);
    io.pod(h.n_overflow_groups);
    io.pod(h.b2n);
    io.vec(h.wild);
    io.pod(h.n_wild);
    io.vec(h.levels);
    io.vec(h.desc);
    io.vec(h.rules);
    io.vec(h.dte);
    io.vec(h.dtl);
    io.pod(h.dt_plog2);
    io.vec(h.dt_pl);
    io.vec(h.dxr_idx);
    io.vec(h.dxr_lines);
    io.vec(h.d16);
    io.pod(h.d16_on);
    io.pod(h.d16_permille);
    io.pod(h.n_lists);
    io.pod(h.n_entries);
    io.pod(h.n_long_entries);
}

template <class K, class V>
void map_write(Writer &w, const std::unordered_map<K, V> &m) {  // sorted by key: the same set gives the same bytes
    w.pod((uint64_t)m.size());
    std::vector<std::pair<K, V>> kv(m.begin(), m.end());
    std::sort(kv.begin(), kv.end(), [](const std::pair<K, V> &a, const std::pair<K, V> &b) { return a.first < b.first; });
    for (const auto &e : kv) {
        w.pod(e.first);
        w.pod(e.second);
    }
}

template <class K, class V>
bool map_read(Reader &r, std::unordered_map<K, V> &m) {
    uint64_t c = 0;
    if (!r.pod(c) || c > (r.size - r.n) / (sizeof(K) + sizeof(V))) return r.ok = false;
    m.clear();
    m.reserve(c);
    for (uint64_t i = 0; i < c; i++) {
        K k;
        V v;
        if (!r.pod(k) || !r.pod(v)) return false;
        m.emplace(k, v);
    }
    return true;
}

uint64_t write_image(const PendingMap &m, const HostTables &h, const IncState &inc, const char *build_id,
                     uint8_t *out) {
    Writer w{out};
    w.pod(make_header(build_id));
    // entry set: the value pool in id order, then the nodes in post-order
    w.pod((uint64_t)m.pool.vals.size());
    for (const auto &v : m.pool.vals) w.put(v.data(), v.size());
    const std::vector<NodeKey> &order = m.ordered();
    w.pod((uint64_t)order.size());
    for (const NodeKey &k : order) {
        const NodeVal &v = m.nodes.find_live(k)->val;
        w.pod(k.plen);
        w.put(k.md, sizeof k.md);
        w.put(v.data, sizeof v.data);
        w.pod(v.vid);
    }
    tables_io(w, h);
    map_write(w, h.tbl8_of);
    const uint8_t valid = inc.valid;
    w.pod(valid);
    map_write(w, inc.slot_of);
    map_write(w, inc.list_of_vid);
    w.vec(inc.list_refs);
    w.pod(inc.dead_lists);
    return w.n;
}

}  // namespace

uint64_t image_bytes(const PendingMap &m, const HostTables &h, const IncState &inc, const char *build_id) {
    return write_image(m, h, inc, build_id, nullptr);
}

void image_write(const PendingMap &m, const HostTables &h, const IncState &inc, const char *build_id, uint8_t *out) {
    write_image(m, h, inc, build_id, out);
}

int image_read(const uint8_t *buf, uint64_t size, const char *build_id, ImageEntries &ent, HostTables &h,
               IncState &inc, std::string *why) {
    Reader r{buf, size};
    Header hd;
    const Header want = make_header(build_id);
    if (!r.pod(hd) || memcmp(hd.magic, kMagic, 8) != 0 || hd.format != kFormat) {
        *why = "not a table image";
        return -EINVAL;
    }
    if (hd.abi != want.abi || memcmp(hd.build_id, want.build_id, sizeof hd.build_id) != 0 ||
        hd.sz_bnode != want.sz_bnode || hd.sz_long != want.sz_long || hd.sz_bucket != want.sz_bucket ||
        hd.sz_line != want.sz_line) {
        *why = std::string("image of another build (") + std::string(hd.build_id, strnlen(hd.build_id, 32)) +
               ", this library is " + build_id + ")";
        return -EINVAL;
    }
    uint64_t nv = 0;
    if (!r.pod(nv) || nv > (size - r.n) / 1200) {
        *why = "truncated value pool";
        return -EINVAL;
    }
    ent.vals.resize(nv * 1200);
    r.get(ent.vals.data(), nv * 1200);
    uint64_t nn = 0;
    if (!r.pod(nn) || nn > (size - r.n) / (4 + 20 + 20 + 4)) {
        *why = "truncated entry set";
        return -EINVAL;
    }
    ent.nodes.resize(nn);
    for (auto &e : ent.nodes) {
        r.pod(e.first.plen);
        r.get(e.first.md, sizeof e.first.md);
        r.get(e.second.data, sizeof e.second.data);
        r.pod(e.second.vid);
        if (r.ok && (e.first.plen > INFW_MAX_PREFIXLEN || e.second.vid >= nv)) {
            *why = "corrupt entry";
            return -EINVAL;
        }
    }
    tables_io(r, h);
    map_read(r, h.tbl8_of);
    uint8_t valid = 0;
    r.pod(valid);
    inc.valid = valid != 0;
    map_read(r, inc.slot_of);
    map_read(r, inc.list_of_vid);
    r.vec(inc.list_refs);
    r.pod(inc.dead_lists);
    if (!r.ok || r.n != size) {
        *why = r.ok ? "trailing bytes after the image" : "truncated image";
        return -EINVAL;
    }
    return 0;
}

// The committed set as the importer's pending map: values interned in id order (distinct values, so each gets the
// id it had), then the nodes with their ids, indexed as update() would.
int PendingMap::install_committed(const ImageEntries &ent, std::string *why) {
    if (!nodes.empty() || !pool.vals.empty() || !dirty_ids.empty()) {
        *why = "the context already holds entries";
        return -EBUSY;
    }
    if (ent.nodes.size() > max_entries) {
        *why = "more entries than max_entries";
        return -ENOSPC;
    }
    const uint64_t nv = ent.vals.size() / 1200;
    for (uint64_t i = 0; i < nv; i++)
        if (pool.intern(ent.vals.data() + 1200 * i) != i) {
            *why = "duplicate values in the image";
            return -EINVAL;
        }
    nodes.reserve(ent.nodes.size());
    order_vec.reserve(ent.nodes.size());
    for (const auto &e : ent.nodes) {
        const uint64_t h = NodeTable::hash(e.first);
        if (nodes.find(e.first, h)) {
            *why = "duplicate key in the image";
            return -EINVAL;
        }
        MapNode *n = nodes.insert(e.first, h);
        n->val = e.second;
        nodes.set_live(n, true);
        index_short(e.first, &n->val);
        order_vec.push_back(e.first);  // post-order already
        len_count[e.first.plen]++;
    }
    if (!std::is_sorted(order_vec.begin(), order_vec.end(), PostOrderLess()))  // written in post-order; if not,
        std::sort(order_vec.begin(), order_vec.end(), PostOrderLess());          // get_next_key still must be
    generation++;
    return 0;
}

void PendingMap::clear() {
    nodes.clear();
    order_vec.clear();
    order_add.clear();
    memset(len_count, 0, sizeof len_count);
    pool.clear();
    dirty_ids.clear();
    sub.clear();
    generation++;
}

}  // namespace infw
