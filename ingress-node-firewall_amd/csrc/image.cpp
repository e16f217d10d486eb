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
// Layout: little-endian; a header (magic, format, ABI version, build id, element sizes, XXH64 of the payload) and
// then length-prefixed arrays.  An image is only accepted by a library of the same build id (the build id hashes
// every source that defines the serialised layout: Makefile BUILDID_SRCS), when the payload hashes to the
// header's value, and when the parsed tables pass check_tables: every index the kernel or the host walk follows
// stays inside its buffer and every probe loop has an empty slot to stop at — an image torn in /dev/shm or written
// by a faulty exporter is refused with -EINVAL before anything is installed or uploaded (the verifier gate of the
// reference's load, pkg/ebpf/ingress_node_firewall_loader.go:85-93, plays that role for its maps).
#include <errno.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "infw_internal.h"

namespace infw {

namespace {

constexpr char kMagic[8] = {'I', 'N', 'F', 'W', 'I', 'M', 'G', '1'};
constexpr uint32_t kFormat = 2;  // 2: payload hash in the header

// XXH64 (seed 0) of the payload, the published xxHash 64-bit algorithm — tests recompute it with the xxhash module.
constexpr uint64_t kP1 = 0x9E3779B185EBCA87ull, kP2 = 0xC2B2AE3D27D4EB4Full, kP3 = 0x165667B19E3779F9ull,
                   kP4 = 0x85EBCA77C2B2AE63ull, kP5 = 0x27D4EB2F165667C5ull;
inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t rd64(const uint8_t *p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}
inline uint32_t rd32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
inline uint64_t xxh_round(uint64_t acc, uint64_t in) { return rotl64(acc + in * kP2, 31) * kP1; }
inline uint64_t xxh_merge(uint64_t acc, uint64_t v) { return (acc ^ xxh_round(0, v)) * kP1 + kP4; }
uint64_t xxh64(const uint8_t *p, uint64_t len) {
    const uint8_t *const end = p + len;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = kP1 + kP2, v2 = kP2, v3 = 0, v4 = 0 - kP1;
        for (const uint8_t *lim = end - 32; p <= lim; p += 32) {
            v1 = xxh_round(v1, rd64(p));
            v2 = xxh_round(v2, rd64(p + 8));
            v3 = xxh_round(v3, rd64(p + 16));
            v4 = xxh_round(v4, rd64(p + 24));
        }
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xxh_merge(xxh_merge(xxh_merge(xxh_merge(h, v1), v2), v3), v4);
    } else {
        h = kP5;
    }
    h += len;
    for (; p + 8 <= end; p += 8) h = rotl64(h ^ xxh_round(0, rd64(p)), 27) * kP1 + kP4;
    if (p + 4 <= end) {
        h = rotl64(h ^ (uint64_t)rd32(p) * kP1, 23) * kP2 + kP3;
        p += 4;
    }
    for (; p < end; p++) h = rotl64(h ^ (uint64_t)*p * kP5, 11) * kP1;
    h ^= h >> 33;
    h *= kP2;
    h ^= h >> 29;
    h *= kP3;
    return h ^ (h >> 32);
}

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
    uint64_t payload_hash;  // XXH64 of every byte after the header
};
static_assert(sizeof(Header) == 72, "image header layout");

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
    io.pod(h.short_mode);
    io.vec(h.ltab);
    io.vec(h.btab);
    io.pod(h.n_buckets);
    io.pod(h.n_overflow_groups);
    io.vec(h.wild);
    io.pod(h.n_wild);
    io.vec(h.levels);
    io.vec(h.desc);
    io.vec(h.rules);
    io.vec(h.dte);
    io.vec(h.dtl);
    io.pod(h.dt_plog2);
    io.vec(h.dt_pl);
    io.vec(h.d16);
    io.pod(h.d16_on);
    io.pod(h.d16_permille);
    io.pod(h.dt_half);
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
    if (out) {
        const uint64_t hv = xxh64(out + sizeof(Header), w.n - sizeof(Header));
        memcpy(out + offsetof(Header, payload_hash), &hv, sizeof hv);
    }
    return w.n;
}

// Structural checks of parsed tables (see the file comment): list+1 values <= n_lists, group / node / line /
// record indices inside their buffers, sizes as the compiler lays them out, the counters the kernel's lean
// instantiation is chosen from equal to what the tables hold, and the incremental-commit state's ids in range.
bool check_tables(const HostTables &h, const IncState &inc, uint64_t n_vals, std::string *why) {
    auto bad = [&](const char *what) {
        *why = std::string("corrupt table image: ") + what;
        return false;
    };
    auto pow2 = [](uint64_t x) { return x && !(x & (x - 1)); };
    const uint64_t L = h.n_lists;  // list+1 values run 1..L (0 = no entry)
    const uint64_t per_list = (uint64_t)INFW_NCLS << h.dt_plog2;
    // never-empty device buffers (the compiler keeps a placeholder element in each)
    if (h.tbl24.empty() || h.tbl8.empty() || h.nodes.empty() || h.vpool.empty() || h.rules.empty() ||
        h.dtl.empty() || h.dte.empty() || h.desc.empty() || h.wild.size() < 3 || h.d16.empty() ||
        h.l16.empty())
        return bad("empty table buffer");
    // ifindex map
    const uint64_t nif = h.if_keys.size();
    if (nif != h.if_slot.size() || !pow2(nif) || nif > (1u << 30) || h.n_slots > nif) return bad("ifindex map size");
    bool if_free = false;
    for (uint32_t s : h.if_slot) {
        if (s == INFW_IF_EMPTY) if_free = true;
        else if (s >= h.n_slots) return bad("ifindex slot out of range");
    }
    if (h.if_mult) {
        int lg = 0;
        while ((1ull << lg) < nif) lg++;
        if (h.if_shift < 32u - (uint32_t)lg || h.if_shift > 31u) return bad("ifindex placement shift");
    } else if (!if_free) {
        return bad("ifindex map without a free slot");
    }
    // rule lists: decision lines, part counts, ballot-mode descriptors
    if (h.dt_plog2 > 4 || h.n_lists >= (1u << 25)) return bad("rule list count or part count");
    if (h.dte.size() < std::max<uint64_t>(L, 1) * per_list || h.desc.size() < std::max<uint64_t>(L, 1) * INFW_DESC_STRIDE)
        return bad("decision / descriptor table size");
    if (!h.dt_pl.empty()) {
        if (h.dt_pl.size() != INFW_DT_PL_LISTS) return bad("part-count table size");
        for (uint32_t w : h.dt_pl)
            for (int c = 0; c < INFW_NCLS; c++)
                if (((w >> (3 * c)) & 7u) > h.dt_plog2) return bad("part count above the image's");
    }
    for (const infw_dt_line &l : h.dte)
        if (l.w[0] & INFW_DT_ROOT) {
            // the root selects leaf index + (keys below v); pad keys (0xFFFF) never count
            uint64_t keys = 0;
            for (int k = 1; k < 16; k++) {
                keys += (l.w[k] & 0xFFFFu) != 0xFFFFu;
                keys += (l.w[k] >> 16) != 0xFFFFu;
            }
            if ((uint64_t)(l.w[0] & INFW_DT_INDEX) + keys >= h.dtl.size()) return bad("decision root past the leaf lines");
        }
    for (uint64_t d : h.desc)
        if ((uint64_t)(uint32_t)d + (d >> 32) > h.rules.size()) return bad("class-list descriptor past the rules");
    // short table (<= 32 address bits)
    auto d24_ok = [&](uint64_t w) {
        if (!(w & INFW_D24_GROUP)) return (w >> 32) == 0 && w <= L;
        if (!(w & INFW_D24_INLINE)) return (uint64_t)(uint32_t)w < h.n_tbl8_groups;
        if (w & INFW_D24_ABA) return (w & INFW_D24_ABA_MAXV) <= L && ((w >> 22) & INFW_D24_ABA_MAXV) <= L;
        return (w & INFW_D24_MAXV) <= L && ((w >> 15) & INFW_D24_MAXV) <= L && ((w >> 30) & INFW_D24_MAXV) <= L;
    };
    const bool dir24_image = h.short_mode == INFW_SHORT_DIR24;
    if (h.short_mode > INFW_SHORT_NONE) return bad("short-table form");
    if (dir24_image) {
        if (h.n_slots == 0 || h.tbl24.size() != ((uint64_t)h.n_slots << 24)) return bad("DIR-24-8 size");
        if (h.tbl8.size() % 256 || h.tbl8.size() < h.n_tbl8_groups * 256) return bad("tbl8 size");
        for (uint64_t w : h.tbl24)
            if (!d24_ok(w)) return bad("DIR-24-8 word");
        for (uint32_t v : h.tbl8)
            if (v > L) return bad("tbl8 value");
        for (const auto &g : h.tbl8_of)
            if (g.second >= h.n_tbl8_groups || (g.first >> 24) >= h.n_slots) return bad("tbl8 group index");
    }
    if (h.d16_on) {
        if (h.short_mode != INFW_SHORT_DIR24 || h.d16.size() != ((uint64_t)h.n_slots << 16)) return bad("/16 words");
        for (uint64_t w : h.d16)
            if ((w & INFW_D16_INLINE) && ((w & 0x7FFFu) > L || ((w >> 15) & 0x7FFFu) > L)) return bad("/16 word value");
    }
    if (h.short_mode == INFW_SHORT_COMPRESSED) {
        if (h.l16.size() != ((uint64_t)std::max<uint32_t>(h.n_slots, 1) << 16)) return bad("compressed short-table size");
        // a first-level node's children may be nodes, a second-level node's may not; each node checked once per level
        std::vector<uint8_t> seen(h.nodes.size(), 0);
        std::vector<std::pair<uint32_t, int>> todo;
        auto value_ok = [&](uint32_t v, int level) {
            if (!(v & INFW_NODE_FLAG)) return v <= L;
            const uint32_t i = v & ~INFW_NODE_FLAG;
            if (level >= 2 || i >= h.nodes.size()) return false;
            if (!(seen[i] & (1u << level))) {
                seen[i] |= (uint8_t)(1u << level);
                todo.emplace_back(i, level + 1);
            }
            return true;
        };
        for (uint32_t w : h.l16)
            if (!value_ok(w, 0)) return bad("compressed short-table word");
        while (!todo.empty()) {
            const auto [i, level] = todo.back();
            todo.pop_back();
            const infw_bnode &n = h.nodes[i];
            uint32_t runs = 0;
            for (uint32_t b : n.bm) runs += (uint32_t)__builtin_popcount(b);
            if (!(n.bm[0] & 1u) || n.nv == 0 || runs != n.nv) return bad("short-table node bitmap");
            if (n.nv > INFW_NODE_INLINE && (uint64_t)n.base + n.nv > h.vpool.size()) return bad("short-table node values");
            for (uint32_t k = 0; k < n.nv; k++)
                if (!value_ok(n.nv <= INFW_NODE_INLINE ? n.v[k] : h.vpool[n.base + k], level)) return bad("short-table node value");
        }
    }
    // prefixes shorter than the ifindex
    if ((uint64_t)h.n_wild * 3 > h.wild.size()) return bad("partial-ifindex list size");
    for (uint32_t i = 0; i < h.n_wild; i++)
        if (h.wild[3 * i] > 31 || h.wild[3 * i + 2] > L) return bad("partial-ifindex entry");
    // IPv6 long prefixes: levels, Waldvogel table, /32-group buckets
    if (h.levels.size() > INFW_MAX_LEVELS) return bad("IPv6 level count");
    for (size_t i = 0; i < h.levels.size(); i++)
        if (h.levels[i] < 33 || h.levels[i] > 128 || (i && h.levels[i] <= h.levels[i - 1])) return bad("IPv6 levels");
    if (!pow2(h.ltab.size())) return bad("long-table size");
    bool l_free = false;
    for (const infw_long_entry &e : h.ltab) {
        l_free |= e.tag == 0;
        if (e.bmp > L) return bad("long-table value");
    }
    if (!l_free) return bad("long table without a free entry");
    auto rec_ok = [&](const infw_v6_rec &r) { return (r.meta & 0x1FFFFFFu) <= L && (r.meta >> 25) >= 1 && (r.meta >> 25) <= 96; };
    uint64_t overflowed = 0;
    {
        if (!pow2(h.btab.size())) return bad("IPv6 bucket-table size");
        bool b_free = false;
        for (const infw_v6_bucket &b : h.btab) {
            if (!b.tag) {
                b_free = true;
                continue;
            }
            if (b.tag > h.n_slots || (b.n > INFW_BUCKET_INLINE && b.n != INFW_BUCKET_OVERFLOW)) return bad("IPv6 bucket");
            if (b.n == INFW_BUCKET_OVERFLOW) overflowed++;
            else
                for (uint32_t k = 0; k < b.n; k++)
                    if (!rec_ok(b.rec[k])) return bad("IPv6 record");
        }
        if (!b_free) return bad("IPv6 bucket table without a free bucket");
    }
    if (overflowed != h.n_overflow_groups || (overflowed && h.levels.empty())) return bad("IPv6 overflow groups");
    if (h.dt_half > 1) return bad("decision-line read form");
    // incremental-commit state
    if (inc.valid) {
        if (inc.list_refs.size() != L) return bad("list reference counts");
        for (const auto &p : inc.slot_of)
            if (p.second >= h.n_slots) return bad("ifindex slot of the commit state");
        for (const auto &p : inc.list_of_vid)
            if (p.first >= n_vals || p.second >= L) return bad("value -> list map");
    }
    return true;
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
    if (xxh64(buf + sizeof(Header), size - sizeof(Header)) != hd.payload_hash) {
        *why = "payload hash mismatch (torn or corrupted image)";
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
    if (!check_tables(h, inc, nv, why)) return -EINVAL;
    h.dt_short_lines = count_dt_short_lines(h);
    return 0;
}

// The committed set as the importer's pending map: values interned in id order (distinct values, so each gets the
// id it had), then the nodes with their ids, indexed as update() would.  A context whose entries were all removed
// and committed counts as empty: its leftover value pool and tombstones are dropped first.
// Everything that can refuse an entry set is checked before the map is touched: a refused import leaves the map (and
// its value pool, which the committed image's incremental state refers to by value id) exactly as it was.
static bool entries_distinct(const ImageEntries &ent, std::string *why) {
    const uint64_t nv = ent.vals.size() / 1200;
    std::vector<std::pair<uint64_t, uint64_t>> hv(nv);  // (hash, index)
    for (uint64_t i = 0; i < nv; i++) hv[i] = {xxh64(ent.vals.data() + 1200 * i, 1200), i};
    std::sort(hv.begin(), hv.end());
    for (uint64_t i = 1; i < nv; i++)
        if (hv[i].first == hv[i - 1].first &&
            memcmp(ent.vals.data() + 1200 * hv[i].second, ent.vals.data() + 1200 * hv[i - 1].second, 1200) == 0) {
            *why = "duplicate values in the image";
            return false;
        }
    std::vector<std::pair<uint64_t, uint64_t>> hk(ent.nodes.size());
    for (size_t i = 0; i < ent.nodes.size(); i++) hk[i] = {NodeTable::hash(ent.nodes[i].first), i};
    std::sort(hk.begin(), hk.end());
    for (size_t i = 1; i < hk.size(); i++)
        if (hk[i].first == hk[i - 1].first && ent.nodes[hk[i].second].first == ent.nodes[hk[i - 1].second].first) {
            *why = "duplicate key in the image";
            return false;
        }
    return true;
}

int PendingMap::install_committed(const ImageEntries &ent, std::string *why) {
    if (!nodes.empty() || !dirty_ids.empty()) {
        *why = "the context already holds entries or uncommitted edits";
        return -EBUSY;
    }
    if (ent.nodes.size() > max_entries) {
        *why = "more entries than max_entries";
        return -ENOSPC;
    }
    if (!entries_distinct(ent, why)) return -EINVAL;
    clear();  // an emptied context: its leftover value pool and tombstones go (nothing below refuses)
    const uint64_t nv = ent.vals.size() / 1200;
    for (uint64_t i = 0; i < nv; i++) (void)pool.intern(ent.vals.data() + 1200 * i);
    nodes.reserve(ent.nodes.size());
    order_vec.reserve(ent.nodes.size());
    for (const auto &e : ent.nodes) {
        const uint64_t h = NodeTable::hash(e.first);
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
