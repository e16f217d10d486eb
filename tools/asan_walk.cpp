// Host-only AddressSanitizer/UBSan run of the table compiler and of the shared
// host/device walk (infw_tables.h) over random tables: every compiled form
// (DIR-24-8, compressed 16-8-8, no short entries, IPv6 buckets and overflow
// groups, decision-table entry/leaf lines) is indexed the way the kernel does.
// Build + run: make asan
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

#include "../ingress-node-firewall_amd/csrc/infw_internal.h"

namespace infw {
void set_error(const std::string &s) { fprintf(stderr, "set_error: %s\n", s.c_str()); }
}  // namespace infw
using namespace infw;

static uint64_t rs = 0x1234567;
static uint32_t rnd() {
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return (uint32_t)(rs >> 11);
}

static void random_value(uint8_t *val, int n_rules) {
    memset(val, 0, 1200);
    for (int i = 0; i < n_rules; i++) {
        uint8_t *r = val + 12 * (1 + rnd() % 99);
        uint32_t id = 1 + rnd() % 5000;
        memcpy(r, &id, 4);
        const uint8_t protos[6] = {0, 6, 17, 132, 1, 58};
        r[4] = protos[rnd() % 6];
        uint16_t ps = (uint16_t)rnd(), pe = (rnd() & 1) ? 0 : (uint16_t)(ps + rnd() % 3000);
        memcpy(r + 5, &ps, 2);
        memcpy(r + 7, &pe, 2);
        r[9] = (uint8_t)(rnd() % 4 ? 8 : rnd());
        r[10] = (uint8_t)(rnd() % 3);
        r[11] = (uint8_t)(1 + rnd() % 3);
    }
}

// The compiler options of this harness: the short-table form asked for, /16 words per ASAN_D16 (the harness's own
// switch; the library reads no environment).
static Options opts(int mode) {
    Options o;
    o.short_table = mode == (int)INFW_SHORT_COMPRESSED ? 1 : mode == (int)INFW_SHORT_DIR24 ? 0 : -1;
    if (const char *e = getenv("ASAN_D16")) o.d16 = atoi(e);
    return o;
}

static int run_case(int n_keys, int v4_share, int max_rules, int mode, int seed) {
    rs = 0x9E3779B97F4A7C15ull * (uint64_t)(seed + 1);
    PendingMap m;
    m.max_entries = 1u << 20;
    static uint8_t val[1200];
    for (int i = 0; i < n_keys; i++) {
        lpm_ip_key_st k;
        memset(&k, 0, sizeof k);
        k.ingress_ifindex = 1 + rnd() % 3;
        const bool v4 = (int)(rnd() % 100) < v4_share;
        const uint32_t len = v4 ? rnd() % 33 : (v4_share < 0 || rnd() % 4 == 0) ? 33 + rnd() % 96 : rnd() % 129;
        k.prefixLen = len + 32;
        for (int b = 0; b < 16; b++) k.ip_data[b] = (uint8_t)rnd();
        if (rnd() % 4 == 0) k.ip_data[0] = k.ip_data[1] = k.ip_data[2] = k.ip_data[3] = 10;  // clustered groups
        random_value(val, 1 + rnd() % max_rules);
        m.update(&k, val, 0);
    }
    HostTables h;
    int rc = compile_tables(m, h, opts(mode));
    if (rc) return rc;
    const infw_dev_tables t = h.view();
    uint64_t hits = 0;
    for (int i = 0; i < 200000; i++) {
        uint32_t sa[4] = {rnd(), rnd(), rnd(), rnd()};
        if (rnd() % 2) sa[0] = 0x0A0A0A0Au;
        const int pk = rnd() % 2 ? INFW_PK_V4 : INFW_PK_V6;
        const uint32_t l1 = infw_lpm(t, pk, rnd() % 5, sa);
        if (!l1) continue;
        hits++;
        const int cls = (int)(rnd() % INFW_NCLS);
        const uint32_t v = rnd() & 0xFFFF;
        const uint32_t a = infw_dt_eval(t, l1 - 1, cls, v);
        const uint32_t b = infw_scan_serial(t, t.desc[(uint64_t)(l1 - 1) * INFW_DESC_STRIDE + cls], v);
        if (a != b) {
            fprintf(stderr, "mismatch: list %u cls %d v %u: table %x scan %x\n", l1 - 1, cls, v, a, b);
            return -1;
        }
    }
    printf("keys %d v4%% %d rules<=%d mode %d: lists %u short_mode %u hits %llu\n", n_keys, v4_share, max_rules, mode,
           h.n_lists, h.short_mode, (unsigned long long)hits);
    return 0;
}

// Incremental commits under ASan: random churn (value rewrites, deletes, re-adds, new keys on known
// ifindexes) patched into the compiled image by patch_tables; after every patch the image must walk
// exactly like a fresh compile of the same map.
static uint32_t walk_result(const infw_dev_tables &t, int pk, uint32_t ifx, const uint32_t sa[4], int cls, uint32_t v) {
    const uint32_t l1 = infw_lpm(t, pk, ifx, sa);
    return l1 ? infw_dt_eval(t, l1 - 1, cls, v) : 0u;
}

static int run_churn(int n_keys, int seed) {
    rs = 0xC2B2AE3D27D4EB4Full * (uint64_t)(seed + 7);
    PendingMap m;
    m.max_entries = 1u << 20;
    static uint8_t val[1200];
    std::vector<lpm_ip_key_st> keys;
    auto rand_key = [&]() {
        lpm_ip_key_st k;
        memset(&k, 0, sizeof k);
        k.ingress_ifindex = 1 + rnd() % 3;
        const bool v4 = rnd() % 2;
        const uint32_t len = v4 ? 8 + rnd() % 25 : 33 + rnd() % 96;
        k.prefixLen = len + 32;
        for (int b = 0; b < 16; b++) k.ip_data[b] = (uint8_t)rnd();
        if (rnd() % 3 == 0) k.ip_data[0] = k.ip_data[1] = k.ip_data[2] = 10;
        return k;
    };
    for (int i = 0; i < n_keys; i++) {
        lpm_ip_key_st k = rand_key();
        random_value(val, 1 + rnd() % 40);
        if (m.update(&k, val, 0) == 0) keys.push_back(k);
    }
    HostTables h;
    IncState inc;
    if (compile_tables(m, h, opts(INFW_SHORT_DIR24), &inc)) return -1;
    m.clear_dirty();
    int patched = 0, full = 0;
    const int rounds = getenv("ASAN_CHURN_ROUNDS") ? atoi(getenv("ASAN_CHURN_ROUNDS")) : 8;
    for (int round = 0; round < rounds; round++) {
        const int edits = 1 + rnd() % (round % 3 == 0 ? 400 : 40);
        for (int e = 0; e < edits; e++) {
            const uint32_t r = rnd() % 10;
            if (r < 5 && !keys.empty()) {  // rewrite
                random_value(val, 1 + rnd() % 40);
                m.update(&keys[rnd() % keys.size()], val, 0);
            } else if (r < 7 && !keys.empty()) {
                m.remove(&keys[rnd() % keys.size()]);
            } else {
                lpm_ip_key_st k = rand_key();
                random_value(val, 1 + rnd() % 40);
                if (m.update(&k, val, 0) == 0) keys.push_back(k);
            }
        }
        std::vector<DirtyRange> ranges;
        std::string why;
        int rc = patch_tables(m, h, inc, ranges, &why, opts(INFW_SHORT_DIR24));
        if (rc != 0) {  // a layout change: recompile, as infw_table_commit does
            full++;
            h = HostTables();
            inc = IncState();
            if (compile_tables(m, h, opts(INFW_SHORT_DIR24), &inc)) return -1;
        } else {
            patched++;
            for (const DirtyRange &d : ranges) {
                const void *p;
                size_t bytes;
                host_buffer(h, (int)d.buf, &p, &bytes);
                if (d.off + d.len > bytes + 64) {
                    fprintf(stderr, "churn: range past buffer %u: %llu + %llu > %zu\n", d.buf,
                            (unsigned long long)d.off, (unsigned long long)d.len, bytes);
                    return -1;
                }
            }
        }
        m.clear_dirty();
        HostTables f;
        if (compile_tables(m, f, opts(INFW_SHORT_DIR24))) return -1;
        const infw_dev_tables tp = h.view(), tf = f.view();
        for (int i = 0; i < 20000; i++) {
            uint32_t sa[4] = {rnd(), rnd(), rnd(), rnd()};
            if (rnd() % 2 && !keys.empty()) {  // aim at a key's prefix
                const lpm_ip_key_st &k = keys[rnd() % keys.size()];
                memcpy(sa, k.ip_data, 4);
            }
            if (rnd() % 3 == 0) sa[0] = (sa[0] & 0xFF000000u) | 0x000A0A0Au;
            const int pk = rnd() % 2 ? INFW_PK_V4 : INFW_PK_V6;
            const uint32_t ifx = 1 + rnd() % 3;
            const int cls = (int)(rnd() % INFW_NCLS);
            const uint32_t v = rnd() & 0xFFFF;
            const uint32_t a = walk_result(tp, pk, ifx, sa, cls, v), b = walk_result(tf, pk, ifx, sa, cls, v);
            if (a != b) {
                fprintf(stderr, "churn seed %d round %d: patched %x vs fresh %x\n", seed, round, a, b);
                return -1;
            }
        }
    }
    printf("churn keys %d seed %d: %d patched commits, %d full\n", n_keys, seed, patched, full);
    return 0;
}

// DIR-24-8 word encoding: every 256-value /24 pattern decodes to itself, inline or via its group.
static int check_d24_words() {
    static uint32_t tbl8[256];
    struct {
        const uint32_t *tbl8;
        const uint64_t *tbl24;
    } t{tbl8, nullptr};
    int bad = 0;
    for (int c = 0; c < 20000; c++) {
        const uint32_t runs = 1 + rnd() % 5, big = c % 7 == 0 ? 0x8000u : 0u;
        uint32_t x = 0;
        for (uint32_t r = 0; r < runs; r++) {
            const uint32_t v = (rnd() % 0x8000u) | (r == 1 ? big : 0u), end = r + 1 == runs ? 256 : x + rnd() % (257 - x);
            for (; x < end; x++) tbl8[x] = v;
        }
        const uint64_t w = infw_d24_encode(tbl8, 0);
        t.tbl24 = &w;
        for (uint32_t a = 0; a < 256; a++) bad |= infw_dir24_lookup(t, 0, a) != tbl8[a];
        bad |= (runs <= 3 && !big) && (w & INFW_D24_GROUP) && !(w & INFW_D24_INLINE) && tbl8[0] != tbl8[255];
    }
    // large list ids (configs[2] with 1M distinct lists): the A | B | A form
    for (int c = 0; c < 20000; c++) {
        const uint32_t A = rnd() % 0x500000u, B = c % 5 == 0 ? A + 1 : rnd() % 0x500000u;
        uint32_t b1 = rnd() % 257, b2 = b1 + rnd() % (257 - b1);
        const int shape = c % 4;  // 0: A B A, 1: A B, 2: B A, 3: A B C (not inlinable when large)
        if (shape == 1) b2 = 256;
        if (shape == 2) b1 = 0;
        for (uint32_t x = 0; x < 256; x++) tbl8[x] = x >= b1 && x < b2 ? B : (shape == 3 && x >= b2 ? A ^ 0x1234u : A);
        const uint64_t w = infw_d24_encode(tbl8, 0);
        t.tbl24 = &w;
        for (uint32_t a = 0; a < 256; a++) bad |= infw_dir24_lookup(t, 0, a) != tbl8[a];
        const bool aba = shape != 3 || b2 == 256;
        bad |= aba && A <= INFW_D24_ABA_MAXV && B <= INFW_D24_ABA_MAXV && !(w & INFW_D24_INLINE) && tbl8[0] != tbl8[255];
    }
    if (bad) printf("d24 word encoding mismatch\n");
    return bad;
}

int main() {
    int bad = check_d24_words();
    // churn seeds: 1 in the CPU test suite, more with ASAN_CHURN_SEEDS (e.g. make asan ASAN_CHURN_SEEDS=3)
    const int churn_seeds = getenv("ASAN_CHURN_SEEDS") ? atoi(getenv("ASAN_CHURN_SEEDS")) : 1;
    for (int s = 0; s < churn_seeds; s++) bad |= run_churn(3000, s) != 0;
    const int modes[3] = {INFW_SHORT_DIR24, INFW_SHORT_COMPRESSED, -1};
    for (int s = 0; s < 3; s++)
        for (int mi = 0; mi < 3; mi++) {
            bad |= run_case(2000, 50, 99, modes[mi], s) != 0;
            bad |= run_case(300, 0, 10, modes[mi], s) != 0;   // IPv6 only (long entries only for some seeds)
            bad |= run_case(50, 100, 3, modes[mi], s) != 0;
            bad |= run_case(1, 0, 1, modes[mi], s) != 0;
            bad |= run_case(100, -1, 20, modes[mi], s) != 0;  // long (/33../128) entries only
        }
    printf(bad ? "FAILED\n" : "ok\n");
    return bad;
}
