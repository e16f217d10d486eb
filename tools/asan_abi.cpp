// AddressSanitizer/UBSan driver of the host-only paths of the C ABI (include/infw.h), linked against the ASan build
// of libinfw.so (make asan-host; no GPU involved): the encoders (infw_build_ebpf_key / infw_make_rule, valid and
// rejected inputs), map edits single and batched with their flag semantics, lookups, the get_next_key walk, full and
// incremental commits, the debug walk of the committed host image, and table images — export, import, re-export,
// incremental edits on exporter and importer alike, and corrupt images: every header byte and bytes spread over the
// whole payload flipped, truncations, trailing bytes, import into a busy context and into one emptied by deletes.
//   asan_abi                 the self-test above; prints "ok"
//   asan_abi import FILE     import FILE into a fresh host-only context; prints "rc=<errno> <last error>"
//                            (tests/test_image_cpu.py feeds it structurally corrupted images with a valid hash)
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "infw.h"

#define CHECK(cond)                                                                                        \
    do {                                                                                                   \
        if (!(cond)) {                                                                                     \
            fprintf(stderr, "%s:%d: check failed: %s (last error: %s)\n", __FILE__, __LINE__, #cond,      \
                    infw_last_error());                                                                    \
            return 1;                                                                                      \
        }                                                                                                  \
    } while (0)

static uint64_t rs = 0x243F6A8885A308D3ull;
static uint32_t rnd() {
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return (uint32_t)(rs >> 11);
}

struct Ctx {
    infw_ctx *c = nullptr;
    int rc;
    explicit Ctx(uint32_t max_entries) { rc = infw_create(&c, nullptr, 0, max_entries, INFW_F_HOST_ONLY); }
    ~Ctx() {
        if (c) infw_destroy(c);
    }
};

// A rule list of n rules through infw_make_rule (the makeIngressFwRulesMap encoder), plus rejected inputs.
static int random_value(rulesVal_st *v, int n) {
    memset(v, 0, sizeof *v);
    static const char *protos[6] = {"TCP", "UDP", "SCTP", "ICMP", "ICMPv6", ""};
    for (int i = 0; i < n; i++) {
        const uint32_t order = 1 + rnd() % 99;
        const char *p = protos[rnd() % 6];
        char ports[32] = "";
        const bool l4 = !strcmp(p, "TCP") || !strcmp(p, "UDP") || !strcmp(p, "SCTP");
        if (l4) {
            const uint32_t a = 1 + rnd() % 60000;
            if (rnd() % 2) snprintf(ports, sizeof ports, "%u", a);
            else snprintf(ports, sizeof ports, "%u-%u", a, a + 1 + rnd() % 2000);
        }
        const int rc = infw_make_rule(v, order, p, l4 ? ports : nullptr, (uint8_t)(rnd() % 4 ? 8 : rnd()),
                                      (uint8_t)(rnd() % 3), rnd() % 2 ? "Allow" : "Deny");
        CHECK(rc == 0);
    }
    // inputs the Go code rejects, and an order past the array (on a scratch value: a rejected call may have
    // written part of its slot, as the Go code does before returning its error)
    rulesVal_st s;
    memset(&s, 0, sizeof s);
    CHECK(infw_make_rule(&s, 5, "TCP", "70000", 0, 0, "Allow") == -EINVAL);
    CHECK(infw_make_rule(&s, 5, "TCP", "9-x", 0, 0, "Allow") == -EINVAL);
    CHECK(infw_make_rule(&s, 5, "TCP", "300-200", 0, 0, "Allow") == -EINVAL);
    CHECK(infw_make_rule(&s, 5, "TCP", nullptr, 0, 0, "Allow") == -EINVAL);
    CHECK(infw_make_rule(&s, 5, "TCP", "80", 0, 0, "Maybe") == -EINVAL);
    CHECK(infw_make_rule(&s, 5, "GRE", nullptr, 0, 0, "Deny") == 0);  // no case in the Go switch: protocol 0
    CHECK(infw_make_rule(&s, 100, "TCP", "80", 0, 0, "Deny") == -E2BIG);
    CHECK(infw_make_rule(nullptr, 5, "TCP", "80", 0, 0, "Deny") == -EINVAL);
    return 0;
}

static int random_key(lpm_ip_key_st *k) {
    char cidr[96];
    const uint32_t ifx = 1 + rnd() % 3;
    if (rnd() % 2) {
        const uint32_t a = rnd() % 4 == 0 ? 10 : rnd() % 224;
        snprintf(cidr, sizeof cidr, "%u.%u.%u.%u/%u", a, rnd() % 256, rnd() % 256, rnd() % 256, 16 + rnd() % 17);
    } else {
        snprintf(cidr, sizeof cidr, "%x:%x:%x:%x:%x::%x/%u", 0x2000 + rnd() % 16, rnd() % 0x10000, rnd() % 0x10000,
                 rnd() % 0x10000, rnd() % 0x10000, rnd() % 0x10000, rnd() % 4 ? 33 + rnd() % 96 : 16 + rnd() % 17);
    }
    CHECK(infw_build_ebpf_key(ifx, cidr, k) == 0);
    return 0;
}

// n tuples {saddr[4], ifindex, pkt_len, meta, l4word}, half aimed at the keys' prefixes.
static std::vector<uint32_t> tuples(const std::vector<lpm_ip_key_st> &keys, uint32_t n) {
    std::vector<uint32_t> t(8ull * n);
    static const uint32_t protos[5] = {6, 17, 132, 1, 58};
    for (uint32_t i = 0; i < n; i++) {
        uint32_t *q = &t[8ull * i];
        const bool v6 = rnd() % 2;
        for (int j = 0; j < 4; j++) q[j] = rnd();
        uint32_t ifx = 1 + rnd() % 4;
        if (rnd() % 2 && !keys.empty()) {
            const lpm_ip_key_st &k = keys[rnd() % keys.size()];
            memcpy(q, k.ip_data, 16);
            ifx = k.ingress_ifindex;
        }
        q[4] = ifx;
        q[5] = 60 + rnd() % 1400;
        q[6] = (v6 ? 0x86DDu : 0x0800u) | protos[rnd() % 5] << 16 | (rnd() % 16 ? 255u : rnd() % 80) << 24;
        q[7] = rnd();
    }
    return t;
}

static int walk(infw_ctx *c, const std::vector<uint32_t> &t, std::vector<uint32_t> &out) {
    out.assign(t.size() / 8, 0);
    CHECK(infw_debug_walk(c, t.data(), t.size() / 8, out.data()) == 0);
    return 0;
}

static int export_image(infw_ctx *c, std::vector<uint8_t> &img) {
    uint64_t n = 0;
    CHECK(infw_table_export(c, nullptr, 0, &n) == 0 && n > 72);
    uint8_t small[16];
    uint64_t m = 0;
    CHECK(infw_table_export(c, small, sizeof small, &m) == -ENOSPC && m == n);
    img.assign(n, 0);
    CHECK(infw_table_export(c, img.data(), n, &m) == 0 && m == n);
    return 0;
}

static int edit(infw_ctx *c, std::vector<lpm_ip_key_st> &keys, const std::vector<rulesVal_st> &vals, int n_edits) {
    for (int e = 0; e < n_edits; e++) {
        const uint32_t r = rnd() % 10;
        if (r < 4 && !keys.empty()) {
            CHECK(infw_table_update(c, &keys[rnd() % keys.size()], &vals[rnd() % vals.size()], 2 /*BPF_EXIST*/) == 0);
        } else if (r < 6 && !keys.empty()) {
            const size_t i = rnd() % keys.size();
            CHECK(infw_table_delete(c, &keys[i]) == 0);
            CHECK(infw_table_delete(c, &keys[i]) == -ENOENT);
            keys[i] = keys.back();
            keys.pop_back();
        } else {
            lpm_ip_key_st k;
            if (random_key(&k)) return 1;
            const int rc = infw_table_update(c, &k, &vals[rnd() % vals.size()], 1 /*BPF_NOEXIST*/);
            CHECK(rc == 0 || rc == -EEXIST);
            if (rc == 0) keys.push_back(k);
        }
    }
    return 0;
}

static int selftest() {
    std::vector<rulesVal_st> vals(48);
    for (size_t i = 0; i < vals.size(); i++)
        if (random_value(&vals[i], 1 + (int)(rnd() % 99))) return 1;
    lpm_ip_key_st k;
    CHECK(infw_build_ebpf_key(3, "1.2.3.4/33", &k) == -EINVAL);
    CHECK(infw_build_ebpf_key(3, "not-a-cidr", &k) == -EINVAL);
    CHECK(infw_build_ebpf_key(3, "::1/129", &k) == -EINVAL);

    Ctx a(1u << 16);
    CHECK(a.rc == 0);
    std::vector<lpm_ip_key_st> keys;
    for (int i = 0; i < 2000; i++) {
        if (random_key(&k)) return 1;
        const int rc = infw_table_update(a.c, &k, &vals[rnd() % vals.size()], 1);
        CHECK(rc == 0 || rc == -EEXIST);
        if (rc == 0) keys.push_back(k);
    }
    {  // batch update with a value index, then a batch delete of part of it
        std::vector<lpm_ip_key_st> bk(1000);
        std::vector<uint32_t> vi(bk.size());
        for (size_t i = 0; i < bk.size(); i++) {
            if (random_key(&bk[i])) return 1;
            bk[i].ip_data[15] ^= 0x5A;  // distinct from the single updates in most cases
            vi[i] = rnd() % vals.size();
        }
        uint64_t done = 0;
        CHECK(infw_table_update_batch(a.c, bk.data(), vals.data(), vi.data(), bk.size(), 0, &done) == 0 && done == bk.size());
    }
    uint64_t count = 0;
    CHECK(infw_table_count(a.c, &count) == 0);
    {  // the key walk visits every entry once; from here on `keys` is exactly the map's key set
        keys.clear();
        lpm_ip_key_st cur, nxt;
        int rc = infw_table_get_next_key(a.c, nullptr, &nxt);
        while (rc == 0) {
            keys.push_back(nxt);
            cur = nxt;
            rc = infw_table_get_next_key(a.c, &cur, &nxt);
        }
        CHECK(rc == -ENOENT && keys.size() == count);
    }
    {  // batch delete of 200 of them; a second pass stops at the first absent key
        uint64_t done = 0;
        CHECK(infw_table_delete_batch(a.c, keys.data(), 200, &done) == 0 && done == 200);
        CHECK(infw_table_delete_batch(a.c, keys.data() + 199, 2, &done) == -ENOENT && done == 0);
        keys.erase(keys.begin(), keys.begin() + 200);
        CHECK(infw_table_count(a.c, &count) == 0 && count == keys.size());
    }
    rulesVal_st got;
    for (int i = 0; i < 500; i++) CHECK(infw_table_lookup(a.c, &keys[rnd() % keys.size()], &got) == 0);
    CHECK(infw_debug_walk(a.c, nullptr, 1, nullptr) == -EINVAL);
    CHECK(infw_table_commit(a.c) == 0);
    struct infw_table_info info;
    CHECK(infw_table_info(a.c, &info) == 0 && info.commit_mode == INFW_COMMIT_FULL && info.n_entries == count);
    const std::vector<uint32_t> tup = tuples(keys, 20000);
    std::vector<uint32_t> ra, rb;
    if (walk(a.c, tup, ra)) return 1;
    if (edit(a.c, keys, vals, 300)) return 1;
    CHECK(infw_table_commit(a.c) == 0);
    CHECK(infw_table_info(a.c, &info) == 0);
    printf("second commit: mode %u (%s)\n", info.commit_mode, info.full_reason);
    // no device on a host-only context
    CHECK(infw_classify(a.c, 0, nullptr, 1, nullptr, nullptr, nullptr) != 0);

    // images: export -> import -> the same bytes and walks; incremental edits keep them equal
    std::vector<uint8_t> img, img_b;
    if (export_image(a.c, img)) return 1;
    Ctx b(1u << 16);
    CHECK(infw_table_import(b.c, img.data(), img.size()) == 0);
    if (export_image(b.c, img_b)) return 1;
    CHECK(img_b == img);
    if (walk(a.c, tup, ra) || walk(b.c, tup, rb)) return 1;
    CHECK(ra == rb);
    for (int round = 0; round < 3; round++) {
        const uint64_t seed = rs;
        std::vector<lpm_ip_key_st> ka = keys, kb = keys;
        if (edit(a.c, ka, vals, 150)) return 1;
        rs = seed;  // the same edits on the importer
        if (edit(b.c, kb, vals, 150)) return 1;
        keys = ka;
        CHECK(infw_table_commit(a.c) == 0 && infw_table_commit(b.c) == 0);
        const std::vector<uint32_t> t2 = tuples(keys, 5000);
        if (walk(a.c, t2, ra) || walk(b.c, t2, rb)) return 1;
        CHECK(ra == rb);
    }

    // corrupt images, one flipped bit at a time: every header byte and 1024 payload bytes spread over every section of
    // an image in the compressed short-table form (small: a fresh copy per flip stays cheap), and 64 payload bytes of
    // the DIR-24-8 image above (128 MiB of tbl24 words per interface)
    size_t refused = 0;
    auto flips = [&](const std::vector<uint8_t> &im, size_t n_payload, bool header) -> int {
        std::vector<size_t> pos;
        if (header)
            for (size_t p = 0; p < 72; p++) pos.push_back(p);
        for (size_t j = 0; j < n_payload; j++) pos.push_back(72 + (im.size() - 73) * j / (n_payload - 1));
        std::vector<uint8_t> bad = im;
        for (size_t p : pos) {
            bad[p] ^= (uint8_t)(1u << (p % 8));
            Ctx c(1u << 16);
            CHECK(infw_table_import(c.c, bad.data(), bad.size()) == -EINVAL);
            CHECK(infw_table_count(c.c, &count) == 0 && count == 0);
            CHECK(infw_table_info(c.c, &info) == 0 && info.epoch == 0);  // nothing installed
            bad[p] = im[p];
            refused++;
        }
        return 0;
    };
    std::vector<uint8_t> small_img;
    {
        Ctx s(1u << 16);
        std::vector<uint32_t> vi(keys.size());
        for (auto &x : vi) x = rnd() % vals.size();
        CHECK(infw_table_update_batch(s.c, keys.data(), vals.data(), vi.data(), keys.size(), 0, nullptr) == 0);
        CHECK(infw_set_option(s.c, "short_table", 1) == 0);
        const int rc = infw_table_commit(s.c);
        CHECK(rc == 0 && infw_table_info(s.c, &info) == 0 && info.short_mode == 1);
        if (export_image(s.c, small_img)) return 1;
    }
    if (flips(small_img, 1024, true) || flips(img, 64, false)) return 1;
    for (size_t len : {img.size() - 1, (size_t)72, (size_t)71, (size_t)0}) {
        Ctx c(1u << 16);
        CHECK(infw_table_import(c.c, img.data(), len) == -EINVAL);
    }
    {
        std::vector<uint8_t> longer = img;
        longer.push_back(0);
        Ctx c(1u << 16);
        CHECK(infw_table_import(c.c, longer.data(), longer.size()) == -EINVAL);
    }
    // a busy context refuses; one emptied by deletes and a commit accepts (its value pool is dropped)
    CHECK(infw_table_import(a.c, img.data(), img.size()) == -EBUSY);
    {
        Ctx d(1u << 16);
        for (int i = 0; i < 50; i++) CHECK(infw_table_update(d.c, &keys[i], &vals[i % vals.size()], 0) == 0);
        CHECK(infw_table_commit(d.c) == 0);
        for (int i = 0; i < 50; i++) CHECK(infw_table_delete(d.c, &keys[i]) == 0);
        CHECK(infw_table_import(d.c, img.data(), img.size()) == -EBUSY);  // uncommitted deletes
        CHECK(infw_table_commit(d.c) == 0);
        CHECK(infw_table_import(d.c, img.data(), img.size()) == 0);
        std::vector<uint8_t> img_d;
        if (export_image(d.c, img_d)) return 1;
        CHECK(img_d == img);
    }
    // options: unknown names and out-of-range values are refused and change nothing; every listed option reads back
    {
        Ctx o(1u << 10);
        int64_t v = 0;
        CHECK(infw_set_option(o.c, "no_such_option", 1) == -EINVAL);
        CHECK(infw_set_option(o.c, nullptr, 1) == -EINVAL);
        CHECK(infw_set_option(o.c, "dt_parts", 3) == -EINVAL);
        CHECK(infw_set_option(o.c, "split", 2) == -EINVAL);
        CHECK(infw_set_option(o.c, "stat_flush_tiles", 0) == -EINVAL);
        CHECK(infw_get_option(o.c, "split", &v) == 0 && v == -1);
        CHECK(infw_get_option(o.c, "stat_flush_tiles", &v) == 0 && v == 1024);
        CHECK(infw_set_option(o.c, "dt_parts", 8) == 0 && infw_get_option(o.c, "dt_parts", &v) == 0 && v == 8);
        int n_opt = 0;
        for (; infw_option_name(n_opt); n_opt++) CHECK(infw_get_option(o.c, infw_option_name(n_opt), &v) == 0);
        CHECK(n_opt == 12);
        char name[256];
        CHECK(infw_classify_variant(o.c, 0, INFW_INPUT_SOA, 0, name, sizeof name) == 0);
        CHECK(infw_classify_variant(o.c, 0, INFW_INPUT_SOA, 0, name, 4) == -ERANGE);
        CHECK(infw_classify_variant(o.c, 0, 7, 0, name, sizeof name) == -EINVAL);
    }
    printf("asan_abi: %zu keys, images %zu / %zu bytes, %zu corrupt images refused\nok\n", keys.size(), img.size(),
           small_img.size(), refused);
    return 0;
}

static int import_file(const char *path) {
    FILE *f = fopen(path, "rb");
    if (!f) {
        perror(path);
        return 2;
    }
    std::vector<uint8_t> buf;
    uint8_t chunk[1 << 16];
    size_t n;
    while ((n = fread(chunk, 1, sizeof chunk, f)) > 0) buf.insert(buf.end(), chunk, chunk + n);
    fclose(f);
    Ctx c(1u << 22);
    if (c.rc) return 2;
    const int rc = infw_table_import(c.c, buf.data(), buf.size());
    uint64_t count = 0;
    infw_table_count(c.c, &count);
    printf("rc=%d count=%llu %s\n", -rc, (unsigned long long)count, rc ? infw_last_error() : "");
    return 0;
}

int main(int argc, char **argv) {
    if (argc == 3 && !strcmp(argv[1], "import")) return import_file(argv[2]);
    return selftest();
}
