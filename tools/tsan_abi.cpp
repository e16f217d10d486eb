// ThreadSanitizer driver of the C ABI's threading contract (include/infw.h "threads"), linked against the TSan build
// of libinfw.so's host sources (make tsan-host; no GPU involved).  The reference keeps classifying on every CPU while
// its syncer edits and reloads the maps under e.mu (ebpfsyncer.go:62, 72-73); here, on one host-only context:
//   - one control-plane thread (the syncer) runs map edits single and batched, deletes, full and incremental commits,
//     option changes and launch-shape changes — serialised among themselves, as the contract asks;
//   - reader threads run, concurrently with it and with each other, the calls the contract lets run anywhere:
//     infw_debug_walk over the committed host image (the kernel's lookup code on the host), infw_table_info,
//     infw_stats_read / _read_all, infw_classify_variant, infw_get_option, infw_get_launch, infw_debug_keys_read.
// Each walk must see one committed epoch: the walked result words of a fixed packet set are checked to be one of the
// epochs' (the syncer commits known epochs, their walks recorded single-threaded first).  TSan reports any data race
// in the instrumented host code.  Prints "ok".
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <set>
#include <thread>
#include <vector>

#include "infw.h"

static std::atomic<int> failures{0};
#define CHECK(cond)                                                                                        \
    do {                                                                                                   \
        if (!(cond)) {                                                                                     \
            fprintf(stderr, "%s:%d: check failed: %s (last error: %s)\n", __FILE__, __LINE__, #cond,      \
                    infw_last_error());                                                                    \
            failures++;                                                                                    \
        }                                                                                                  \
    } while (0)

struct Rng {
    uint64_t s;
    uint32_t operator()() {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        return (uint32_t)(s >> 11);
    }
};

// A value of n rules through the makeIngressFwRulesMap encoder.
static void make_value(rulesVal_st *v, Rng &r, int n) {
    memset(v, 0, sizeof *v);
    for (int i = 0; i < n; i++) {
        char ports[32];
        const uint32_t a = 1 + r() % 60000;
        snprintf(ports, sizeof ports, "%u-%u", a, a + 1 + r() % 3000);
        const char *p = r() % 3 == 0 ? "UDP" : "TCP";
        (void)infw_make_rule(v, 1 + r() % 99, p, ports, 0, 0, r() % 2 ? "Allow" : "Deny");
    }
}

static lpm_ip_key_st make_key(Rng &r) {
    lpm_ip_key_st k;
    memset(&k, 0, sizeof k);
    k.ingress_ifindex = 1 + r() % 2;
    if (r() % 3) {  // IPv4 /8../32 under 10.0.0.0/8
        const uint32_t len = 8 + r() % 25;
        k.prefixLen = 32 + len;
        const uint32_t a = (10u << 24) | (r() & 0x00FFFFFFu);
        for (int b = 0; b < 4; b++) k.ip_data[b] = (uint8_t)(a >> (24 - 8 * b));
    } else {        // IPv6 /33../128 under 2001:db8::/32
        k.prefixLen = 32 + 33 + r() % 96;
        k.ip_data[0] = 0x20, k.ip_data[1] = 0x01, k.ip_data[2] = 0x0d, k.ip_data[3] = 0xb8;
        for (int b = 4; b < 16; b++) k.ip_data[b] = (uint8_t)r();
    }
    return k;
}

// Tuples {saddr[4], ifindex, pkt_len, meta, l4word} of TCP packets aimed at the keys.
static std::vector<uint32_t> make_tuples(const std::vector<lpm_ip_key_st> &keys, Rng &r, size_t n) {
    std::vector<uint32_t> t(8 * n, 0);
    for (size_t i = 0; i < n; i++) {
        const lpm_ip_key_st &k = keys[r() % keys.size()];
        uint32_t *q = &t[8 * i];
        const bool v6 = k.prefixLen > 64;
        memcpy(q, k.ip_data, 16);
        if (!v6) q[1] = q[2] = q[3] = 0;
        q[4] = k.ingress_ifindex;
        q[5] = 64 + r() % 1400;
        q[6] = INFW_META(v6 ? 0x86DD : 0x0800, 6, 255);
        const uint32_t port = r() % 65536;
        q[7] = (port >> 8 | (port & 0xFF) << 8) << 16;  // dest port, network order, at bytes 2..3
    }
    return t;
}

int main() {
    infw_ctx *c = nullptr;
    if (infw_create(&c, nullptr, 0, 1u << 16, INFW_F_HOST_ONLY)) {
        fprintf(stderr, "create failed: %s\n", infw_last_error());
        return 1;
    }
    Rng r{0x9E3779B97F4A7C15ull};
    const int kKeys = 2000, kEpochs = 8, kVals = 24;
    std::vector<rulesVal_st> vals(kVals);
    for (auto &v : vals) make_value(&v, r, 1 + r() % 20);
    std::vector<lpm_ip_key_st> keys;
    for (int i = 0; i < kKeys; i++) keys.push_back(make_key(r));
    // the epochs: epoch 0 = every key with value i % kVals; epoch e rewrites, deletes and re-adds a slice
    struct Edit {
        int key, val;  // val < 0: delete
    };
    std::vector<std::vector<Edit>> epochs(kEpochs);
    for (int i = 0; i < kKeys; i++) epochs[0].push_back({i, i % kVals});
    for (int e = 1; e < kEpochs; e++)
        for (int j = 0; j < 150; j++) epochs[e].push_back({(int)(r() % kKeys), r() % 4 == 0 ? -1 : (int)(r() % kVals)});
    const std::vector<uint32_t> tup = make_tuples(keys, r, 4096);
    const size_t nt = tup.size() / 8;
    // each epoch's walk, recorded single-threaded on a second context
    std::vector<std::vector<uint32_t>> want(kEpochs, std::vector<uint32_t>(nt));
    {
        infw_ctx *ref = nullptr;
        CHECK(infw_create(&ref, nullptr, 0, 1u << 16, INFW_F_HOST_ONLY | INFW_F_FULL_COMMIT) == 0);
        for (int e = 0; e < kEpochs; e++) {
            for (const Edit &x : epochs[e]) {
                if (x.val < 0) (void)infw_table_delete(ref, &keys[x.key]);
                else CHECK(infw_table_update(ref, &keys[x.key], &vals[x.val], INFW_BPF_ANY) == 0);
            }
            CHECK(infw_table_commit(ref) == 0);
            CHECK(infw_debug_walk(ref, tup.data(), nt, want[e].data()) == 0);
        }
        infw_destroy(ref);
    }
    std::set<std::vector<uint32_t>> known(want.begin(), want.end());
    known.insert(std::vector<uint32_t>(nt, 0));  // the empty epoch of a fresh context
    std::atomic<bool> done{false};
    std::atomic<uint64_t> walks{0}, reads{0};
    auto walker = [&](int id) {
        std::vector<uint32_t> got(nt);
        while (!done.load()) {
            CHECK(infw_debug_walk(c, tup.data(), nt, got.data()) == 0);
            CHECK(known.count(got) == 1);  // exactly one committed epoch's results
            walks++;
            (void)id;
        }
    };
    auto reader = [&]() {
        char name[256];
        ruleStatistics_st all[INFW_MAX_TARGETS], one[1];
        struct infw_table_info info;
        int64_t v;
        int b, g, p, ns;
        uint32_t nk;
        while (!done.load()) {
            CHECK(infw_table_info(c, &info) == 0);
            CHECK(infw_stats_read_all(c, all) == 0);
            CHECK(infw_stats_read(c, 7, one, &ns) == 0);
            CHECK(infw_classify_variant(c, 0, INFW_INPUT_SOA, 0, name, sizeof name) == 0);
            CHECK(infw_classify_variant(c, 0, INFW_INPUT_FRAMES, INFW_VARIANT_EVENTS, name, sizeof name) == 0);
            CHECK(infw_get_option(c, "split", &v) == 0);
            CHECK(infw_get_launch(c, &b, &g, &p) == 0);
            CHECK(infw_debug_keys_read(c, nullptr, 0, &nk) == 0);
            reads++;
        }
    };
    std::vector<std::thread> th;
    for (int i = 0; i < 3; i++) th.emplace_back(walker, i);
    th.emplace_back(reader);
    th.emplace_back(reader);
    // the syncer: every epoch's edits (batched for epoch 0, single calls after), a commit each, options and shapes
    // changed between commits
    for (int e = 0; e < kEpochs; e++) {
        if (e == 0) {
            std::vector<lpm_ip_key_st> ks;
            std::vector<uint32_t> vi;
            for (const Edit &x : epochs[0]) ks.push_back(keys[x.key]), vi.push_back((uint32_t)x.val);
            uint64_t n_done = 0;
            CHECK(infw_table_update_batch(c, ks.data(), vals.data(), vi.data(), ks.size(), INFW_BPF_ANY, &n_done) == 0);
        } else {
            for (const Edit &x : epochs[e]) {
                if (x.val < 0) (void)infw_table_delete(c, &keys[x.key]);
                else CHECK(infw_table_update(c, &keys[x.key], &vals[x.val], INFW_BPF_ANY) == 0);
            }
        }
        CHECK(infw_set_option(c, "split", e % 3 - 1) == 0);
        CHECK(infw_set_option(c, "dt_half", e % 2) == 0);  // read by the next full compile
        CHECK(infw_set_launch(c, e % 2 ? 512 : 768, 0, e % 2 ? 3 : 2) == 0);
        CHECK(infw_debug_lookup_set(c, e % 2) == 0);
        if (e == kEpochs / 2) CHECK(infw_set_option(c, "short_table", 1) == 0);  // the next full compile changes form
        CHECK(infw_table_commit(c) == 0);
        struct infw_table_info info;
        CHECK(infw_table_info(c, &info) == 0 && info.epoch == (uint64_t)e + 1);
        std::vector<uint32_t> got(nt);
        CHECK(infw_debug_walk(c, tup.data(), nt, got.data()) == 0 && got == want[e]);
    }
    done = true;
    for (auto &t : th) t.join();
    infw_destroy(c);
    printf("tsan_abi: %d epochs, %llu concurrent walks, %llu reader rounds\n", kEpochs, (unsigned long long)walks.load(),
           (unsigned long long)reads.load());
    if (failures.load()) {
        printf("FAILED (%d checks)\n", failures.load());
        return 1;
    }
    printf("ok\n");
    return 0;
}
