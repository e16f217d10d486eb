// patch_bench.cpp — host cost of incremental commits without a GPU: the pending-map edits
// (update / delete, as infw_table_update_batch / _delete_batch apply them) and patch_tables, per phase, on a
// BASELINE workload's full table.  Build: make patch_bench; run: build/patch_bench [cfg] [edits] [rounds]
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <random>
#include <string>
#include <vector>

#include "../ingress-node-firewall_amd/csrc/infw_internal.h"
#include "../ingress-node-firewall_amd/csrc/workload.h"

namespace infw {
void set_error(const std::string &) {}
}  // namespace infw
using namespace infw;

static double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main(int argc, char **argv) {
    const int cfg = argc > 1 ? atoi(argv[1]) : 4;
    const int edits = argc > 2 ? atoi(argv[2]) : 1000;
    const int rounds = argc > 3 ? atoi(argv[3]) : 20;
    infw_wl *wl;
    if (infw_wl_create(&wl, cfg, 0x1F000000ull + cfg, 0, 0)) return 1;
    const uint64_t ne = infw_wl_n_entries(wl);
    const lpm_ip_key_st *keys = infw_wl_keys(wl);
    const uint32_t *vi = infw_wl_val_index(wl);
    const rulesVal_st *tv = infw_wl_templates(wl);
    const uint32_t nt = infw_wl_n_templates(wl);
    PendingMap m;
    m.max_entries = (uint32_t)ne + 65536;
    for (uint64_t i = 0; i < ne; i++) m.update(&keys[i], reinterpret_cast<const uint8_t *>(&tv[vi[i]]), 0);
    HostTables h;
    IncState inc;
    auto t = std::chrono::steady_clock::now();
    if (compile_tables(m, h, Options(), &inc)) return 1;
    printf("cfg%d: %zu entries, compile %.0f ms\n", cfg, m.nodes.size(), ms_since(t));
    m.clear_dirty();
    std::mt19937_64 rng(7);
    std::vector<double> upd, del, pat;
    std::vector<uint32_t> vids(nt);
    for (uint32_t j = 0; j < nt; j++) vids[j] = m.pool.intern(reinterpret_cast<const uint8_t *>(&tv[j]));
    auto micro = [&]() {  // node lookups alone: one after the other, and pipelined as the batch calls run them
        if (!getenv("PB_MICRO")) return;
        std::vector<uint64_t> idx(edits);
        double tf = 0, tp = 0;
        uint64_t found = 0;
        for (int r = 0; r < rounds; r++) {
            for (auto &x : idx) x = rng() % ne;
            for (int pass = 0; pass < 2; pass++) {
                t = std::chrono::steady_clock::now();
                for (int k = 0; k < edits; k++) {
                    if (pass && k + 16 < edits) m.prefetch_slot(&keys[idx[k + 16]]);
                    if (pass && k + 8 < edits) m.prefetch_node(&keys[idx[k + 8]]);
                    found += m.lookup(&keys[idx[k]], nullptr) == 0;
                }
                double &d = pass ? tp : tf;
                d = r ? std::min(d, ms_since(t)) : ms_since(t);
            }
        }
        printf("micro: %d lookups %.3f ms, pipelined %.3f ms (%llu found)\n", edits, tf, tp, (unsigned long long)found);
    };
    micro();
    for (int r = 0; r < rounds; r++) {
        std::vector<uint64_t> idx(edits);
        for (auto &x : idx) x = rng() % ne;
        t = std::chrono::steady_clock::now();
        for (int k = 0; k < edits / 16; k++) {  // as infw_table_delete_batch / _update_batch run them
            if (k + 16 < edits / 16) m.prefetch_slot(&keys[idx[k + 16]]);
            if (k + 8 < edits / 16) m.prefetch_node(&keys[idx[k + 8]]);
            m.remove(&keys[idx[k]]);
        }
        del.push_back(ms_since(t));
        t = std::chrono::steady_clock::now();
        for (int k = 0; k < edits; k++) {
            if (k + 16 < edits) m.prefetch_slot(&keys[idx[k + 16]]);
            if (k + 8 < edits) m.prefetch_node(&keys[idx[k + 8]]);
            m.update_vid(&keys[idx[k]], vids[rng() % nt], 0);
        }
        upd.push_back(ms_since(t));
        std::vector<DirtyRange> ranges;
        std::string why;
        t = std::chrono::steady_clock::now();
        Options po;
        if (getenv("PB_TRACE")) po.trace = 2;  // the patch's per-phase trace (option trace, bit 2)
        const int rc = patch_tables(m, h, inc, ranges, &why, po);
        pat.push_back(ms_since(t));
        if (rc == 1) {  // the edit needs a full compile (counted apart)
            printf("round %d: full compile (%s)\n", r, why.c_str());
            pat.pop_back();
            h = HostTables();
            inc = IncState();
            if (compile_tables(m, h, Options(), &inc)) return 1;
        } else if (rc) {
            printf("round %d: patch rc %d\n", r, rc);
            return 1;
        }
        m.clear_dirty();
    }
    micro();
    auto med = [](std::vector<double> v) {
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    printf("%d edits/commit (%d deletes): update %.3f ms, delete %.3f ms, patch %.3f ms (medians of %d)\n", edits,
           edits / 16, med(upd), med(del), med(pat), rounds);
    infw_wl_destroy(wl);
    return 0;
}
