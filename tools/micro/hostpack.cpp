// Microbenchmark: the host packer of infw_classify_xdp_host (csrc/infw_hostpack.h) alone, on the CPU.
//
// An AF_XDP-style umem of 2048-B chunks holding synthetic Ethernet/IPv4/IPv6 headers (60 % IPv4, 38 % IPv6, 2 % ARP;
// 1 % of frames shorter than 58 B), one RX descriptor per frame, and T threads each packing a contiguous 1/T of the
// descriptors into the family-compact streams — what one chunk of infw_classify_xdp_host does on the host.  Sweeps
// threads x prefetch distance x store kind (4-B non-temporal stores: pf16nt), with the umem on 4-KiB pages or transparent huge pages, and reports
// Mframes/s.  The umem is much larger than the last-level cache, so every header is a DRAM miss, as after a NIC's DMA.
// Output streams (--out): malloc'd memory (vector), hipHostMalloc'd (pinned: what libinfw's slots are) or malloc'd and
// hipHostRegister'ed; input order (--keep K): every frame in address order (1), or each frame kept with probability
// 1/K — one interface's ring out of K, addresses ascending with gaps — and --shuffle: a fill ring's arbitrary order.
//   hipcc -O3 -std=c++17 -pthread -Iinclude tools/micro/hostpack.cpp -o tools/micro/hostpack && tools/micro/hostpack
//   options: --umem-gib G (8)  --descs M (16, millions)  --threads 1,2,4,8,16  --shuffle  --keep K  --out vector|pinned|registered
//            --thp 0|1|2 (4-KiB pages, huge pages, both: 2)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../ingress-node-firewall_amd/csrc/infw_hostpack.h"

using Fn = void (*)(const uint8_t *, const infw_xdp_desc *, uint64_t, uint32_t, const infw_hostpack_out &);

template <int kPF, bool kNT>
static void packer(const uint8_t *u, const infw_xdp_desc *d, uint64_t n, uint32_t ifx, const infw_hostpack_out &o) {
    infw_hostpack_xdp<kPF, kNT>(u, d, n, ifx, o);
}

// The streams in one allocation: saddr4, ifindex, pkt_len, meta, l4word (4n B each), v6tail (12 B per packet)
struct Streams {
    uint8_t *base = nullptr;
    uint64_t n;
    std::string kind;
    Streams(uint64_t n_, const std::string &k) : n(n_), kind(k) {
        const size_t bytes = 20 * n + (n + 63) / 64 * 768;
        if (kind == "pinned") {
            if (hipHostMalloc(reinterpret_cast<void **>(&base), bytes, hipHostMallocDefault) != hipSuccess) abort();
        } else {
            base = static_cast<uint8_t *>(aligned_alloc(4096, (bytes + 4095) & ~size_t(4095)));
            if (kind == "registered" && hipHostRegister(base, bytes, hipHostRegisterDefault) != hipSuccess) abort();
        }
        memset(base, 0, bytes);
    }
    ~Streams() {
        if (kind == "pinned") (void)hipHostFree(base);
        else {
            if (kind == "registered") (void)hipHostUnregister(base);
            free(base);
        }
    }
    uint32_t *st(int i) const { return reinterpret_cast<uint32_t *>(base) + i * n; }
    uint32_t *saddr4() const { return st(0); }
    uint32_t *pkt_len() const { return st(2); }
    uint32_t *meta() const { return st(3); }
    uint32_t *l4word() const { return st(4); }
    infw_hostpack_out part(uint64_t a) {
        return {st(0) + a, base + 20 * n + a / 64 * 768, st(1) + a, st(2) + a, st(3) + a, st(4) + a};
    }
};

static double run(Fn fn, const uint8_t *umem, const infw_xdp_desc *d, uint64_t n, Streams &s, int threads) {
    const uint64_t per = (n / threads + 63) & ~63ull;
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
        const uint64_t a = std::min<uint64_t>(n, t * per), b = std::min<uint64_t>(n, a + per);
        th.emplace_back([=, &s] { fn(umem, d + a, b - a, 7, s.part(a)); });
    }
    for (auto &x : th) x.join();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

int main(int argc, char **argv) {
    double umem_gib = 8;
    uint64_t descs_m = 16;
    bool shuffle = false;
    uint64_t keep = 1;
    int thp = 1;
    std::string out = "vector";
    std::vector<int> threads = {1, 2, 4, 8, 16};
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        if (a == "--umem-gib" && i + 1 < argc) umem_gib = atof(argv[++i]);
        else if (a == "--descs" && i + 1 < argc) descs_m = strtoull(argv[++i], nullptr, 10);
        else if (a == "--shuffle") shuffle = true;
        else if (a == "--keep" && i + 1 < argc) keep = strtoull(argv[++i], nullptr, 10);
        else if (a == "--out" && i + 1 < argc) out = argv[++i];
        else if (a == "--thp" && i + 1 < argc) thp = atoi(argv[++i]);
        else if (a == "--threads" && i + 1 < argc) {
            threads.clear();
            for (char *p = argv[++i]; *p;) {
                threads.push_back((int)strtol(p, &p, 10));
                if (*p == ',') p++;
            }
        }
    }
    const uint64_t stride = 2048, frames = (uint64_t)(umem_gib * (1ull << 30)) / stride, n = descs_m << 20;
    Streams s(n, out);
    std::vector<infw_xdp_desc> d(n);
    std::mt19937_64 rng(0x1F00);
    std::vector<uint64_t> slot;
    for (uint64_t i = 0; i < frames; i++)
        if (keep <= 1 || rng() % keep == 0) slot.push_back(i);
    if (shuffle) std::shuffle(slot.begin(), slot.end(), rng);
    for (int huge = thp == 2 ? 0 : thp; huge < (thp == 2 ? 2 : thp + 1); huge++) {
        const size_t bytes = frames * stride;
        auto *umem = static_cast<uint8_t *>(mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
        if (umem == MAP_FAILED) return 1;
        int adv = madvise(umem, bytes, huge ? MADV_HUGEPAGE : MADV_NOHUGEPAGE);
        std::mt19937_64 g(0x1F01);
        std::vector<uint32_t> lens(frames);
        for (uint64_t f = 0; f < frames; f++) {  // headers only: the first 64 B of every chunk
            uint8_t *h = umem + f * stride;
            const uint64_t r = g();
            const uint32_t kind = r % 100;
            const uint16_t et = kind < 60 ? 0x0800 : kind < 98 ? 0x86DD : 0x0806;
            h[12] = et >> 8, h[13] = et & 0xFF;
            for (int b = 14; b < 64; b++) h[b] = (uint8_t)(g() >> 7);
            static const uint8_t protos[] = {6, 17, 1, 58, 132};
            h[23] = h[20] = protos[(r >> 8) % 5];
            lens[f] = (r >> 16) % 100 == 0 ? 14 + (uint32_t)((r >> 24) % 44) : 64 + (uint32_t)((r >> 24) % 1451);
        }
        for (uint64_t i = 0; i < n; i++) {
            const uint64_t f = slot[i % slot.size()];
            d[i] = infw_xdp_desc{f * stride, lens[f], 0};
        }
        // spot check of the branch-free form against infw_pack_header on the first 64k frames
        run(packer<16, false>, umem, d.data(), 1 << 16, s, 1);
        uint64_t bad = 0;
        for (uint64_t i = 0; i < (1u << 16); i++) {
            infw_tuple t;
            infw_pack_header(infw_xdp_frame(umem, d[i].addr), d[i].len, d[i].len, 7, &t);
            bad += t.saddr[0] != s.saddr4()[i] || t.meta != s.meta()[i] || t.l4word != s.l4word()[i] ||
                   s.pkt_len()[i] != d[i].len;
        }
        printf("{\"umem_gib\": %.1f, \"descs\": %llu, \"thp\": %d, \"madvise_rc\": %d, \"shuffle\": %d, \"keep\": %llu, "
               "\"distinct_frames\": %zu, \"out\": \"%s\", \"check_mismatches\": %llu}\n",
               umem_gib, (unsigned long long)n, huge, adv, shuffle ? 1 : 0, (unsigned long long)keep, slot.size(),
               out.c_str(), (unsigned long long)bad);
        fflush(stdout);
        struct V {
            const char *name;
            Fn fn;
        } vs[] = {{"pf0", packer<0, false>},   {"pf8", packer<8, false>},   {"pf16", packer<16, false>},
                  {"pf32", packer<32, false>}, {"pf64", packer<64, false>}, {"pf128", packer<128, false>},
                  {"pf16nt", packer<16, true>}, {"pf64nt", packer<64, true>}};
        for (int t : threads) {
            std::string line = "{\"thp\": " + std::to_string(huge) + ", \"out\": \"" + out + "\", \"keep\": " +
                               std::to_string(keep) + ", \"shuffle\": " + std::to_string(shuffle ? 1 : 0) +
                               ", \"threads\": " + std::to_string(t);
            for (const V &v : vs) {
                run(v.fn, umem, d.data(), n, s, t);  // warm the output pages
                double best = 1e9;
                for (int r = 0; r < 2; r++) best = std::min(best, run(v.fn, umem, d.data(), n, s, t));
                char buf[96];
                snprintf(buf, sizeof buf, ", \"%s_Mpps\": %.1f", v.name, n / best / 1e6);
                line += buf;
            }
            printf("%s}\n", line.c_str());
            fflush(stdout);
        }
        munmap(umem, bytes);
    }
    return 0;
}
