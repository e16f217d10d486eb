// tsan_hostpool.cpp — the packer pool of infw_classify_xdp_host (csrc/hostfeed.cpp, HostPackPool) without a device,
// under ThreadSanitizer (make tsan-host; tests/test_threads_cpu.py runs it).
//
// The calling thread plays the coordinator of abi.cpp xdp_host_chunks: it starts a job of ragged chunks over three
// host slots, waits for chunk k to be packed, checks the slot's streams against the packer run on the calling thread
// over the same descriptors (infw_hostpack_xdp, the bytes infw_pack_xdp_host writes), and then releases chunk k + 3
// into the slot it has just freed — for several thread counts and chunk sizes, jobs back to back on one pool (the
// signals only grow across jobs), and a job aborted half-way (end(true): no worker may still touch the job after).
// Prints "tsan_hostpool OK ..." and exits 0.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "../ingress-node-firewall_amd/csrc/infw_hostfeed.h"

#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

namespace {

constexpr uint64_t kStride = 2048;
constexpr int kSlots = 3;

struct Slot {  // one chunk's family-compact streams (the layout of abi.cpp XdpPipe::slot_out)
    std::vector<uint8_t> b;
    uint64_t C;
    explicit Slot(uint64_t c) : b(28 * c), C(c) {}
    infw_hostpack_out out() {
        uint8_t *p = b.data();
        return {reinterpret_cast<uint32_t *>(p), p + 16 * C, nullptr, reinterpret_cast<uint32_t *>(p + 4 * C),
                reinterpret_cast<uint32_t *>(p + 8 * C), reinterpret_cast<uint32_t *>(p + 12 * C)};
    }
};

// The slot's first n packets against the calling thread's packing of the same descriptors.
void compare(Slot &got, const infw::XdpChunk &c, Slot &ref) {
    const infw_hostpack_out r = ref.out(), g = got.out();
    infw_hostpack_xdp<16, false>(c.umem, c.descs, c.n, c.ifindex, r);
    CHECK(memcmp(g.saddr4, r.saddr4, 4 * c.n) == 0);
    CHECK(memcmp(g.pkt_len, r.pkt_len, 4 * c.n) == 0);
    CHECK(memcmp(g.meta, r.meta, 4 * c.n) == 0);
    CHECK(memcmp(g.l4word, r.l4word, 4 * c.n) == 0);
    for (uint64_t grp = 0; grp * INFW_V6_GROUP < c.n; grp++) {  // the tails the group's IPv6 packets own
        uint64_t v6 = 0;
        for (uint64_t i = grp * INFW_V6_GROUP; i < c.n && i < (grp + 1) * INFW_V6_GROUP; i++)
            v6 += (r.meta[i] & 0xFFFFu) == 0x86DDu;
        CHECK(memcmp(g.v6tail + grp * 12 * INFW_V6_GROUP, r.v6tail + grp * 12 * INFW_V6_GROUP, 12 * v6) == 0);
    }
}

}  // namespace

int main() {
    // umem: F frames of random header bytes with IPv4 / IPv6 / ARP ethertypes, 1 % shorter than 58 B (the packer's
    // slow path); rings of ragged sizes over shuffled frames, unaligned-mode offsets on some
    const uint64_t F = 60000;
    std::vector<uint8_t> umem(F * kStride + 4096);
    std::mt19937_64 g(7);
    for (uint64_t f = 0; f < F; f++) {
        uint8_t *h = umem.data() + f * kStride;
        for (int b = 0; b < 80; b++) h[b] = (uint8_t)g();
        const uint32_t k = g() % 100;
        const uint16_t et = k < 60 ? 0x0800 : k < 97 ? 0x86DD : 0x0806;
        h[12] = et >> 8, h[13] = et & 0xFF;
    }
    const uint64_t ring_sizes[] = {0, 1, 63, 4097, 20000, 35000 - 1};
    std::vector<std::vector<infw_xdp_desc>> rings;
    for (uint64_t sz : ring_sizes) {
        std::vector<infw_xdp_desc> d(sz);
        for (auto &x : d) {
            const uint64_t f = g() % F, off = (g() % 4 == 0) ? (g() % 512) : 0;
            x.addr = f * kStride | off << 48;
            x.len = g() % 100 == 0 ? (uint32_t)(g() % 58) : 60 + (uint32_t)(g() % 1400);
            x.options = 0;
        }
        rings.push_back(std::move(d));
    }
    uint64_t jobs = 0, chunks_checked = 0;
    for (int threads : {1, 2, 3, 8}) {
        infw::HostPackPool pool(threads);
        for (uint64_t C : {512ull, 4096ull, 8192ull + 512}) {
            for (int abort_at : {-1, 3}) {
                std::vector<infw::XdpChunk> chunks;  // as infw_classify_xdp_host cuts the rings
                for (size_t r = 0; r < rings.size(); r++)
                    for (uint64_t a = 0; a < rings[r].size(); a += C)
                        chunks.push_back({umem.data(), rings[r].data() + a, std::min(C, rings[r].size() - a),
                                          (uint32_t)(10 + r)});
                std::vector<Slot> slots(kSlots, Slot(C));
                Slot ref(C);
                std::vector<infw_hostpack_out> outs;
                for (auto &s : slots) outs.push_back(s.out());
                const uint64_t K = chunks.size();
                pool.begin(&chunks, outs, std::min<uint64_t>(K, kSlots));
                bool aborted = false;
                for (uint64_t k = 0; k < K; k++) {
                    if ((int64_t)k == abort_at) {
                        aborted = true;
                        break;
                    }
                    pool.wait_packed(k);
                    compare(slots[k % kSlots], chunks[k], ref);
                    chunks_checked++;
                    pool.release(k + kSlots + 1);  // slot k % 3 is free again: chunk k + 3 may fill it
                }
                pool.end(aborted);
                jobs++;
            }
        }
    }
    printf("tsan_hostpool OK: %llu jobs, %llu chunks checked against the calling thread's packing\n",
           (unsigned long long)jobs, (unsigned long long)chunks_checked);
    return 0;
}
