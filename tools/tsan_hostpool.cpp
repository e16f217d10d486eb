// tsan_hostpool.cpp — the packer pool of infw_classify_xdp_host (csrc/hostfeed.cpp, HostPackPool) without a device,
// under ThreadSanitizer (make tsan-host; tests/test_threads_cpu.py runs it).
//
// The calling thread plays the coordinator of abi.cpp xdp_host_chunks: it cuts ragged rings into chunks that run on
// from one ring into the next (chunks of several interfaces: the packers write the ifindex stream, and a group may
// start in one ring's segment and end in the next's), starts a job over three host slots, packs units itself until
// chunk k is packed, checks the slot's streams against infw_pack_header on every descriptor, and then releases chunk
// k + 3 into the slot it has just freed — for several thread counts and chunk sizes, jobs back to back on one pool
// (small ones wake no worker), and a job aborted half-way (end(true): no worker may still touch the job after).
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

// The chunk's streams against infw_pack_header (infw_pack.h: what kernel.c reads) on every descriptor, position by
// position; the v6tail blocks hold each group's IPv6 packets' address bytes 4..15 in position order.
void check_chunk(const infw::XdpChunk &c, const std::vector<infw::XdpSeg> &segs) {
    std::vector<uint32_t> tails;
    uint64_t group = 0;
    auto flush = [&]() {
        CHECK(memcmp(c.out.v6tail + group * 12 * INFW_V6_GROUP, tails.data(), 4 * tails.size()) == 0);
        tails.clear();
    };
    for (uint32_t si = c.seg0; si < c.seg1; si++) {
        const infw::XdpSeg &g = segs[si];
        for (uint64_t i = 0; i < g.n; i++) {
            const uint64_t p = g.pos + i;
            if (p / INFW_V6_GROUP != group) {
                flush();
                group = p / INFW_V6_GROUP;
            }
            const infw_xdp_desc &d = g.descs[i];
            infw_tuple t;
            infw_pack_header(infw_xdp_frame(g.umem, d.addr), d.len, d.len, g.ifindex, &t);
            CHECK(c.out.saddr4[p] == t.saddr[0] && c.out.meta[p] == t.meta && c.out.l4word[p] == t.l4word &&
                  c.out.pkt_len[p] == d.len);
            if (c.mixed) CHECK(c.out.ifindex[p] == g.ifindex);
            if ((t.meta & 0xFFFFu) == 0x86DDu) tails.insert(tails.end(), {t.saddr[1], t.saddr[2], t.saddr[3]});
        }
    }
    flush();
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
    uint64_t jobs = 0, chunks_checked = 0, mixed = 0;
    for (int threads : {1, 2, 3, 8}) {
        infw::HostPackPool pool(threads);
        for (uint64_t C : {512ull, 4096ull, 8192ull + 512}) {
            for (int abort_at : {-1, 3}) {
                // the rings cut as infw_classify_xdp_host cuts them: chunks of C running on from ring to ring
                std::vector<infw::XdpSeg> segs;
                std::vector<infw::XdpChunk> chunks;
                for (size_t r = 0; r < rings.size(); r++)
                    for (uint64_t a = 0; a < rings[r].size();) {
                        if (chunks.empty() || chunks.back().n == C)
                            chunks.push_back({(uint32_t)segs.size(), (uint32_t)segs.size(), 0, false, {}});
                        infw::XdpChunk &c = chunks.back();
                        const uint64_t take = std::min(C - c.n, rings[r].size() - a);
                        c.mixed |= c.seg1 > c.seg0 && segs[c.seg0].ifindex != 10 + r;
                        segs.push_back({umem.data(), rings[r].data() + a, take, c.n, (uint32_t)(10 + r)});
                        c.seg1++, c.n += take, a += take;
                    }
                std::vector<std::vector<uint8_t>> slots(kSlots, std::vector<uint8_t>(32 * C));
                for (size_t k = 0; k < chunks.size(); k++) {  // the slot layout of abi.cpp, stride S
                    const uint64_t S = (chunks[k].n + 63) & ~63ull;
                    uint8_t *b = slots[k % kSlots].data();
                    chunks[k].out = {reinterpret_cast<uint32_t *>(b), b + 16 * S, reinterpret_cast<uint32_t *>(b + 28 * S),
                                     reinterpret_cast<uint32_t *>(b + 4 * S), reinterpret_cast<uint32_t *>(b + 8 * S),
                                     reinterpret_cast<uint32_t *>(b + 12 * S)};
                    mixed += chunks[k].mixed;
                }
                const uint64_t K = chunks.size();
                pool.begin(&chunks, &segs, std::min<uint64_t>(K, kSlots));
                bool aborted = false;
                for (uint64_t k = 0; k < K; k++) {
                    if ((int64_t)k == abort_at) {
                        aborted = true;
                        break;
                    }
                    pool.help_until_packed(k);  // the coordinator packs too
                    check_chunk(chunks[k], segs);
                    chunks_checked++;
                    pool.release(k + kSlots + 1);  // slot k % 3 is free again: chunk k + 3 may fill it
                }
                pool.end(aborted);
                jobs++;
                // small calls right behind it, while workers may still be waking for the last job: one chunk of a
                // 1-descriptor and a 63-descriptor ring (one unit, no worker woken), packed by the coordinator
                for (int rep = 0; rep < 20; rep++) {
                    std::vector<infw::XdpSeg> ss = {{umem.data(), rings[1].data(), 1, 0, 11},
                                                    {umem.data(), rings[2].data(), 63, 1, 12}};
                    std::vector<infw::XdpChunk> cc = {{0, 2, 64, true, {}}};
                    uint8_t *b = slots[0].data();
                    cc[0].out = {reinterpret_cast<uint32_t *>(b), b + 16 * 64, reinterpret_cast<uint32_t *>(b + 28 * 64),
                                 reinterpret_cast<uint32_t *>(b + 4 * 64), reinterpret_cast<uint32_t *>(b + 8 * 64),
                                 reinterpret_cast<uint32_t *>(b + 12 * 64)};
                    pool.begin(&cc, &ss, 1);
                    pool.help_until_packed(0);
                    check_chunk(cc[0], ss);
                    pool.end(false);
                    jobs++, chunks_checked++, mixed++;
                }
            }
        }
    }
    printf("tsan_hostpool OK: %llu jobs, %llu chunks (%llu of several interfaces) checked against infw_pack_header\n",
           (unsigned long long)jobs, (unsigned long long)chunks_checked, (unsigned long long)mixed);
    return 0;
}
