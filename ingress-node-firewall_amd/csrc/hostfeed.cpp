// hostfeed.cpp — the host packer threads of infw_classify_xdp_host (infw_hostfeed.h).
#include "infw_hostfeed.h"

#include <errno.h>
#include <string.h>

#include "../../include/infw_host.h"

#include <sched.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

// The packer's prefetch distance (frames) and store kind (non-temporal or not): build-time knobs for same-box A/Bs
// of two libraries (tools/hostfeed_ab.sh); the shipped library uses the defaults.
#ifndef INFW_PACK_PF
#define INFW_PACK_PF 16
#endif
#ifndef INFW_PACK_NT
#define INFW_PACK_NT 0
#endif

namespace infw {

void Signal::set(uint64_t v) {
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (v <= v_.load(std::memory_order_relaxed)) return;
        v_.store(v, std::memory_order_release);
    }
    cv_.notify_all();
}

void Signal::wait_at_least(uint64_t target) {
    // ~50 us of spinning covers the gap between two chunks of one call; past that the waiter sleeps
    for (int i = 0; i < 4096; i++) {
        if (get() >= target) return;
#if defined(__x86_64__)
        _mm_pause();
#endif
    }
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return get() >= target; });
}

HostPackPool::HostPackPool(int threads) : n_threads_(threads) {
    workers_.reserve(threads);
    for (int t = 0; t < threads; t++) workers_.emplace_back([this] { work(); });
}

HostPackPool::~HostPackPool() {
    quit_.store(true);
    job_.set(gen_ + 1);
    for (auto &w : workers_) w.join();
}

void HostPackPool::begin(const std::vector<XdpChunk> *chunks, const std::vector<XdpSeg> *segs, uint64_t released) {
    // closed_ is set: no worker reads the fields below while they are written
    chunks_ = chunks;
    segs_ = segs;
    const size_t K = chunks->size();
    unit_base_.assign(K + 1, 0);
    for (size_t k = 0; k < K; k++)
        unit_base_[k + 1] = unit_base_[k] + std::max<uint64_t>(1, ((*chunks)[k].n + kPackUnit - 1) / kPackUnit);
    done_.reset(new std::atomic<uint32_t>[std::max<size_t>(K, 1)]());
    next_unit_.store(0);
    frontier_ = 0;
    abort_.store(false);
    pack_ns_.store(0);
    release_wait_ns_.store(0);
    released_.set(base_ + released);
    closed_.store(false, std::memory_order_seq_cst);  // publishes the job to workers that check it
    if (unit_base_.back() > 2) job_.set(++gen_);        // a call of one or two units wakes no worker
}

void HostPackPool::end(bool abort) {
    if (abort) {
        abort_.store(true);
        released_.set(base_ + chunks_->size());
    }
    closed_.store(true, std::memory_order_seq_cst);
    // a worker inside the job finishes at most the unit it holds; one that arrives now sees closed_ and leaves
    for (int i = 0; active_.load(std::memory_order_seq_cst) != 0; i++) {
        if (i < 4096) {
#if defined(__x86_64__)
            _mm_pause();
#endif
        } else {
            std::this_thread::yield();
        }
    }
    base_ += chunks_->size();
    chunks_ = nullptr;
    segs_ = nullptr;
}

void HostPackPool::advance_frontier() {
    std::lock_guard<std::mutex> lk(frontier_mu_);
    const uint64_t K = chunks_->size(), f0 = frontier_;
    while (frontier_ < K &&
           done_[frontier_].load(std::memory_order_acquire) == unit_base_[frontier_ + 1] - unit_base_[frontier_])
        frontier_++;
    if (frontier_ != f0) packed_.set(base_ + frontier_);
}

void HostPackPool::pack_unit(uint64_t u, uint64_t k) {
    const XdpChunk &c = (*chunks_)[k];
    const uint64_t a = std::min(c.n, (u - unit_base_[k]) * kPackUnit), b = std::min(c.n, a + kPackUnit);
    if (a < b && !abort_.load(std::memory_order_relaxed)) pack_chunk_range(c, *segs_, a, b);
}

bool HostPackPool::claim_and_pack(bool coordinator) {
    using clk = std::chrono::steady_clock;
    const uint64_t U = unit_base_.back();
    uint64_t u, k;
    auto chunk_of = [&](uint64_t unit) {
        return (uint64_t)(std::upper_bound(unit_base_.begin(), unit_base_.end(), unit) - unit_base_.begin()) - 1;
    };
    auto t0 = clk::now();
    if (coordinator) {  // only units of released chunks: the coordinator is the one that releases
        u = next_unit_.load(std::memory_order_relaxed);
        for (;;) {
            if (u >= U) return false;
            k = chunk_of(u);
            if (base_ + k + 1 > released_.get()) return false;
            if (next_unit_.compare_exchange_weak(u, u + 1, std::memory_order_relaxed)) break;
        }
    } else {
        u = next_unit_.fetch_add(1, std::memory_order_relaxed);
        if (u >= U) return false;
        k = chunk_of(u);
        released_.wait_at_least(base_ + k + 1);
    }
    const auto t1 = clk::now();
    pack_unit(u, k);
    const auto t2 = clk::now();
    release_wait_ns_.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count(),
                               std::memory_order_relaxed);
    pack_ns_.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count(), std::memory_order_relaxed);
    if (done_[k].fetch_add(1, std::memory_order_acq_rel) + 1 == unit_base_[k + 1] - unit_base_[k]) advance_frontier();
    return true;
}

void HostPackPool::help_until_packed(uint64_t k) {
    const uint64_t target = base_ + k + 1;
    while (packed_.get() < target)
        if (!claim_and_pack(true)) {
            packed_.wait_at_least(target);  // the last units are on workers
            return;
        }
}

void HostPackPool::work() {
    uint64_t seen = 0;
    for (;;) {
        job_.wait_at_least(seen + 1);
        seen = job_.get();
        if (quit_.load()) return;
        active_.fetch_add(1, std::memory_order_seq_cst);
        if (!closed_.load(std::memory_order_seq_cst))
            while (claim_and_pack(false)) {
            }
        active_.fetch_sub(1, std::memory_order_seq_cst);
    }
}

void hostpack_burst(const uint8_t *const *frames, const uint32_t *linear_len, const uint32_t *pkt_len, uint64_t n,
                    uint32_t ifindex, const infw_hostpack_out &o) {
    constexpr uint64_t kPF = 16;  // frames ahead (infw_hostpack.h: the headers are DRAM misses)
    uint32_t rank = 0;
    uint32_t *tail = nullptr;
    for (uint64_t i = 0; i < n; i++) {
        if (i + kPF < n) {
            __builtin_prefetch(frames[i + kPF] + 10);
            __builtin_prefetch(frames[i + kPF] + 57);
        }
        if ((i & (INFW_V6_GROUP - 1)) == 0) {
            rank = 0;
            tail = reinterpret_cast<uint32_t *>(o.v6tail + (i / INFW_V6_GROUP) * (12ull * INFW_V6_GROUP));
        }
        const uint8_t *f = frames[i];
        const uint32_t lin = linear_len[i], plen = pkt_len ? pkt_len[i] : lin;
        uint32_t s0, s1, s2, s3, l4, meta;
        if (__builtin_expect(lin >= 58, 1)) {  // every field in place: infw_hostpack_xdp's branch-free form
            const uint32_t et = (uint32_t)f[12] << 8 | f[13];
            const bool v4 = et == 0x0800, v6 = et == 0x86DD;
            const uint32_t ip = (v4 || v6) ? ~0u : 0u;
            const uint32_t proto = f[v6 ? 20 : 23] & ip;
            s0 = infw_ld32(f + (v6 ? 22 : 26)) & ip;
            l4 = infw_ld32(f + (v6 ? 54 : 34)) & ip;
            s1 = infw_ld32(f + 26);
            s2 = infw_ld32(f + 30);
            s3 = infw_ld32(f + 34);
            meta = et | proto << 16 | (lin > 255u ? 255u : lin) << 24;
        } else {
            infw_tuple t;
            infw_pack_header(f, lin, plen, ifindex, &t);
            s0 = t.saddr[0], s1 = t.saddr[1], s2 = t.saddr[2], s3 = t.saddr[3];
            l4 = t.l4word;
            meta = t.meta;
        }
        const bool is6 = (meta & 0xFFFFu) == 0x86DDu;
        tail[3 * rank] = s1, tail[3 * rank + 1] = s2, tail[3 * rank + 2] = s3;
        rank += is6;
        o.saddr4[i] = s0;
        if (o.ifindex) o.ifindex[i] = ifindex;
        o.pkt_len[i] = plen;
        o.meta[i] = meta;
        o.l4word[i] = l4;
    }
}

void pack_chunk_range(const XdpChunk &c, const std::vector<XdpSeg> &segs, uint64_t a, uint64_t b) {
    constexpr uint64_t G = INFW_V6_GROUP;
    // the segment holding descriptor a (positions ascend within a chunk; a chunk of bursts may hold thousands)
    uint32_t first = c.seg0;
    if (c.seg1 - c.seg0 > 8)
        first = (uint32_t)(std::upper_bound(segs.begin() + c.seg0, segs.begin() + c.seg1, a,
                                            [](uint64_t v, const XdpSeg &g) { return v < g.pos; }) -
                           segs.begin()) - 1;
    for (uint32_t si = first; si < c.seg1 && segs[si].pos < b; si++) {
        const XdpSeg &s = segs[si];
        const uint64_t s0 = std::max(a, s.pos), s1 = std::min(b, s.pos + s.n);
        for (uint64_t p = s0; p < s1;) {
            const uint64_t g0 = p & ~(G - 1);
            uint32_t rank = 0;  // IPv6 packets an earlier segment put into this group: they hold its first tail slots
            uint64_t e = s1;
            if (p != g0) {  // (the same thread packed them: units start on group boundaries)
                for (uint64_t q = g0; q < p; q++) rank += (c.out.meta[q] & 0xFFFFu) == 0x86DDu;
                e = std::min(s1, g0 + G);  // up to the group's end, so the packer's group boundaries stay aligned
            }
            const infw_hostpack_out o{c.out.saddr4 + p, c.out.v6tail + g0 / G * (12 * G) + 12 * rank,
                                      c.mixed ? c.out.ifindex + p : nullptr, c.out.pkt_len + p, c.out.meta + p,
                                      c.out.l4word + p};
            if (s.frames && p == s0 && si + 1 < c.seg1 && segs[si + 1].frames) {
                // a burst's first frames are not prefetched by its own loop (which runs 16 frames ahead of itself):
                // issue them while this segment packs, so rx_burst-sized bursts keep as many misses in flight
                const XdpSeg &nx = segs[si + 1];
                for (uint64_t q = 0, m = std::min<uint64_t>(nx.n, 16); q < m; q++) {
                    __builtin_prefetch(nx.frames[q] + 10);
                    __builtin_prefetch(nx.frames[q] + 57);
                }
            }
            if (s.frames)
                hostpack_burst(s.frames + (p - s.pos), s.linear_len + (p - s.pos),
                               s.pkt_len ? s.pkt_len + (p - s.pos) : nullptr, e - p, s.ifindex, o);
            else
                infw_hostpack_xdp<INFW_PACK_PF, INFW_PACK_NT != 0>(s.umem, s.descs + (p - s.pos), e - p, s.ifindex,
                                                                   o);
            p = e;
        }
    }
}

int host_threads_auto() {
    int n = 0;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
    if (n <= 0) n = (int)std::thread::hardware_concurrency();
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {  // cgroup v2 "quota period" (or "max period")
        long long quota = 0, period = 0;
        if (fscanf(f, "%lld %lld", &quota, &period) == 2 && quota > 0 && period > 0)
            n = std::min<int>(n, (int)((quota + period - 1) / period));
        fclose(f);
    }
    return std::max(1, std::min(n, 16));
}

}  // namespace infw

extern "C" int infw_xdp_host_events(const uint8_t *umem, const struct infw_xdp_desc *descs, uint64_t n,
                                    uint32_t ifindex, const uint32_t *results, struct infw_event_sample *samples,
                                    uint64_t cap, uint64_t *count);

// Shared by the two event builders: sample k of a denied packet (kernel.c:392-399, infw_events_capture's layout).
static void infw_fill_sample(infw_event_sample &s, const uint8_t *f, uint32_t linear, uint32_t plen, uint32_t ifindex,
                             uint32_t r) {
    const uint32_t captured = plen < INFW_MAX_EVENT_DATA ? plen : INFW_MAX_EVENT_DATA;
    s.size = ((8u + captured + 4u + 7u) & ~7u) - 4u;
    memset(s.raw, 0, sizeof s.raw);
    event_hdr_st h{};
    h.ifId = (uint16_t)ifindex;
    h.ruleId = (uint16_t)(r >> 8);
    h.action = INFW_XDP_DROP;
    h.pktLength = (uint16_t)plen;
    memcpy(s.raw, &h, sizeof h);
    memcpy(s.raw + sizeof h, f, captured < linear ? captured : linear);  // past the linear part: zeros
}

extern "C" int infw_burst_host_events(const struct infw_frame_burst *b, const uint32_t *results,
                                      struct infw_event_sample *samples, uint64_t cap, uint64_t *count) {
    if (!b || !count || (b->n && (!b->frames || !b->linear_len || !results)) || (cap && !samples)) return -EINVAL;
    uint64_t k = 0;
    for (uint64_t i = 0; i < b->n; i++) {
        if ((results[i] & 0xFFu) != INFW_XDP_DROP) continue;
        if (k < cap)
            infw_fill_sample(samples[k], b->frames[i], b->linear_len[i], b->pkt_len ? b->pkt_len[i] : b->linear_len[i],
                             b->ifindex, results[i]);
        k++;
    }
    *count = k;
    return 0;
}

extern "C" int infw_pack_burst_host(const struct infw_frame_burst *b, const struct infw_batch_soa_c_out *out) {
    if (!b || !out) return -EINVAL;
    if (b->n == 0) return 0;
    bool ok = b->frames && b->linear_len && out->saddr4 && out->v6tail && out->pkt_len && out->meta && out->l4word;
    for (const void *q : {(const void *)out->saddr4, (const void *)out->v6tail, (const void *)out->ifindex,
                          (const void *)out->pkt_len, (const void *)out->meta, (const void *)out->l4word})
        ok = ok && ((uintptr_t)q & 3) == 0;
    if (!ok) return -EINVAL;
    infw::hostpack_burst(b->frames, b->linear_len, b->pkt_len, b->n, b->ifindex,
                         {out->saddr4, out->v6tail, out->ifindex, out->pkt_len, out->meta, out->l4word});
    return 0;
}

extern "C" int infw_xdp_host_events(const uint8_t *umem, const struct infw_xdp_desc *descs, uint64_t n,
                                    uint32_t ifindex, const uint32_t *results, struct infw_event_sample *samples,
                                    uint64_t cap, uint64_t *count) {
    if (!count || (n && (!umem || !descs || !results)) || (cap && !samples)) return -EINVAL;
    uint64_t k = 0;
    for (uint64_t i = 0; i < n; i++) {
        if ((results[i] & 0xFFu) != INFW_XDP_DROP) continue;
        if (k < cap)  // a single-buffer AF_XDP frame: linear = frame length = the descriptor's len
            infw_fill_sample(samples[k], infw_xdp_frame(umem, descs[i].addr), descs[i].len, descs[i].len, ifindex,
                             results[i]);
        k++;
    }
    *count = k;
    return 0;
}
