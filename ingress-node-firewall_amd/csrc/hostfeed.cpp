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

void pack_chunk_range(const XdpChunk &c, const std::vector<XdpSeg> &segs, uint64_t a, uint64_t b) {
    constexpr uint64_t G = INFW_V6_GROUP;
    for (uint32_t si = c.seg0; si < c.seg1; si++) {
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
            infw_hostpack_xdp<INFW_PACK_PF, INFW_PACK_NT != 0>(s.umem, s.descs + (p - s.pos), e - p, s.ifindex, o);
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
                                    uint64_t cap, uint64_t *count) {
    if (!count || (n && (!umem || !descs || !results)) || (cap && !samples)) return -EINVAL;
    uint64_t k = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t r = results[i];
        if ((r & 0xFFu) != INFW_XDP_DROP) continue;
        if (k < cap) {
            infw_event_sample &s = samples[k];
            const uint32_t len = descs[i].len;
            const uint32_t captured = len < INFW_MAX_EVENT_DATA ? len : INFW_MAX_EVENT_DATA;
            s.size = ((8u + captured + 4u + 7u) & ~7u) - 4u;
            memset(s.raw, 0, sizeof s.raw);
            event_hdr_st h{};
            h.ifId = (uint16_t)ifindex;
            h.ruleId = (uint16_t)(r >> 8);
            h.action = INFW_XDP_DROP;
            h.pktLength = (uint16_t)len;
            memcpy(s.raw, &h, sizeof h);
            memcpy(s.raw + sizeof h, infw_xdp_frame(umem, descs[i].addr), captured);
        }
        k++;
    }
    *count = k;
    return 0;
}
