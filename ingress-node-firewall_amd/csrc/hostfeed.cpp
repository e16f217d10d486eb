// hostfeed.cpp — the host packer threads of infw_classify_xdp_host (infw_hostfeed.h).
#include "infw_hostfeed.h"

#include <sched.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>

#if defined(__x86_64__)
#include <immintrin.h>
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

void HostPackPool::begin(const std::vector<XdpChunk> *chunks, std::vector<infw_hostpack_out> slots, uint64_t released) {
    chunks_ = chunks;
    slots_ = std::move(slots);
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
    job_.set(++gen_);  // publishes the job (the signal's mutex orders the fields above before the workers' reads)
}

void HostPackPool::end(bool abort) {
    if (abort) {
        abort_.store(true);
        released_.set(base_ + chunks_->size());
    }
    idle_.wait_at_least(gen_ * n_threads_);
    base_ += chunks_->size();
    chunks_ = nullptr;
}

void HostPackPool::advance_frontier() {
    std::lock_guard<std::mutex> lk(frontier_mu_);
    const uint64_t K = chunks_->size(), f0 = frontier_;
    while (frontier_ < K &&
           done_[frontier_].load(std::memory_order_acquire) == unit_base_[frontier_ + 1] - unit_base_[frontier_])
        frontier_++;
    if (frontier_ != f0) packed_.set(base_ + frontier_);
}

void HostPackPool::work() {
    uint64_t seen = 0;
    for (;;) {
        job_.wait_at_least(seen + 1);
        seen = job_.get();
        if (quit_.load()) return;
        const std::vector<XdpChunk> &ch = *chunks_;
        const uint64_t NS = slots_.size(), base = base_, U = unit_base_.back();
        using clk = std::chrono::steady_clock;
        uint64_t wait_ns = 0, busy_ns = 0, k = 0;
        for (;;) {
            const uint64_t u = next_unit_.fetch_add(1, std::memory_order_relaxed);
            if (u >= U) break;
            while (unit_base_[k + 1] <= u) k++;  // a worker's units only grow, so its chunk index does too
            const auto t0 = clk::now();
            released_.wait_at_least(base + k + 1);
            const auto t1 = clk::now();
            wait_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
            const XdpChunk &c = ch[k];
            const uint64_t a = std::min(c.n, (u - unit_base_[k]) * kPackUnit), b = std::min(c.n, a + kPackUnit);
            if (a < b && !abort_.load(std::memory_order_relaxed)) {
                const infw_hostpack_out &s = slots_[k % NS];
                const infw_hostpack_out o{s.saddr4 + a, s.v6tail + a / INFW_V6_GROUP * (12ull * INFW_V6_GROUP),
                                          nullptr, s.pkt_len + a, s.meta + a, s.l4word + a};
                infw_hostpack_xdp<16, false>(c.umem, c.descs + a, b - a, c.ifindex, o);
            }
            busy_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t1).count();
            if (done_[k].fetch_add(1, std::memory_order_acq_rel) + 1 == unit_base_[k + 1] - unit_base_[k])
                advance_frontier();
        }
        pack_ns_.fetch_add(busy_ns);
        release_wait_ns_.fetch_add(wait_ns);
        idle_.set(idle_total_.fetch_add(1) + 1);
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
