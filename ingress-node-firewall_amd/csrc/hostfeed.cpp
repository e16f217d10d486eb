// hostfeed.cpp — the host packer threads of infw_classify_xdp_host (infw_hostfeed.h).
#include "infw_hostfeed.h"

#include <sched.h>
#include <stdio.h>

#include <algorithm>

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

HostPackPool::HostPackPool(int threads) : shares_done_(8), n_threads_(threads) {
    workers_.reserve(threads);
    for (int t = 0; t < threads; t++) workers_.emplace_back([this, t] { work(t); });
}

HostPackPool::~HostPackPool() {
    quit_.store(true);
    job_.set(gen_ + 1);
    for (auto &w : workers_) w.join();
}

void HostPackPool::begin(const std::vector<XdpChunk> *chunks, std::vector<infw_hostpack_out> slots, uint64_t released) {
    chunks_ = chunks;
    slots_ = std::move(slots);
    if (slots_.size() > shares_done_.size()) slots_.resize(shares_done_.size());
    for (auto &c : shares_done_) c.store(0, std::memory_order_relaxed);
    abort_.store(false);
    released_.set(base_ + released);
    job_.set(++gen_);  // publishes chunks_, slots_, base_ (the signal's mutex orders them before the workers' reads)
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

void HostPackPool::work(int t) {
    uint64_t seen = 0;
    for (;;) {
        job_.wait_at_least(seen + 1);
        seen = job_.get();
        if (quit_.load()) return;
        const std::vector<XdpChunk> &ch = *chunks_;
        const uint64_t T = n_threads_, NS = slots_.size(), base = base_;
        for (uint64_t k = 0; k < ch.size(); k++) {
            released_.wait_at_least(base + k + 1);
            const XdpChunk &c = ch[k];
            const uint64_t share = ((c.n + T - 1) / T + (INFW_V6_GROUP - 1)) & ~(uint64_t)(INFW_V6_GROUP - 1);
            const uint64_t a = std::min<uint64_t>(c.n, t * share), b = std::min<uint64_t>(c.n, a + share);
            if (a < b && !abort_.load(std::memory_order_relaxed)) {
                const infw_hostpack_out &s = slots_[k % NS];
                const infw_hostpack_out o{s.saddr4 + a, s.v6tail + a / INFW_V6_GROUP * (12ull * INFW_V6_GROUP),
                                          nullptr, s.pkt_len + a, s.meta + a, s.l4word + a};
                infw_hostpack_xdp<16, false>(c.umem, c.descs + a, b - a, c.ifindex, o);
            }
            // slot k % NS sees chunks k % NS, k % NS + NS, ... in order: its counter is cumulative over the job
            const int done = shares_done_[k % NS].fetch_add(1, std::memory_order_acq_rel) + 1;
            if ((uint64_t)done == T * (k / NS + 1)) packed_.set(base + k + 1);
        }
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
