// infw_hostfeed.h — the host packer threads of infw_classify_xdp_host (include/infw.h).
//
// A pool of worker threads packs a call's chunks (each a run of one AF_XDP ring's descriptors) into a ring of pinned
// host slots, in chunk order, while the calling thread — the coordinator — moves packed chunks through the device
// (H2D, classify, D2H on three HIP streams).  Every worker owns the same share of every chunk and runs through the
// chunks without a barrier: chunk k counts as packed when its last share is done (shares finish in chunk order, so
// packed() only grows), and a worker may start chunk k once the coordinator has released it (its slot's previous
// chunk has left for the device).  Waits spin briefly and then sleep on a condition variable.
#pragma once
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/infw.h"
#include "infw_hostpack.h"

namespace infw {

// A monotonic counter that threads wait on (spin, then sleep).
class Signal {
   public:
    uint64_t get() const { return v_.load(std::memory_order_acquire); }
    void set(uint64_t v);                // v never decreases
    void wait_at_least(uint64_t target);  // returns once get() >= target
   private:
    std::atomic<uint64_t> v_{0};
    std::mutex mu_;
    std::condition_variable cv_;
};

struct XdpChunk {
    const uint8_t *umem;
    const infw_xdp_desc *descs;
    uint64_t n;
    uint32_t ifindex;
};

class HostPackPool {
   public:
    explicit HostPackPool(int threads);
    ~HostPackPool();
    int threads() const { return n_threads_; }
    // Start packing `chunks` (at most `released` of them before release() allows more); chunk k goes to
    // slot(k).  The vector and the slots must outlive end().
    void begin(const std::vector<XdpChunk> *chunks, std::vector<infw_hostpack_out> slots, uint64_t released);
    void wait_packed(uint64_t k) { packed_.wait_at_least(base_ + k + 1); }  // chunk k is in its slot
    void release(uint64_t upto) { released_.set(base_ + upto); }           // chunks < upto may be packed
    // Stop (abort: chunks not yet started are skipped) and wait until no worker touches the job.
    void end(bool abort);

   private:
    void work(int t);
    std::vector<std::thread> workers_;
    Signal job_;       // generation of the current job (workers wait for the next one)
    Signal released_;  // base_ + chunks released
    Signal packed_;    // base_ + chunks fully packed
    Signal idle_;      // workers that finished the current job (cumulative)
    std::vector<std::atomic<int>> shares_done_;  // per slot (at most 8): shares of its chunks done in this job
    const std::vector<XdpChunk> *chunks_ = nullptr;
    std::vector<infw_hostpack_out> slots_;
    uint64_t base_ = 0;  // chunk sequence number of the job's chunk 0 (the signals only grow)
    uint64_t gen_ = 0;
    std::atomic<bool> abort_{false}, quit_{false};
    std::atomic<uint64_t> idle_total_{0};
    int n_threads_;
};

// Worker threads for a pool: option host_threads, or (0) the CPUs this process may run on — its affinity mask, capped
// by a cgroup v2 CPU quota (cpu.max) — at most 16.
int host_threads_auto();

}  // namespace infw
