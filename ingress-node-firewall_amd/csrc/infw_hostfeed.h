// infw_hostfeed.h — the host packer threads of infw_classify_xdp_host (include/infw.h).
//
// A pool of worker threads packs a call's chunks (each a run of one AF_XDP ring's descriptors) into a ring of pinned
// host slots, in chunk order, while the calling thread — the coordinator — moves packed chunks through the device
// (H2D, classify, D2H on three HIP streams).  Work is handed out dynamically: every chunk is cut into units of
// kPackUnit descriptors (whole INFW_V6_GROUP groups), numbered across the call, and a worker claims the next unit
// with one atomic increment — a worker that is descheduled or slower (an SMT sibling, a remote NUMA node) delays one
// unit, not a fixed share of every chunk.  A worker may pack a unit of chunk k once the coordinator has released k
// (its slot's previous chunk has left for the device); chunk k counts as packed when all of its units are done and
// so are all earlier chunks (the packed frontier only grows).  Waits spin briefly and then sleep on a condition
// variable.
#pragma once
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <memory>
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

constexpr uint64_t kPackUnit = 4096;  // descriptors per claimed unit (~30 us of one core's packing)

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
    // Worker time since the last begin(), summed over the workers (ns): packing, and waiting for a chunk's release
    // (its host slot still on its way to the device) — read after end()
    uint64_t pack_ns() const { return pack_ns_.load(); }
    uint64_t release_wait_ns() const { return release_wait_ns_.load(); }

   private:
    void work();
    void advance_frontier();
    std::vector<std::thread> workers_;
    Signal job_;       // generation of the current job (workers wait for the next one)
    Signal released_;  // base_ + chunks released
    Signal packed_;    // base_ + chunks fully packed (the frontier)
    Signal idle_;      // workers that finished the current job (cumulative)
    std::vector<uint64_t> unit_base_;                // first unit of chunk k; back() = units of the job
    std::unique_ptr<std::atomic<uint32_t>[]> done_;  // units of chunk k done
    std::atomic<uint64_t> next_unit_{0};
    std::mutex frontier_mu_;
    uint64_t frontier_ = 0;  // chunks < frontier_ are packed (under frontier_mu_)
    const std::vector<XdpChunk> *chunks_ = nullptr;
    std::vector<infw_hostpack_out> slots_;
    uint64_t base_ = 0;  // chunk sequence number of the job's chunk 0 (the signals only grow)
    uint64_t gen_ = 0;
    std::atomic<bool> abort_{false}, quit_{false};
    std::atomic<uint64_t> idle_total_{0};
    std::atomic<uint64_t> pack_ns_{0}, release_wait_ns_{0};
    int n_threads_;
};

// Worker threads for a pool: option host_threads, or (0) the CPUs this process may run on — its affinity mask, capped
// by a cgroup v2 CPU quota (cpu.max) — at most 16.
int host_threads_auto();

}  // namespace infw
