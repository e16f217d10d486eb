// infw_hostfeed.h — the host packer threads of infw_classify_xdp_host (include/infw.h).
//
// A call's AF_XDP rings (or bursts) are cut into chunks of at most `chunk` descriptors that run on from one ring into
// the next (a chunk holds the tail of one, whole ones, the head of another, back to back), and a pool of worker threads packs the chunks into a ring of
// pinned host slots, in chunk order, while the calling thread — the coordinator — moves packed chunks through the
// device (H2D, classify, D2H) and packs too whenever it would otherwise wait.  Work is handed out dynamically: every
// chunk is cut into units of kPackUnit descriptors (whole INFW_V6_GROUP groups), numbered across the call, and a
// thread claims the next unit with one atomic operation — a worker that is descheduled or slower (an SMT sibling, a
// remote NUMA node) delays one unit, not a fixed share of every chunk.  A unit of chunk k may be packed once the
// coordinator has released k (its slot's previous chunk has left for the device); chunk k counts as packed when all of
// its units are done and so are all earlier chunks (the packed frontier only grows).
//
// Latency of small calls (a daemon polling rings of a few thousand descriptors): workers that find the pool idle spin
// briefly before they sleep, a call of one or two units wakes no worker at all (the coordinator packs it), and a call
// ends as soon as no worker is inside it — a worker that wakes late for a job already closed leaves without touching
// it (an active count and a closed flag, checked in that order on both sides).
#pragma once
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/infw.h"
#include "../../include/infw_host.h"
#include "infw_hostpack.h"

namespace infw {

// A monotonic counter that threads wait on (spin, then sleep).
class Signal {
   public:
    uint64_t get() const { return v_.load(std::memory_order_acquire); }
    void set(uint64_t v);                 // v never decreases
    void wait_at_least(uint64_t target);  // returns once get() >= target
   private:
    std::atomic<uint64_t> v_{0};
    std::mutex mu_;
    std::condition_variable cv_;
};

// A call's sources as the caller handed them over — AF_XDP rings (umem + descriptors) or DPDK-style bursts (frame
// pointers + linear and frame lengths): exactly one of `rings` / `bursts` is set — laid end to end at call positions:
// source i holds positions [start[i], start[i + 1]).  No per-source copy is made: a call of half a million
// rx_burst-sized bursts costs one pass that writes 8 B per burst.
struct HostFedSrc {
    const infw_xdp_ring *rings = nullptr;
    const infw_frame_burst *bursts = nullptr;
    const uint64_t *start = nullptr;  // count + 1 entries
    uint32_t count = 0;
    uint32_t ifindex(uint32_t i) const { return rings ? rings[i].ifindex : bursts[i].ifindex; }
    uint32_t *results(uint32_t i) const { return rings ? rings[i].results : bursts[i].results; }
    uint8_t *verdicts(uint32_t i) const { return rings ? rings[i].verdicts : bursts[i].verdicts; }
    // the source holding call position pos < start[count] (empty sources share their start with the next one)
    uint32_t at(uint64_t pos) const;
};

// A burst's frames [0, n) -> the family-compact streams (host code; the burst form of infw_hostpack_xdp).
void hostpack_burst(const uint8_t *const *frames, const uint32_t *linear_len, const uint32_t *pkt_len, uint64_t n,
                    uint32_t ifindex, const infw_hostpack_out &o);

// One D2H copy of a chunk's result words or verdicts: chunk positions [pos, pos + n) to dst.
struct XdpCopy {
    uint64_t pos, n;
    uint8_t *dst;
};
constexpr uint32_t kXdpMaxCopies = 16;  // copies per chunk before its words are staged and scattered on the host

// A chunk: call positions [begin, begin + n), sources [src0, src1).  `mixed`: its sources carry more than one
// ifindex, so the packers write the ifindex stream (else the device fills it).  Its D2H copies: result words
// rcopies[r0, r1), verdicts vcopies[v0, v1) — sources whose arrays continue one another merge into one copy — or,
// `staged`, more than kXdpMaxCopies of them: the chunk comes back in one copy of each kind, scattered on the host.
// `out`: the chunk's streams in its host slot (positions 0..n-1).
struct XdpChunk {
    uint64_t begin, n;
    uint32_t src0, src1;
    bool mixed, staged, any_res, any_ver;
    uint32_t r0, r1, v0, v1;
    infw_hostpack_out out;
};

// A call's cut: source positions, chunks and their D2H copies (src.start points into `start`: not copyable).
struct CutPlan {
    std::vector<uint64_t> start;  // count + 1 entries
    std::vector<XdpChunk> chunks;  // their `out` left for the caller
    std::vector<XdpCopy> rcopies, vcopies;
    HostFedSrc src;
    uint64_t ce = 0;  // positions per chunk (the last may hold fewer)
    CutPlan() = default;
    CutPlan(const CutPlan &) = delete;
    CutPlan &operator=(const CutPlan &) = delete;
};

// Positions per chunk for a call of `total`: `chunk` (a multiple of INFW_V6_GROUP), or with auto_chunk, for a call of
// fewer than four chunks, a quarter of the call (at least 32K), so that its packing overlaps its copies.
uint64_t chunk_positions(uint64_t total, uint64_t chunk, bool auto_chunk);

// The sources cut into chunks of chunk_positions(total) positions running on from one source into the next, with
// their D2H copies: two passes over the caller's array (validate and count, then cut), each split over up to
// `threads` threads for a call of many sources, whose pieces of a shared chunk are merged in order — the plan is the
// same at any thread count.  -EINVAL for a source with flags set or a null array it needs (nothing is packed then).
int cut_chunks(const infw_xdp_ring *rings, const infw_frame_burst *bursts, uint32_t count, uint64_t chunk,
               bool auto_chunk, int threads, CutPlan &plan);

constexpr uint64_t kPackUnit = 4096;  // descriptors per claimed unit (~30 us of one core's packing)

class HostPackPool {
   public:
    explicit HostPackPool(int threads);
    ~HostPackPool();
    int threads() const { return n_threads_; }
    // Start packing `chunks` of `src` (at most `released` chunks before release() allows more).  Both must outlive
    // end().
    void begin(const std::vector<XdpChunk> *chunks, const HostFedSrc *src, uint64_t released);
    // The coordinator's wait for chunk k: it packs released units itself until k is packed.
    void help_until_packed(uint64_t k);
    void release(uint64_t upto) { released_.set(base_ + upto); }  // chunks < upto may be packed
    // Stop (abort: units not yet claimed are skipped) and wait until no worker is inside the job.
    void end(bool abort);
    // Thread time since the last begin(), summed over the workers and the coordinator (ns): packing, and waiting for
    // a chunk's release (its host slot still on its way to the device) — read after end()
    uint64_t pack_ns() const { return pack_ns_.load(); }
    uint64_t release_wait_ns() const { return release_wait_ns_.load(); }

   private:
    void work();
    bool claim_and_pack(bool coordinator);  // one unit; false when none is left (or none released, coordinator)
    void pack_unit(uint64_t u, uint64_t k);
    void advance_frontier();
    std::vector<std::thread> workers_;
    Signal job_;       // generation of the current job (workers wait for the next one)
    Signal released_;  // base_ + chunks released
    Signal packed_;    // base_ + chunks fully packed (the frontier)
    std::vector<uint64_t> unit_base_;                // first unit of chunk k; back() = units of the job
    std::unique_ptr<std::atomic<uint32_t>[]> done_;  // units of chunk k done
    std::atomic<uint64_t> next_unit_{0};
    std::atomic<int> active_{0};      // workers inside the current job
    std::atomic<bool> closed_{true};  // no job open: workers must not touch the job's data
    std::mutex frontier_mu_;
    uint64_t frontier_ = 0;  // chunks < frontier_ are packed (under frontier_mu_)
    const std::vector<XdpChunk> *chunks_ = nullptr;
    const HostFedSrc *src_ = nullptr;
    uint64_t base_ = 0;  // chunk sequence number of the job's chunk 0 (the signals only grow)
    uint64_t gen_ = 0;
    std::atomic<bool> abort_{false}, quit_{false};
    std::atomic<uint64_t> pack_ns_{0}, release_wait_ns_{0};
    int n_threads_;
};

// Pack chunk positions [a, b) of `c` (a on an INFW_V6_GROUP boundary) from its sources into c.out.
void pack_chunk_range(const XdpChunk &c, const HostFedSrc &src, uint64_t a, uint64_t b);

// Worker threads for a pool: option host_threads, or (0) the CPUs this process may run on — its affinity mask, capped
// by a cgroup v2 CPU quota (cpu.max) — at most 16.
int host_threads_auto();

}  // namespace infw
