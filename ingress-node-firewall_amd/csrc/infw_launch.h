// infw_launch.h — the launch interface between the C ABI (abi.cpp) and the kernels (classify.hip).
//
// One call describes one classify launch: the epoch's table view, the batch in one of its three forms, the outputs,
// the launch shape (infw_set_launch) and the sidebands.  The kernel instantiation it runs is chosen by one
// deterministic selector from the epoch's kind (lean, per-list part counts, /16 words, half-first reads, two-phase)
// and the shape; every instantiation the selector can return is listed in one registry (classify.hip), which the
// tests enumerate (infw_kernel_variant_name) and run one by one against the oracle.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/infw.h"
#include "infw_tables.h"

struct infw_launch_args {
    const infw_dev_tables *T;      // the epoch's view, split / stat_flush_tiles already decided by the caller
    int input;                     // INFW_INPUT_SOA / _COMPACT / _FRAMES / _XDP (include/infw.h)
    const infw_batch_soa *soa;
    const infw_batch_soa_c *compact;
    const infw_frame_batch *frames;
    const uint8_t *umem;             // INFW_INPUT_XDP (infw_classify_xdp): AF_XDP descriptors, frames at
    const infw_xdp_desc *xdp;        // umem + addr, one ifindex for the ring
    uint32_t xdp_ifindex;
    uint64_t n;
    uint32_t *results;
    uint8_t *verdicts;
    uint64_t *stats;
    uint32_t cus;
    int block, group, blocks_per_cu;  // a shape infw_launch_shape_ok accepts
    hipStream_t stream;
    hipMemPool_t pool;             // the context's pool for the two-phase scratch (null: the fused kernel runs)
    uint64_t *split_counts;        // non-null: [0] += 1 per two-phase launch, [1] += 1 per two-phase launch that ran
                                   // the fused kernel for want of scratch (host-side atomics; infw_launch_counts)
    infw_event_rec *ev;
    uint64_t ev_cap;
    uint64_t *ev_count;            // non-null: the deny-event sideband
    uint64_t *dbg_fp;              // non-null: the debug-lookup sideband
    uint32_t *dbg_keys;
    uint32_t *dbg_count;
    uint32_t dbg_slots;
};

extern "C" {
// Launch (asynchronous).  0, or -EIO on a launch error.
int infw_launch_classify(const infw_launch_args *a);
// The instantiation(s) the launch would run, by registry name ("<phase 1>+decide.512" for the two-phase form),
// without launching anything (host code: no device needed).  0, -ERANGE when cap is too small.
int infw_launch_variant(const infw_launch_args *a, char *name, size_t cap);
int infw_launch_variant_count(void);
const char *infw_launch_variant_name(int i);
// The launch shapes infw_set_launch accepts.
int infw_launch_shape_ok(int block, int group, int blocks_per_cu);
}
