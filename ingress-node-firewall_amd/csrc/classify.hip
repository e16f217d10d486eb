// classify.hip — gfx950 kernel for the batched XDP classification
// (bpf/ingress_node_firewall_kernel.c:412-457 over one SoA batch).
//
// One workgroup = 4 waves x 64 lanes; a persistent grid strides over the
// batch 256 packets at a time.  Per tile:
//   1. each lane loads one 32-B tuple (five coalesced streams), parses it
//      (infw_parse) and walks the LPM (ifindex hash -> IPv6 long table ->
//      DIR-24-8), then gathers its rule-list descriptor for its class;
//   2. the wave resolves first-match cooperatively, one lane per rule: for
//      each lane j that needs a scan (s_ff1 over a ballot), the 64 lanes load
//      64 consecutive rule records of j's class list, test lo <= v_j <= hi,
//      and __ballot/ffs picks the first match — the reference's in-order scan
//      (kernel.c:222-258) in one wave step per 64 rules;
//   3. result words and verdicts are stored coalesced; allow/deny counters
//      accumulate in LDS (u32 packets, u64 bytes per rule id) and are flushed
//      with one u64 atomic per touched counter when the workgroup retires.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/infw.h"
#include "infw_tables.h"

namespace {

constexpr int kBlock = 256;
constexpr int kStatKeys = INFW_MAX_TARGETS;

__device__ __forceinline__ uint32_t readlane(uint32_t v, int lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}

template <bool kResults, bool kVerdicts>
__global__ __launch_bounds__(kBlock) void classify_kernel(const infw_dev_tables T,
                                                          const infw_batch_soa in, uint64_t n,
                                                          uint32_t *__restrict__ results,
                                                          uint8_t *__restrict__ verdicts,
                                                          unsigned long long *__restrict__ stats) {
    __shared__ uint32_t s_pk[2 * kStatKeys];            // [rule][allow=0, deny=1]
    __shared__ unsigned long long s_by[2 * kStatKeys];
    for (int i = threadIdx.x; i < 2 * kStatKeys; i += kBlock) {
        s_pk[i] = 0;
        s_by[i] = 0;
    }
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const uint4 *sa4 = reinterpret_cast<const uint4 *>(in.saddr);
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;

    for (uint64_t base = (uint64_t)blockIdx.x * kBlock; base < n; base += stride) {
        const uint64_t i = base + threadIdx.x;
        const bool valid = i < n;
        uint32_t meta = 0, l4w = 0, ifx = 0, plen = 0;
        uint4 sa = make_uint4(0, 0, 0, 0);
        if (valid) {
            meta = in.meta[i];
            l4w = in.l4word[i];
            ifx = in.ifindex[i];
            plen = in.pkt_len[i];
            sa = sa4[i];
        }
        int cls = 0;
        uint32_t val = 0;
        int pk = valid ? infw_parse(meta, l4w, &cls, &val) : INFW_PK_PASS_NONIP;
        uint64_t d = 0;
        if (pk >= INFW_PK_V4) {
            const uint32_t sw[4] = {sa.x, sa.y, sa.z, sa.w};
            uint32_t l1 = infw_lpm(T, pk, ifx, sw);
            if (l1) d = T.desc[(uint64_t)(l1 - 1) * INFW_DESC_STRIDE + cls];
        }
        const uint32_t off = (uint32_t)d, cnt = (uint32_t)(d >> 32);

        // ---- first match, one lane per rule
        uint32_t result = 0;
        uint64_t pending = __ballot(cnt != 0);
        while (pending) {
            const int j = __builtin_ctzll(pending);
            pending &= pending - 1;
            const uint32_t oj = readlane(off, j), cj = readlane(cnt, j), vj = readlane(val, j);
            uint32_t r = 0;
            for (uint32_t k0 = 0; k0 < cj; k0 += 64) {
                const uint32_t k = k0 + lane;
                uint64_t rec = 0;
                bool m = false;
                if (k < cj) {
                    rec = T.rules[(uint64_t)oj + k];
                    const uint32_t lo = (uint32_t)rec & 0xFFFFu, hi = (uint32_t)(rec >> 16) & 0xFFFFu;
                    m = lo <= vj && vj <= hi;
                }
                const uint64_t mb = __ballot(m);
                if (mb) {
                    r = readlane((uint32_t)(rec >> 32), __builtin_ctzll(mb));
                    break;
                }
            }
            if (lane == j) result = r;
        }

        // ---- verdict (kernel.c:444-456) and statistics (kernel.c:376-387)
        const uint32_t action = result & 0xFFu;
        const uint32_t key = (result >> 8) & 0xFFFFu;
        if (valid) {
            if (kResults) results[i] = result;
            if (kVerdicts)
                verdicts[i] = (pk == INFW_PK_DROP_SHORT || action == INFW_XDP_DROP) ? INFW_XDP_DROP
                                                                                    : INFW_XDP_PASS;
            if ((action == INFW_XDP_DROP || action == INFW_XDP_PASS) && key < kStatKeys) {
                const int s = (int)key * 2 + (action == INFW_XDP_DROP);
                atomicAdd(&s_pk[s], 1u);
                atomicAdd(&s_by[s], (unsigned long long)plen);
            }
        }
    }

    __syncthreads();
    for (int s = threadIdx.x; s < 2 * kStatKeys; s += kBlock) {
        const uint32_t p = s_pk[s];
        if (p) {
            unsigned long long *dst = stats + (s >> 1) * 4 + (s & 1) * 2;
            atomicAdd(dst, (unsigned long long)p);
            atomicAdd(dst + 1, s_by[s]);
        }
    }
}

}  // namespace

// Host-side launcher (called from abi.cpp).  grid: persistent workgroup count.
extern "C" int infw_launch_classify(const infw_dev_tables *T, const infw_batch_soa *in, uint64_t n,
                                    uint32_t *results, uint8_t *verdicts, uint64_t *stats,
                                    uint32_t grid, hipStream_t stream) {
    if (n == 0) return 0;
    uint64_t tiles = (n + kBlock - 1) / kBlock;
    uint32_t g = (uint32_t)(tiles < grid ? tiles : grid);
    auto *st = reinterpret_cast<unsigned long long *>(stats);
    if (results && verdicts)
        hipLaunchKernelGGL((classify_kernel<true, true>), dim3(g), dim3(kBlock), 0, stream, *T, *in, n, results, verdicts, st);
    else if (results)
        hipLaunchKernelGGL((classify_kernel<true, false>), dim3(g), dim3(kBlock), 0, stream, *T, *in, n, results, verdicts, st);
    else if (verdicts)
        hipLaunchKernelGGL((classify_kernel<false, true>), dim3(g), dim3(kBlock), 0, stream, *T, *in, n, results, verdicts, st);
    else
        hipLaunchKernelGGL((classify_kernel<false, false>), dim3(g), dim3(kBlock), 0, stream, *T, *in, n, results, verdicts, st);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
