// Microbenchmark: random per-lane gathers on gfx950 — what one packet's table
// touches cost.  Each lane issues `iters` independent lookups (index from a
// counter hash), each reading W bytes (4, 8, 16, 32, 64) of one random
// W-aligned record of a T-byte table.  Reports lookups/s and record bytes/s.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/gather.hip -o gather && ./gather
#include <hip/hip_runtime.h>
#include <string.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

template <int W, bool kDep>
__global__ __launch_bounds__(512, 8) void gather(const uint32_t *__restrict__ tab, uint32_t mask, int iters,
                                                 uint32_t *__restrict__ out) {
    const uint32_t tid = blockIdx.x * 512 + threadIdx.x;
    uint32_t acc = 0, idx = mix(tid);
    for (int it = 0; it < iters; it++) {
        const uint32_t rec = (kDep ? mix(idx ^ acc) : mix(idx + it * 0x9E3779B9u)) & mask;
        if (W == 4) {
            acc += tab[rec];
        } else if (W == 8) {
            const uint2 v = reinterpret_cast<const uint2 *>(tab)[rec];
            acc += v.x ^ v.y;
        } else {
            const u32x4 *p = reinterpret_cast<const u32x4 *>(tab) + (uint64_t)rec * (W / 16);
#pragma unroll
            for (int k = 0; k < W / 16; k++) {
                const u32x4 v = p[k];
                acc += v[0] ^ v[1] ^ v[2] ^ v[3];
            }
        }
    }
    out[tid] = acc;
}

// Scalar-path gathers (the "mix" test): of every wave's 64 lookups, the first kScalar lanes' go through the scalar
// data cache one at a time — readlane makes the index wave-uniform, so the 8-B load is an s_load — and the other lanes'
// are ordinary per-lane vector loads.  Does the scalar path add random-gather capacity beside the vector L1's?
template <int kScalar>
__global__ __launch_bounds__(512, 8) void gather_mix(const uint2 *__restrict__ tab, uint32_t mask, int iters,
                                                     uint32_t *__restrict__ out) {
    const uint32_t tid = blockIdx.x * 512 + threadIdx.x, lane = threadIdx.x & 63;
    uint32_t acc = 0, idx = mix(tid);
    for (int it = 0; it < iters; it++) {
        const uint32_t rec = mix(idx + it * 0x9E3779B9u) & mask;
        uint2 vv = make_uint2(0, 0);
        if (lane >= (uint32_t)kScalar) vv = tab[rec];  // the vector lanes' loads first, consumed last
        // all the wave's scalar loads issued before any is consumed (up to 16 in flight per wave: SGPR budget)
        uint2 sv = make_uint2(0, 0);
#pragma unroll
        for (int j0 = 0; j0 < kScalar; j0 += 16) {
            uint2 v[16];
#pragma unroll
            for (int j = 0; j < 16 && j0 + j < kScalar; j++) v[j] = tab[__builtin_amdgcn_readlane(rec, j0 + j)];
#pragma unroll
            for (int j = 0; j < 16 && j0 + j < kScalar; j++)
                if (lane == (uint32_t)(j0 + j)) sv = v[j];
        }
        acc += lane >= (uint32_t)kScalar ? (vv.x ^ vv.y) : (sv.x ^ sv.y);
    }
    out[tid] = acc;
}

template <int kScalar>
void run_mix(const uint32_t *tab, uint64_t tbytes, uint32_t *out, int grid, int iters) {
    const uint32_t mask = (uint32_t)(tbytes / 8 - 1);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    gather_mix<kScalar><<<grid, 512>>>(reinterpret_cast<const uint2 *>(tab), mask, iters, out);
    hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; r++)
        gather_mix<kScalar><<<grid, 512>>>(reinterpret_cast<const uint2 *>(tab), mask, iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double lookups = (double)grid * 512 * iters * reps;
    printf("{\"test\": \"mix\", \"scalar_lanes\": %d, \"table_MiB\": %.1f, \"Glookups_s\": %.2f, "
           "\"scalar_Glookups_s\": %.2f, \"vector_Glookups_s\": %.2f}\n",
           kScalar, tbytes / 1048576.0, lookups / (ms * 1e-3) / 1e9, lookups * kScalar / 64 / (ms * 1e-3) / 1e9,
           lookups * (64 - kScalar) / 64 / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

// Spread footprint: `lines` distinct 128-B lines (16 B read from each), one at a random 128-B slot of each
// `stride`-byte window, so the L2 footprint stays the same while the address span (pages the lookups
// touch) grows with the stride.
__global__ __launch_bounds__(512, 8) void gather_spread(const uint32_t *__restrict__ tab, uint32_t lmask, uint32_t stride_w,
                                                        int iters, uint32_t *__restrict__ out) {
    const uint32_t tid = blockIdx.x * 512 + threadIdx.x;
    uint32_t acc = 0, idx = mix(tid);
    for (int it = 0; it < iters; it++) {
        const uint32_t l = mix(idx + it * 0x9E3779B9u) & lmask;
        // a random 128-B slot inside the line's stride window, so the lines spread over all L2 sets
        const uint32_t slot = (mix(l ^ 0x5bd1e995u) % (stride_w / 32u)) * 32u;
        const u32x4 v = *reinterpret_cast<const u32x4 *>(tab + (uint64_t)l * stride_w + slot);
        acc += v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    out[tid] = acc;
}

void run_spread(const uint32_t *tab, uint64_t fbytes, uint64_t span, uint32_t *out, int grid, int iters) {
    const uint64_t lines = fbytes / 128, stride = span / lines;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    gather_spread<<<grid, 512>>>(tab, (uint32_t)(lines - 1), (uint32_t)(stride / 4), iters, out);
    hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; r++) gather_spread<<<grid, 512>>>(tab, (uint32_t)(lines - 1), (uint32_t)(stride / 4), iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double lookups = (double)grid * 512 * iters * reps;
    printf("{\"test\": \"spread\", \"footprint_MiB\": %.1f, \"span_MiB\": %.1f, \"stride_B\": %llu, \"Glookups_s\": %.2f}\n",
           fbytes / 1048576.0, span / 1048576.0, (unsigned long long)stride, lookups / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

template <int W, bool kDep>
void run(const uint32_t *tab, uint64_t tbytes, uint32_t *out, int grid, int iters, const char *name) {
    const uint32_t mask = (uint32_t)(tbytes / W - 1);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    gather<W, kDep><<<grid, 512>>>(tab, mask, iters, out);
    hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; r++) gather<W, kDep><<<grid, 512>>>(tab, mask, iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double lookups = (double)grid * 512 * iters * reps;
    printf("{\"test\": \"%s\", \"W\": %d, \"dep\": %d, \"table_MiB\": %.1f, \"Glookups_s\": %.2f, \"rec_TBs\": %.2f, \"ns_per_lookup_per_CU\": %.3f}\n",
           name, W, (int)kDep, tbytes / 1048576.0, lookups / (ms * 1e-3) / 1e9, lookups * W / (ms * 1e-3) / 1e12,
           (ms * 1e6) / (lookups / 256.0));
    fflush(stdout);
}

int main(int argc, char **argv) {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int grid = cus * 4;
    // "bigspread": the same measurement over spans up to 12 GiB (configs[2]'s one-list-per-key tables span 10.6 GiB)
    const bool big = argc > 1 && strcmp(argv[1], "bigspread") == 0;
    const uint64_t max_t = big ? 12ull << 30 : 1ull << 30;
    uint32_t *tab, *out;
    if (hipMalloc(&tab, max_t) != hipSuccess) return 1;
    hipMemset(tab, 1, max_t);
    hipMalloc(&out, (size_t)grid * 512 * 4);
    if (big) {
        for (uint64_t f : {64ull << 20, 1ull << 30})
            for (uint64_t span : {1ull << 30, 2ull << 30, 4ull << 30, 8ull << 30, 12ull << 30})
                run_spread(tab, f, span, out, grid, 64);
        return 0;
    }
    if (argc > 1 && strcmp(argv[1], "mix") == 0) {  // scalar-path gathers beside vector ones
        for (uint64_t t : {1ull << 20, 16ull << 20, 1ull << 30}) {
            run_mix<0>(tab, t, out, grid, 16);
            run_mix<4>(tab, t, out, grid, 16);
            run_mix<8>(tab, t, out, grid, 16);
            run_mix<16>(tab, t, out, grid, 16);
            run_mix<32>(tab, t, out, grid, 16);
            run_mix<64>(tab, t, out, grid, 16);
        }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 's') {  // "spread": same L2 footprint over a growing address span
        for (uint64_t f : {2ull << 20, 16ull << 20, 64ull << 20})
            for (uint64_t span : {(uint64_t)f, (uint64_t)128 << 20, (uint64_t)1 << 30})
                if (span >= f) run_spread(tab, f, span, out, grid, 64);
        return 0;
    }
    if (argc > 1) {  // one configuration (PMC calibration): W=4 or 64, table MiB
        const int w = atoi(argv[1]);
        const uint64_t t = (uint64_t)atoi(argv[2]) << 20;
        if (w == 4) run<4, false>(tab, t, out, grid, 64, "indep");
        else if (w == 16) run<16, false>(tab, t, out, grid, 64, "indep");
        else run<64, false>(tab, t, out, grid, 64, "indep");
        return 0;
    }
    const uint64_t sizes[] = {1ull << 20, 16ull << 20, 128ull << 20, 1ull << 30};
    for (uint64_t t : sizes) {
        run<4, false>(tab, t, out, grid, 64, "indep");
        run<8, false>(tab, t, out, grid, 64, "indep");
        run<16, false>(tab, t, out, grid, 64, "indep");
        run<32, false>(tab, t, out, grid, 64, "indep");
        run<64, false>(tab, t, out, grid, 64, "indep");
        run<4, true>(tab, t, out, grid, 64, "dep");
        run<64, true>(tab, t, out, grid, 64, "dep");
    }
    return 0;
}
