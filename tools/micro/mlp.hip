// Microbenchmark: random 16-B gathers from a table far larger than the L2 (every lookup an L2 miss) at
// increasing memory-level parallelism — U independent loads issued per lane before any is waited for, at
// several occupancies — to tell whether the ~55 G misses/s the classify kernel reaches is the chip's
// miss-path ceiling or a latency x in-flight limit.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/mlp.hip -o tools/micro/mlp && tools/micro/mlp
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

template <int U>
__global__ __launch_bounds__(256) void gather_mlp(const u32x4 *__restrict__ tab, uint32_t mask, int iters,
                                                  uint32_t *__restrict__ out) {
    const uint32_t tid = blockIdx.x * 256 + threadIdx.x;
    uint32_t acc = 0, idx = mix(tid);
    for (int it = 0; it < iters; it += U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = tab[mix(idx + (it + u) * 0x9E3779B9u) & mask];
#pragma unroll
        for (int u = 0; u < U; u++) acc += v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
    }
    out[tid] = acc;
}

template <int U>
void run(const u32x4 *tab, uint32_t mask, uint32_t *out, int cus, int blocks_per_cu, int iters) {
    const int grid = cus * blocks_per_cu;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    gather_mlp<U><<<grid, 256>>>(tab, mask, iters, out);
    hipEventRecord(a);
    const int reps = 3;
    for (int r = 0; r < reps; r++) gather_mlp<U><<<grid, 256>>>(tab, mask, iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double lookups = (double)grid * 256 * iters * reps;
    printf("{\"U\": %d, \"waves_per_cu\": %d, \"Glookups_s\": %.2f}\n", U, blocks_per_cu * 4,
           lookups / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

int main() {
    const uint64_t bytes = 1ull << 32;  // 4 GiB: every lookup misses the 4-MiB XCD L2s and the 256-MiB MALL
    u32x4 *tab;
    uint32_t *out;
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    if (hipMalloc(&tab, bytes) != hipSuccess || hipMalloc(&out, (size_t)cus * 32 * 256 * 4) != hipSuccess) return 1;
    hipMemset(tab, 1, bytes);
    const uint32_t mask = (uint32_t)(bytes / 16 - 1);
    for (int bpc : {2, 4, 6, 8}) {
        run<1>(tab, mask, out, cus, bpc, 64);
        run<2>(tab, mask, out, cus, bpc, 64);
        run<4>(tab, mask, out, cus, bpc, 64);
        run<8>(tab, mask, out, cus, bpc, 64);
    }
    hipFree(tab);
    hipFree(out);
    return 0;
}
