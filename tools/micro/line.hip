// Microbenchmark: what one random 64-B table line costs a lane, by read form (the L2-hit path).
// Every lane reads one random 64-B line per iteration and consumes all of it, as the classify kernel reads a
// decision-table entry line; U lines per lane are in flight at once.  Forms:
//   1  one 16-B load (a quarter line: the single-request baseline)
//   4  four 16-B loads of the lane's own line, issued back to back (the classify kernel's dt_lookup form)
//   2  two 32-B loads (dwordx4 pairs: global_load_dwordx4 x 2 at 32-B stride... as b128 + b128 of one half each)
//   8  cooperative: the wave's 64 lines are loaded 16 at a time, lanes 4j..4j+3 loading the four 16-B quarters of
//      line j of the group (one coalesced request per line), then each owner lane reads its line back from LDS
// Table sizes span L2-resident to HBM.  Prints one JSON line per (form, table size): G lines/s.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/line.hip -o tools/micro/line && tools/micro/line [form MiB]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

constexpr int kBlock = 768;

template <int F, int U>
__global__ __launch_bounds__(kBlock, 6) void lines(const u32x4 *__restrict__ tab, uint32_t nlines, int iters,
                                                   uint32_t *__restrict__ out) {
    __shared__ u32x4 s_l[kBlock / 64][16 * 4];  // per wave: 16 lines of 4 quarters (cooperative form)
    const uint32_t tid = blockIdx.x * kBlock + threadIdx.x;
    const int lane = threadIdx.x & 63;
    u32x4 *wl = s_l[threadIdx.x >> 6];
    uint32_t acc = 0, idx = mix(tid * 2654435761u + 1);
    for (int it = 0; it < iters; it += U) {
        uint32_t line[U];
#pragma unroll
        for (int u = 0; u < U; u++) line[u] = mix(idx + (it + u) * 0x9E3779B9u) & (nlines - 1);
        if (F == 1) {
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; u++) v[u] = tab[4ull * line[u]];
#pragma unroll
            for (int u = 0; u < U; u++) acc += v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
        } else if (F == 4) {
            u32x4 a[U], b[U], c[U], d[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const u32x4 *p = tab + 4ull * line[u];
                a[u] = p[0]; b[u] = p[1]; c[u] = p[2]; d[u] = p[3];
            }
#pragma unroll
            for (int u = 0; u < U; u++) acc += (a[u] ^ b[u] ^ c[u] ^ d[u])[0] + (a[u] ^ b[u])[1] + (c[u] ^ d[u])[2] + d[u][3];
        } else if (F == 2) {
            u32x4 a[U], b[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const u32x4 *p = tab + 4ull * line[u];
                a[u] = p[0]; b[u] = p[1];
            }
#pragma unroll
            for (int u = 0; u < U; u++) acc += (a[u] ^ b[u])[0] + a[u][1] + b[u][2] + a[u][3];
        } else {  // cooperative
#pragma unroll
            for (int u = 0; u < U; u++) {
                u32x4 q[4];
#pragma unroll
                for (int r = 0; r < 4; r++) {  // round r: quarter (lane & 3) of the line of lane 16 r + (lane >> 2)
                    const uint32_t owner = 16u * r + (lane >> 2);
                    const uint32_t l = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(owner << 2), (int)line[u]);
                    q[r] = tab[4ull * l + (lane & 3)];
                }
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    wl[(lane >> 2) * 4 + (lane & 3)] = q[r];
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    if ((lane >> 4) == r) {
                        const u32x4 *m = wl + (lane & 15) * 4;
                        const u32x4 a = m[0], b = m[1], c = m[2], d = m[3];
                        acc += (a ^ b ^ c ^ d)[0] + (a ^ b)[1] + (c ^ d)[2] + d[3];
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                }
            }
        }
    }
    out[tid] = acc;
}

template <int F, int U>
double run(const u32x4 *tab, uint32_t nlines, uint32_t *out, int cus, int iters) {
    const int grid = cus * 2;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    lines<F, U><<<grid, kBlock>>>(tab, nlines, iters, out);
    hipEventRecord(a);
    const int reps = 3;
    for (int r = 0; r < reps; r++) lines<F, U><<<grid, kBlock>>>(tab, nlines, iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return (double)grid * kBlock * iters * reps / (ms * 1e-3) / 1e9;
}

template <int F>
void sweep(const u32x4 *tab, uint64_t mib, uint32_t *out, int cus) {
    const uint32_t nlines = (uint32_t)(mib * (1u << 20) / 64);
    const double g1 = run<F, 1>(tab, nlines, out, cus, 64), g2 = run<F, 2>(tab, nlines, out, cus, 64);
    printf("{\"form\": %d, \"table_MiB\": %llu, \"Glines_s_U1\": %.2f, \"Glines_s_U2\": %.2f}\n", F,
           (unsigned long long)mib, g1, g2);
    fflush(stdout);
}

int main(int argc, char **argv) {
    const uint64_t max_mib = 2048;
    u32x4 *tab;
    uint32_t *out;
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    if (hipMalloc(&tab, max_mib << 20) != hipSuccess || hipMalloc(&out, (size_t)cus * 2 * kBlock * 4) != hipSuccess)
        return 1;
    hipMemset(tab, 1, max_mib << 20);
    const int only_form = argc > 1 ? atoi(argv[1]) : 0;
    const uint64_t only_mib = argc > 2 ? strtoull(argv[2], nullptr, 10) : 0;
    for (uint64_t mib : {1ull, 16ull, 128ull, 2048ull}) {
        if (only_mib && mib != only_mib) continue;
        if (!only_form || only_form == 1) sweep<1>(tab, mib, out, cus);
        if (!only_form || only_form == 2) sweep<2>(tab, mib, out, cus);
        if (!only_form || only_form == 4) sweep<4>(tab, mib, out, cus);
        if (!only_form || only_form == 8) sweep<8>(tab, mib, out, cus);
    }
    hipFree(tab);
    hipFree(out);
    return 0;
}
