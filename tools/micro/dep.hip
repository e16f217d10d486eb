// dep.hip — dependent pairs of random reads: a 16-B word from a 64-MiB table (the LPM step's stand-in), whose
// value picks a 64-B line (four 16-B loads, the decision line's form) among `lines` lines spread one per
// `stride`-byte window over a span of lines x stride bytes.  Same footprint, growing span: does the second,
// dependent read slow down with the span, as configs[2]'s one-list-per-key tables in random order suggest
// ?  Usage: tools/micro/dep   (JSON lines: footprint, span, G pairs/s)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    return x ^ (x >> 16);
}

__global__ __launch_bounds__(768, 6) void dep_pairs(const uint32_t *__restrict__ a, uint32_t amask,
                                                     const uint32_t *__restrict__ b, uint32_t lmask, uint64_t stride_w,
                                                     int iters, uint32_t *__restrict__ out) {
    const uint32_t tid = blockIdx.x * 768 + threadIdx.x;
    uint32_t acc = 0;
    for (int it = 0; it < iters; it++) {
        const uint32_t i = mix(tid * 0x9E3779B9u + it) & amask;           // first read: 16 B of a 64-MiB table
        const u32x4 w = *reinterpret_cast<const u32x4 *>(a + 4ull * i);
        const uint32_t l = mix(w[0] ^ w[1] ^ it ^ tid) & lmask;            // the line it selects (dependent)
        const uint64_t slot = (uint64_t)(mix(l ^ 0x5bd1e995u) % (uint32_t)(stride_w / 16u)) * 16u;
        const u32x4 *p = reinterpret_cast<const u32x4 *>(b + (uint64_t)l * stride_w + slot);
        const u32x4 x = p[0], y = p[1], z = p[2], v = p[3];
        acc += x[0] ^ y[1] ^ z[2] ^ v[3];
    }
    out[tid] = acc;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int grid = cus * 2;
    const uint64_t abytes = 64ull << 20, max_b = 12ull << 30;
    uint32_t *a, *b, *out;
    if (hipMalloc(&a, abytes) != hipSuccess || hipMalloc(&b, max_b) != hipSuccess) return 1;
    if (hipMalloc(&out, (size_t)grid * 768 * 4) != hipSuccess) return 1;
    // random words in the first table so the dependent index is unpredictable
    uint32_t *h = (uint32_t *)malloc(abytes);
    for (uint64_t k = 0; k < abytes / 4; k++) h[k] = (uint32_t)(k * 0x9E3779B97F4A7C15ull >> 32) ^ (uint32_t)k;
    if (hipMemcpy(a, h, abytes, hipMemcpyHostToDevice) != hipSuccess) return 1;
    free(h);
    if (hipMemset(b, 1, max_b) != hipSuccess) return 1;
    const int iters = 32, reps = 5;
    for (uint64_t f : {64ull << 20, 1ull << 30})
        for (uint64_t span : {1ull << 30, 4ull << 30, 8ull << 30, 12ull << 30}) {
            const uint64_t lines = f / 128, stride = span / lines;  // a 64-B line at a random 16-B slot per window
            hipLaunchKernelGGL(dep_pairs, dim3(grid), dim3(768), 0, 0, a, (uint32_t)(abytes / 16 - 1), b,
                               (uint32_t)(lines - 1), stride / 4, iters, out);
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0, 0);
            for (int r = 0; r < reps; r++)
                hipLaunchKernelGGL(dep_pairs, dim3(grid), dim3(768), 0, 0, a, (uint32_t)(abytes / 16 - 1), b,
                                   (uint32_t)(lines - 1), stride / 4, iters, out);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double pairs = (double)grid * 768 * iters * reps;
            printf("{\"test\": \"dep_pairs\", \"footprint_MiB\": %.0f, \"span_MiB\": %.0f, \"Gpairs_s\": %.2f}\n",
                   f / 1048576.0, span / 1048576.0, pairs / (ms * 1e-3) / 1e9);
            fflush(stdout);
        }
    return 0;
}
