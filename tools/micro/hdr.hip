// Microbenchmark: reading the header window of N frames in HBM (128-B stride, AF_XDP-style chunks) — the
// first 64 B of each frame, where every byte the classifier needs sits (frame[12..58)) — in three ways:
//   lane    each lane loads its own frame's four 16-B chunks (4 non-temporal dwordx4 per lane; every
//           instruction touches 64 lines)
//   lane_l1 the same with plain (L1-allocating) loads
//   staged  per round of 16 frames, lanes 4j..4j+3 load the four chunks of frame j (one instruction = 16 whole
//           64-B windows), the wave parks them in a 1-KiB LDS buffer of its own, and the round's 16 owner lanes
//           read the dwords the tuple needs (7 ds_read2_b32) — the pattern a fused frames classifier would use
// Each lane folds the dwords into a checksum stored per frame (4 B), so the loads cannot be elided.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/hdr.hip -o tools/micro/hdr && tools/micro/hdr
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool kNT>
__global__ __launch_bounds__(256) void hdr_lane(const uint8_t *__restrict__ frames, uint64_t stride, uint64_t n,
                                                uint32_t *__restrict__ out) {
    const uint64_t step = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += step) {
        const u32x4 *f = reinterpret_cast<const u32x4 *>(frames + i * stride);
        u32x4 a, b, c, d;
        if (kNT) {
            a = __builtin_nontemporal_load(f);
            b = __builtin_nontemporal_load(f + 1);
            c = __builtin_nontemporal_load(f + 2);
            d = __builtin_nontemporal_load(f + 3);
        } else {
            a = f[0];
            b = f[1];
            c = f[2];
            d = f[3];
        }
        const uint32_t s = a[3] ^ b[1] ^ b[2] ^ b[3] ^ c[0] ^ c[1] ^ c[2] ^ d[1] ^ d[2];
        __builtin_nontemporal_store(s, &out[i]);
    }
}

template <int kBlock>
__global__ __launch_bounds__(kBlock) void hdr_staged(const uint8_t *__restrict__ frames, uint64_t stride, uint64_t n,
                                                     uint32_t *__restrict__ out) {
    constexpr int kWaves = kBlock / 64;
    __shared__ uint32_t buf[kWaves][16 * 17];  // 16 frames x (64 B + 4 B pad)
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t *bw = buf[wv];
    const uint64_t step = (uint64_t)gridDim.x * kBlock;
    for (uint64_t base = (uint64_t)blockIdx.x * kBlock + 64u * wv; base < n; base += step) {
        uint32_t s = 0;
        u32x4 v[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {  // all four rounds' loads in flight together
            const uint64_t fi = base + 16 * r + (lane >> 2);
            v[r] = fi < n ? __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(frames + fi * stride) + (lane & 3))
                          : u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            uint32_t *d = bw + (lane >> 2) * 17 + 4 * (lane & 3);
            d[0] = v[r][0];
            d[1] = v[r][1];
            d[2] = v[r][2];
            d[3] = v[r][3];
            __builtin_amdgcn_wave_barrier();
            if ((lane >> 4) == (uint32_t)r) {
                const uint32_t *w = bw + (lane & 15) * 17;
                s = w[3] ^ w[5] ^ w[6] ^ w[7] ^ w[8] ^ w[9] ^ w[13] ^ w[14];
            }
            __builtin_amdgcn_wave_barrier();
        }
        const uint64_t i = base + lane;
        if (i < n) __builtin_nontemporal_store(s, &out[i]);
    }
}

template <class F>
void timeit(const char *name, int bpc, int block, uint64_t n, F launch) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    launch();
    hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; r++) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    printf("{\"variant\": \"%s\", \"block\": %d, \"blocks_per_cu\": %d, \"frames\": %llu, \"ms\": %.3f, \"Gframes_s\": %.2f, "
           "\"GBps_64B\": %.0f}\n", name, block, bpc, (unsigned long long)n, ms, n / (ms * 1e-3) / 1e9,
           n * 64.0 / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

int main() {
    const uint64_t n = 1ull << 27, stride = 128;
    uint8_t *frames;
    uint32_t *out;
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    if (hipMalloc(&frames, n * stride) != hipSuccess || hipMalloc(&out, n * 4) != hipSuccess) return 1;
    hipMemset(frames, 3, n * stride);
    for (int bpc : {4, 8}) {
        const uint32_t g = (uint32_t)(cus * bpc);
        timeit("lane", bpc, 256, n, [&] { hdr_lane<true><<<g, 256>>>(frames, stride, n, out); });
        timeit("lane_l1", bpc, 256, n, [&] { hdr_lane<false><<<g, 256>>>(frames, stride, n, out); });
        timeit("staged", bpc, 256, n, [&] { hdr_staged<256><<<g, 256>>>(frames, stride, n, out); });
    }
    timeit("staged", 2, 768, n, [&] { hdr_staged<768><<<(uint32_t)(cus * 2), 768>>>(frames, stride, n, out); });
    hipFree(frames);
    hipFree(out);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
