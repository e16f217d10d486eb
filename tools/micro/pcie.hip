// Microbenchmark: what the GPU can read from pinned host memory over PCIe — the ceiling of the AF_XDP feed with the
// umem in host memory (infw_classify_xdp reads one 64-B header window and one 16-B descriptor per frame in place).
//   dense     every lane streams consecutive 16-B words (the coalesced bandwidth)
//   win4      frame f's 64-B window at f * stride read by 4 lanes, 16 B each (the classify kernel's staging form)
//   win1      the same window read by one lane, four 16-B loads
//   win4desc  win4 plus a 16-B descriptor per frame read before it (the descriptor names the frame: dependent)
// at 8 / 16 / 24 / 32 waves per CU; reports GB/s and frames/s.  HBM as the source for comparison.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/pcie.hip -o tools/micro/pcie && ./tools/micro/pcie
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                         \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                    \
        }                                                                                \
    } while (0)

template <int kMode>  // 0 dense, 1 win4, 2 win1, 3 win4desc
__global__ __launch_bounds__(512) void rd(const uint8_t *__restrict__ src, const u32x4 *__restrict__ desc,
                                          uint64_t n_units, uint64_t stride, uint32_t *__restrict__ out) {
    const uint64_t tid = (uint64_t)blockIdx.x * 512 + threadIdx.x, nth = (uint64_t)gridDim.x * 512;
    uint32_t acc = 0;
    if (kMode == 0) {  // n_units 16-B words
        const u32x4 *p = reinterpret_cast<const u32x4 *>(src);
        for (uint64_t i = tid; i < n_units; i += nth) {
            const u32x4 v = __builtin_nontemporal_load(p + i);
            acc += v[0] ^ v[1] ^ v[2] ^ v[3];
        }
    } else if (kMode == 1 || kMode == 3) {  // n_units frames, 4 lanes each
        for (uint64_t i = tid; i < 4 * n_units; i += nth) {
            const uint64_t f = i >> 2;
            uint64_t base = f * stride;
            if (kMode == 3) {
                const u32x4 d = __builtin_nontemporal_load(desc + f);
                base = (uint64_t)d[1] << 32 | d[0];
            }
            const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src + base) + (i & 3));
            acc += v[0] ^ v[1] ^ v[2] ^ v[3];
        }
    } else {  // one lane per frame
        for (uint64_t f = tid; f < n_units; f += nth) {
            const u32x4 *p = reinterpret_cast<const u32x4 *>(src + f * stride);
            const u32x4 a = __builtin_nontemporal_load(p), b = __builtin_nontemporal_load(p + 1),
                        c = __builtin_nontemporal_load(p + 2), d = __builtin_nontemporal_load(p + 3);
            acc += a[0] ^ b[1] ^ c[2] ^ d[3];
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int kMode>
static double run(const uint8_t *src, const u32x4 *desc, uint64_t n, uint64_t stride, uint32_t *out, int cus, int wpc) {
    const int blocks = cus * wpc / 8;  // 512 threads = 8 waves
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(rd<kMode>, dim3(blocks), dim3(512), 0, 0, src, desc, n, stride, out);
    (void)hipEventRecord(a, 0);
    const int reps = 5;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(rd<kMode>, dim3(blocks), dim3(512), 0, 0, src, desc, n, stride, out);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return ms / reps;
}

int main() {
    int cus = 256;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint64_t stride = 2048, frames = 1ull << 21, bytes = frames * stride;  // 4 GiB of 2048-B chunks
    uint8_t *host = nullptr, *dev = nullptr;
    u32x4 *hdesc = nullptr, *ddesc = nullptr;
    uint32_t *out = nullptr;
    CHECK(hipHostMalloc(reinterpret_cast<void **>(&host), bytes, hipHostMallocDefault));
    CHECK(hipHostMalloc(reinterpret_cast<void **>(&hdesc), frames * 16, hipHostMallocDefault));
    CHECK(hipMalloc(&dev, bytes));
    CHECK(hipMalloc(&ddesc, frames * 16));
    CHECK(hipMalloc(&out, 4));
    memset(host, 1, bytes);
    for (uint64_t f = 0; f < frames; f++) {
        const uint64_t a = f * stride;
        hdesc[f] = u32x4{(uint32_t)a, (uint32_t)(a >> 32), 64u, 0u};
    }
    CHECK(hipMemcpy(dev, host, bytes, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(ddesc, hdesc, frames * 16, hipMemcpyHostToDevice));
    for (int where = 0; where < 2; where++) {
        const uint8_t *src = where ? dev : host;
        const u32x4 *desc = where ? ddesc : hdesc;
        const char *w = where ? "hbm" : "host";
        for (int wpc : {8, 16, 24, 32}) {
            const double d = run<0>(src, desc, bytes / 16 / 8, stride, out, cus, wpc);  // 512 MiB dense
            const double w4 = run<1>(src, desc, frames, stride, out, cus, wpc);
            const double w1 = run<2>(src, desc, frames, stride, out, cus, wpc);
            const double wd = run<3>(src, desc, frames, stride, out, cus, wpc);
            printf("{\"src\": \"%s\", \"waves_per_cu\": %d, \"dense_GBps\": %.1f, \"win4_Mframes_s\": %.1f, "
                   "\"win1_Mframes_s\": %.1f, \"win4desc_Mframes_s\": %.1f}\n",
                   w, wpc, bytes / 8 / d / 1e6, frames / w4 / 1e3, frames / w1 / 1e3, frames / wd / 1e3);
            fflush(stdout);
        }
    }
    CHECK(hipDeviceSynchronize());
    // The copy engines instead of the compute units (SDMA): hipMemcpy2DAsync gathering each chunk's 64-B header window
    // (width 64 at pitch 2048) from pinned host memory into a dense HBM array — the one-copy-per-batch alternative to
    // the classify kernel reading windows in place — on 1, 2 and 4 streams (each stream's copies go to one engine),
    // beside dense H2D / D2H copies of the same bytes for the link's bulk rate.
    {
        uint8_t *dense = nullptr;
        CHECK(hipMalloc(&dense, frames * 64));
        hipStream_t st[4];
        for (auto &s : st) CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        auto timed = [&](int ns, int kind) -> double {  // kind 0: 2D gather, 1: dense H2D, 2: dense D2H
            double best = 1e30;
            for (int rep = 0; rep < 4; rep++) {
                CHECK(hipDeviceSynchronize());
                CHECK(hipEventRecord(a, st[0]));
                for (int s = 1; s < ns; s++) CHECK(hipStreamWaitEvent(st[s], a, 0));
                const uint64_t per = frames / ns;
                for (int s = 0; s < ns; s++) {
                    const uint64_t f0 = s * per;
                    if (kind == 0)
                        CHECK(hipMemcpy2DAsync(dense + f0 * 64, 64, host + f0 * stride, stride, 64, per,
                                               hipMemcpyHostToDevice, st[s]));
                    else if (kind == 1)
                        CHECK(hipMemcpyAsync(dense + f0 * 64, host + f0 * 64, per * 64, hipMemcpyHostToDevice, st[s]));
                    else
                        CHECK(hipMemcpyAsync(host + f0 * 64, dense + f0 * 64, per * 64, hipMemcpyDeviceToHost, st[s]));
                }
                for (int s = 1; s < ns; s++) {
                    hipEvent_t e;
                    CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
                    CHECK(hipEventRecord(e, st[s]));
                    CHECK(hipStreamWaitEvent(st[0], e, 0));
                    CHECK(hipEventDestroy(e));
                }
                CHECK(hipEventRecord(b, st[0]));
                CHECK(hipEventSynchronize(b));
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, a, b));
                if (ms < best) best = ms;
            }
            return best;
        };
        for (int ns : {1, 2, 4}) {
            const double g = timed(ns, 0), h = timed(ns, 1), d = timed(ns, 2);
            printf("{\"sdma_streams\": %d, \"gather2d_Mwindows_s\": %.1f, \"gather2d_GBps\": %.2f, "
                   "\"dense_h2d_GBps\": %.1f, \"dense_d2h_GBps\": %.1f, \"frames\": %llu}\n",
                   ns, frames / g / 1e3, frames * 64 / g / 1e6, frames * 64 / h / 1e6, frames * 64 / d / 1e6,
                   (unsigned long long)frames);
            fflush(stdout);
        }
        CHECK(hipFree(dense));
    }
    return 0;
}
