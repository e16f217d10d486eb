// patch.hip — copy the byte ranges an incremental commit changed (incremental.cpp)
// into a device table image: one staging upload, then one scatter launch.
#include <hip/hip_runtime.h>
#include <stdint.h>

struct infw_patch_desc {
    uint64_t dst;     // device address (4-byte aligned)
    uint64_t src;     // word offset into the staging buffer
    uint64_t nwords;
};

namespace {

// One workgroup per range at a time; consecutive lanes write consecutive words.
__global__ __launch_bounds__(256) void scatter_words(const uint32_t *__restrict__ src,
                                                     const infw_patch_desc *__restrict__ d, uint32_t n) {
    for (uint32_t r = blockIdx.x; r < n; r += gridDim.x) {
        uint32_t *dst = reinterpret_cast<uint32_t *>(d[r].dst);
        const uint32_t *s = src + d[r].src;
        const uint64_t nw = d[r].nwords;
        for (uint64_t k = threadIdx.x; k < nw; k += 256) dst[k] = s[k];
    }
}

}  // namespace

extern "C" int infw_launch_scatter(const uint32_t *staging, const void *descs, uint32_t n, uint32_t cus,
                                   hipStream_t stream) {
    if (n == 0) return 0;
    const uint32_t grid = n < 4 * cus ? n : 4 * cus;
    hipLaunchKernelGGL(scatter_words, dim3(grid), dim3(256), 0, stream, staging,
                       static_cast<const infw_patch_desc *>(descs), n);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
