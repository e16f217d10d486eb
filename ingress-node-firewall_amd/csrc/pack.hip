// pack.hip — raw frames in HBM -> SoA header tuples.
//
// One lane per frame.  The lane reads only the bytes the XDP program reads
// (ethertype, L3 proto, source address, first L4 word: kernel.c:104-166,
// :204, :291) and never a byte at or past the frame's linear length, so
// frames packed back to back in HBM are safe to read; the tuple is exactly
// infw_pack_header()'s (infw_pack.h), which the host packer and the generator
// share.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/infw.h"
#include "infw_pack.h"

namespace {

__device__ __forceinline__ uint32_t byte_at(const uint8_t *f, uint32_t cap, uint32_t off) {
    return off < cap ? (uint32_t)f[off] : 0u;
}

__global__ __launch_bounds__(256) void pack_frames_kernel(const infw_frame_batch fb, uint64_t n,
                                                          infw_batch_soa_out out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t *f = fb.frames + (fb.offsets ? fb.offsets[i] : i * fb.stride);
        const uint32_t cap = fb.linear_len[i];
        const uint32_t plen = fb.pkt_len ? fb.pkt_len[i] : cap;
        uint32_t ethertype = 0, proto = 0, l4off = 0, soff = 0, slen = 0;
        if (cap >= 14) {
            ethertype = byte_at(f, cap, 12) << 8 | byte_at(f, cap, 13);
            if (ethertype == 0x0800) {
                proto = byte_at(f, cap, 23);
                l4off = 34; soff = 26; slen = 4;
            } else if (ethertype == 0x86DD) {
                proto = byte_at(f, cap, 20);
                l4off = 54; soff = 22; slen = 16;
            }
        }
        uint32_t sw[4] = {0, 0, 0, 0};
        for (uint32_t k = 0; k < 16; k++)
            if (k < slen) sw[k >> 2] |= byte_at(f, cap, soff + k) << (8 * (k & 3));
        uint32_t l4 = 0;
        if (l4off)
            for (uint32_t k = 0; k < 4; k++) l4 |= byte_at(f, cap, l4off + k) << (8 * k);
        reinterpret_cast<uint4 *>(out.saddr)[i] = make_uint4(sw[0], sw[1], sw[2], sw[3]);
        out.ifindex[i] = fb.ifindex[i];
        out.pkt_len[i] = plen;
        out.meta[i] = ethertype | proto << 16 | (cap > 255u ? 255u : cap) << 24;
        out.l4word[i] = l4;
    }
}

}  // namespace

extern "C" int infw_launch_pack_frames(const infw_frame_batch *fb, uint64_t n, const infw_batch_soa_out *out,
                                       uint32_t cus, hipStream_t stream) {
    if (n == 0) return 0;
    uint64_t blocks = (n + 255) / 256, cap = (uint64_t)cus * 8;
    hipLaunchKernelGGL(pack_frames_kernel, dim3((uint32_t)(blocks < cap ? blocks : cap)), dim3(256), 0, stream, *fb,
                       n, *out);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
