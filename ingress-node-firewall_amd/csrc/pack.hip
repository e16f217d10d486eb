// pack.hip — raw frames in HBM -> SoA header tuples.
//
// One lane per frame; the tuple is exactly infw_pack_header()'s (infw_pack.h), which the host packer and the
// generator share: the bytes the XDP program reads (ethertype, L3 proto, source address, first L4 word:
// kernel.c:104-166, :204, :291), each read as 0 at or past the frame's linear length.
//
// Frames sit at a stride or at arbitrary byte offsets, so a lane reading its own frame's bytes would issue ~25
// byte loads each touching a different cache line per wave.  Instead a wave stages the header window of its 64
// frames — bytes [10, 58) of each, covered by four 16-B aligned chunks from ((frame + 10) & ~15) — through LDS:
// in each of four rounds, lanes 4j..4j+3 load the four chunks of one frame (64 contiguous bytes: one request per
// frame instead of one per byte), then every lane picks its frame's bytes out of LDS.  A chunk is loaded only if
// it starts before min(linear length, 58): it then holds a byte of the frame, so the aligned 16-B access never
// leaves the frame's memory (frames packed back to back stay safe to read); chunks not loaded read as zero.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/infw.h"
#include "infw_pack.h"

namespace {

struct PackOut {  // standard (saddr) or family-compact (saddr4 + v6tail) address layout
    uint8_t *saddr;
    uint32_t *saddr4;
    uint8_t *v6tail;
    uint32_t *ifindex, *pkt_len, *meta, *l4word;
};

constexpr uint32_t kWinLo = 10, kWinHi = 58;  // header bytes any tuple field can come from
constexpr uint32_t kWinWords = 17;             // 64-B window + 4 B: lanes' windows 17 banks apart

template <bool kC>
__global__ __launch_bounds__(256) void pack_frames_kernel(const infw_frame_batch fb, uint64_t n, PackOut out) {
    __shared__ uint32_t win[4][64 * kWinWords];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t *ww = win[wv];
    // block-uniform trip count (the barriers below); the compact layout ranks a group's IPv6 lanes with one ballot
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < n; base += stride) {
        const uint64_t wbase = base + 64u * wv;
        for (uint32_t r = 0; r < 4; r++) {  // round r: chunk (lane & 3) of frame 16r + (lane >> 2)
            const uint32_t j = 16 * r + (lane >> 2), c = lane & 3u;
            const uint64_t fi = wbase + j;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (fi < n) {
                const uint8_t *f = fb.frames + (fb.offsets ? fb.offsets[fi] : fi * fb.stride);
                const uint32_t lin = fb.linear_len[fi];
                const uintptr_t first = ((uintptr_t)f + kWinLo) & ~(uintptr_t)15, at = first + 16u * c;
                if (lin > kWinLo && at < (uintptr_t)f + (lin < kWinHi ? lin : kWinHi))
                    v = *reinterpret_cast<const uint4 *>(at);
            }
            uint32_t *d = ww + j * kWinWords + 4 * c;
            d[0] = v.x;
            d[1] = v.y;
            d[2] = v.z;
            d[3] = v.w;
        }
        __syncthreads();
        const uint64_t i = wbase + lane;
        const bool valid = i < n;
        uint32_t ethertype = 0, proto = 0, l4off = 0, soff = 0, slen = 0, cap = 0, plen = 0, d = 0;
        if (valid) {
            const uint8_t *f = fb.frames + (fb.offsets ? fb.offsets[i] : i * fb.stride);
            cap = fb.linear_len[i];
            plen = fb.pkt_len ? fb.pkt_len[i] : cap;
            d = (uint32_t)(((uintptr_t)f + kWinLo) & 15u);  // the window's byte kWinLo sits at chunk offset d
        }
        const uint8_t *wb = reinterpret_cast<const uint8_t *>(ww + lane * kWinWords) + d - kWinLo;
        auto byte_at = [&](uint32_t off) -> uint32_t { return off < cap ? (uint32_t)wb[off] : 0u; };
        if (valid && cap >= 14) {
            ethertype = byte_at(12) << 8 | byte_at(13);
            if (ethertype == 0x0800) {
                proto = byte_at(23);
                l4off = 34; soff = 26; slen = 4;
            } else if (ethertype == 0x86DD) {
                proto = byte_at(20);
                l4off = 54; soff = 22; slen = 16;
            }
        }
        uint32_t sw[4] = {0, 0, 0, 0};
        for (uint32_t k = 0; k < 16; k++)
            if (k < slen) sw[k >> 2] |= byte_at(soff + k) << (8 * (k & 3));
        uint32_t l4 = 0;
        if (l4off)
            for (uint32_t k = 0; k < 4; k++) l4 |= byte_at(l4off + k) << (8 * k);
        if (kC) {
            const bool is6 = ethertype == 0x86DD;  // == the meta ethertype the classifier ranks by
            const uint64_t m6 = __ballot(is6);
            if (valid) out.saddr4[i] = sw[0];
            if (is6) {
                const uint32_t rank = __popcll(m6 & ((1ull << lane) - 1));
                uint32_t *t = reinterpret_cast<uint32_t *>(out.v6tail + (i >> 6) * (12ull * INFW_V6_GROUP)) + 3 * rank;
                t[0] = sw[1];
                t[1] = sw[2];
                t[2] = sw[3];
            }
        } else if (valid) {
            reinterpret_cast<uint4 *>(out.saddr)[i] = make_uint4(sw[0], sw[1], sw[2], sw[3]);
        }
        if (valid) {
            out.ifindex[i] = fb.ifindex[i];
            out.pkt_len[i] = plen;
            out.meta[i] = ethertype | proto << 16 | (cap > 255u ? 255u : cap) << 24;
            out.l4word[i] = l4;
        }
        __syncthreads();  // the window is rewritten by the next iteration
    }
}

}  // namespace

// out: standard layout, or (out == nullptr) out_c: the family-compact layout.
extern "C" int infw_launch_pack_frames(const infw_frame_batch *fb, uint64_t n, const infw_batch_soa_out *out,
                                       const infw_batch_soa_c_out *out_c, uint32_t cus, hipStream_t stream) {
    if (n == 0) return 0;
    uint64_t blocks = (n + 255) / 256, cap = (uint64_t)cus * 8;
    const dim3 grid((uint32_t)(blocks < cap ? blocks : cap));
    if (out) {
        const PackOut o{out->saddr, nullptr, nullptr, out->ifindex, out->pkt_len, out->meta, out->l4word};
        hipLaunchKernelGGL(pack_frames_kernel<false>, grid, dim3(256), 0, stream, *fb, n, o);
    } else {
        const PackOut o{nullptr, out_c->saddr4, out_c->v6tail, out_c->ifindex, out_c->pkt_len, out_c->meta, out_c->l4word};
        hipLaunchKernelGGL(pack_frames_kernel<true>, grid, dim3(256), 0, stream, *fb, n, o);
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// Deny-event perf samples (kernel.c:392-399): one wave per ring record, lane l writes bytes [8l, 8l + 8) of the
// record's 272-B slot {u32 raw size, event_hdr_st, min(len, 256) frame bytes, zero pad}.  Events are a small
// fraction of a batch, so the byte-granular frame reads (frames sit at arbitrary offsets) are not the cost.
namespace {
__global__ __launch_bounds__(256) void event_samples_kernel(const infw_frame_batch fb,
                                                            const infw_event_rec *__restrict__ ev, uint64_t cap,
                                                            const uint64_t *__restrict__ count, uint64_t n_frames,
                                                            uint8_t *__restrict__ out) {
    static_assert(INFW_EVENT_SAMPLE_BYTES % 8 == 0 && INFW_EVENT_SAMPLE_BYTES / 8 <= 64, "one wave per slot");
    const uint64_t c = *count;
    const uint64_t n = c < cap ? c : cap;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t r = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < n; r += waves) {
        if (lane >= INFW_EVENT_SAMPLE_BYTES / 8) continue;
        const infw_event_rec e = ev[r];
        const uint64_t i = e.pkt_index;
        const bool in_batch = i < n_frames;  // a record of another batch: header only, no frame read
        const uint8_t *f = in_batch ? fb.frames + (fb.offsets ? fb.offsets[i] : i * fb.stride) : nullptr;
        const uint32_t linear = in_batch ? fb.linear_len[i] : 0u;
        const uint32_t captured = e.captured;
        const uint32_t size = ((8u + captured + 4u + 7u) & ~7u) - 4u;
        uint64_t hw;
        __builtin_memcpy(&hw, &e.hdr, 8);
        uint64_t w = 0;
        for (uint32_t k = 0; k < 8; k++) {
            const uint32_t b = 8 * lane + k;
            uint32_t v = 0;
            if (b < 4)
                v = size >> (8 * b) & 0xFFu;
            else if (b < 12)
                v = (uint32_t)(hw >> (8 * (b - 4))) & 0xFFu;
            else if (b - 12 < captured && b - 12 < linear)
                v = f[b - 12];
            w |= (uint64_t)v << (8 * k);
        }
        reinterpret_cast<uint64_t *>(out + r * INFW_EVENT_SAMPLE_BYTES)[lane] = w;
    }
}
}  // namespace

extern "C" int infw_launch_event_samples(const infw_frame_batch *fb, const infw_event_rec *ev, uint64_t cap,
                                         const uint64_t *count, uint64_t n_frames, infw_event_sample *samples,
                                         uint32_t cus, hipStream_t stream) {
    if (cap == 0) return 0;
    const uint64_t blocks = (cap + 3) / 4, lim = 4ull * cus;  // 4 waves (records) per block
    hipLaunchKernelGGL(event_samples_kernel, dim3((uint32_t)(blocks < lim ? blocks : lim)), dim3(256), 0, stream, *fb,
                       ev, cap, count, n_frames, reinterpret_cast<uint8_t *>(samples));
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// Standard -> family-compact address layout (infw_batch_soa_c): one lane per packet,
// packets of a wave = one INFW_V6_GROUP group; an IPv6 lane's rank among the group's
// IPv6 lanes places its 12 tail bytes.
namespace {
__global__ __launch_bounds__(256) void soa_compact_kernel(const uint8_t *__restrict__ saddr, const uint32_t *__restrict__ meta,
                                                          uint64_t n, uint32_t *__restrict__ saddr4,
                                                          uint8_t *__restrict__ v6tail) {
    static_assert(INFW_V6_GROUP == 64, "one wave per group");
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < n; base += stride) {
        const uint64_t i = base + threadIdx.x;
        const bool valid = i < n;
        const uint32_t *s = reinterpret_cast<const uint32_t *>(saddr + 16 * (valid ? i : 0));
        const bool is6 = valid && (meta[i] & 0xFFFFu) == 0x86DDu;
        const uint64_t m6 = __ballot(is6);
        if (valid) saddr4[i] = s[0];
        if (is6) {
            const uint32_t lane = threadIdx.x & 63u;
            const uint32_t rank = __popcll(m6 & ((1ull << lane) - 1));
            uint32_t *t = reinterpret_cast<uint32_t *>(v6tail + (i >> 6) * (12ull * INFW_V6_GROUP)) + 3 * rank;
            t[0] = s[1];
            t[1] = s[2];
            t[2] = s[3];
        }
    }
}
}  // namespace

extern "C" int infw_launch_soa_compact(const infw_batch_soa *in, uint64_t n, uint32_t *saddr4, uint8_t *v6tail,
                                       uint32_t cus, hipStream_t stream) {
    if (n == 0) return 0;
    const uint64_t blocks = (n + 255) / 256, cap = 8ull * cus;
    hipLaunchKernelGGL(soa_compact_kernel, dim3((uint32_t)(blocks < cap ? blocks : cap)), dim3(256), 0, stream,
                       in->saddr, in->meta, n, saddr4, v6tail);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
