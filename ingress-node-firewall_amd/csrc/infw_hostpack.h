// infw_hostpack.h — AF_XDP RX descriptors over a host umem -> family-compact SoA tuples, on host CPU threads.
//
// The host half of infw_classify_xdp_host (include/infw.h): a frame's header window is read by the CPU where the NIC
// left it (host memory, never touched by the GPU), and only the tuple the classifier needs crosses PCIe — 20 B per
// packet plus 12 B of address tail for IPv6 — in bulk DMA copies instead of one 64-B read request per frame
// (infw_classify_xdp over a host umem is bound by that request rate: DESIGN.md §6).
//
// The tuple is infw_pack_header()'s (infw_pack.h) — the bytes bpf/ingress_node_firewall_kernel.c reads at fixed
// offsets: ethertype frame[12..13] (:427), L3 proto frame[23] / frame[20] (:108, :115), source address frame[26..29] /
// frame[22..37] (:204, :291), first L4 word frame[34..37] / frame[54..57] (:125-166), each byte read as 0 at or past
// the frame's linear length.  A frame of at least 58 linear bytes (every field in place) takes the branch-free form
// below; shorter ones go through infw_pack_header itself.  Both give identical tuples (tests/test_hostpack_cpu.py).
//
// Host code only (no HIP): libinfw's packer threads and tools/micro/hostpack.cpp include it.
#pragma once
#include <stdint.h>
#include <string.h>

#include "../../include/infw.h"
#include "infw_pack.h"

#if defined(__x86_64__)
#include <immintrin.h>
#endif

// One part of a chunk's family-compact streams (include/infw.h infw_batch_soa_c): index 0 of every stream is packet 0
// of the part, and the part starts on an INFW_V6_GROUP boundary of the chunk, so v6tail points at the part's first
// group block.
struct infw_hostpack_out {  // ifindex may be null (not written)
    uint32_t *saddr4;
    uint8_t *v6tail;
    uint32_t *ifindex, *pkt_len, *meta, *l4word;
};

// Frame bytes of descriptor `addr`: aligned mode, or unaligned mode's offset in bits 48..63
// (XSK_UNALIGNED_BUF_OFFSET_SHIFT) — as infw_classify_xdp reads them.
static inline const uint8_t *infw_xdp_frame(const uint8_t *umem, uint64_t addr) {
    return umem + (addr & ((1ull << 48) - 1)) + (addr >> 48);
}

static inline uint32_t infw_ld32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}

// Stores of the packed streams.  kNT: around the cache (non-temporal — the streams are written once and then read by
// the DMA engine: no read-for-ownership of the pinned destination lines, no eviction of headers still to be read),
// at the price of write-combining buffers that the header loads' misses also need.
template <bool kNT>
static inline void infw_st32(uint32_t *p, uint32_t v) {
#if defined(__x86_64__)
    if (kNT) {
        _mm_stream_si32(reinterpret_cast<int *>(p), (int)v);
        return;
    }
#endif
    *p = v;
}

// Pack descriptors [0, n) into `o` (n may be ragged: the last group is partial).  kPF: prefetch distance in frames —
// the headers are DRAM misses (a NIC wrote them; one 64-B line per 2-KiB chunk), so a core keeps kPF of them in flight.
template <int kPF, bool kNT>
static inline void infw_hostpack_xdp(const uint8_t *umem, const infw_xdp_desc *d, uint64_t n, uint32_t ifindex,
                                     const infw_hostpack_out &o) {
    uint32_t rank = 0;       // IPv6 packets so far in the current group
    uint32_t *tail = nullptr;  // the current group's v6tail block
    for (uint64_t i = 0; i < n; i++) {
        if (kPF && i + kPF < n) {
            const uint8_t *p = infw_xdp_frame(umem, d[i + kPF].addr);
            __builtin_prefetch(p + 10);
            __builtin_prefetch(p + 57);
        }
        if ((i & (INFW_V6_GROUP - 1)) == 0) {
            rank = 0;
            tail = reinterpret_cast<uint32_t *>(o.v6tail + (i / INFW_V6_GROUP) * (12ull * INFW_V6_GROUP));
        }
        const uint64_t addr = d[i].addr;
        const uint32_t len = d[i].len;
        const uint8_t *f = infw_xdp_frame(umem, addr);
        uint32_t s0, s1, s2, s3, l4, meta;
        if (__builtin_expect(len >= 58, 1)) {
            const uint32_t et = (uint32_t)f[12] << 8 | f[13];
            const bool v4 = et == 0x0800, v6 = et == 0x86DD;
            const uint32_t ip = (v4 || v6) ? ~0u : 0u;
            const uint32_t proto = f[v6 ? 20 : 23] & ip;
            s0 = infw_ld32(f + (v6 ? 22 : 26)) & ip;
            l4 = infw_ld32(f + (v6 ? 54 : 34)) & ip;
            s1 = infw_ld32(f + 26);
            s2 = infw_ld32(f + 30);
            s3 = infw_ld32(f + 34);
            meta = et | proto << 16 | (len > 255u ? 255u : len) << 24;
        } else {
            infw_tuple t;
            infw_pack_header(f, len, len, ifindex, &t);
            s0 = t.saddr[0], s1 = t.saddr[1], s2 = t.saddr[2], s3 = t.saddr[3];
            l4 = t.l4word;
            meta = t.meta;
        }
        const bool is6 = (meta & 0xFFFFu) == 0x86DDu;  // the ethertype the classifier ranks a group's tails by
        // the tail slot is written unconditionally and kept only for IPv6 (the next packet overwrites it otherwise):
        // no branch on the family, and rank <= 63 keeps the slot inside the group's block
        infw_st32<kNT>(tail + 3 * rank, s1);
        infw_st32<kNT>(tail + 3 * rank + 1, s2);
        infw_st32<kNT>(tail + 3 * rank + 2, s3);
        rank += is6;
        infw_st32<kNT>(o.saddr4 + i, s0);
        if (o.ifindex) infw_st32<kNT>(o.ifindex + i, ifindex);  // null: the ifindex stream is filled on the device
        infw_st32<kNT>(o.pkt_len + i, len);
        infw_st32<kNT>(o.meta + i, meta);
        infw_st32<kNT>(o.l4word + i, l4);
    }
#if defined(__x86_64__)
    if (kNT) _mm_sfence();  // the non-temporal stores are globally visible before the part is reported done
#endif
}
