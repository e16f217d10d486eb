/*
 * infw_host.h — host-side helpers of the host-fed AF_XDP path (libinfw.so; the types are infw.h's).
 *
 * infw_classify_xdp_host (infw.h) classifies AF_XDP rings whose umem sits in host memory and returns result words,
 * verdicts and per-rule counters.  The reference's program also emits a perf event for every denied packet
 * (bpf/ingress_node_firewall_kernel.c:392-399) that the events reader turns into syslog lines
 * (pkg/ebpf/ingress_node_firewall_events.go:77-166).  For frames in HBM the device writes those samples
 * (infw_classify_frames_ex + infw_events_capture); for frames in host memory the daemon already holds every frame, so
 * the samples are built on the host from the ring and the result words — byte for byte the layout
 * infw_events_capture writes.
 */
#ifndef INFW_HOST_H
#define INFW_HOST_H

#include "infw.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Deny-event perf samples of one AF_XDP ring (kernel.c:392-399).  For every    */
/* descriptor i whose result word (results[i], as infw_classify_xdp_host wrote  */
/* it) has action XDP_DROP, in ring order, slot k of `samples` gets size =       */
/* round_up(8 + captured + 4, 8) - 4 and raw = event_hdr_st {ifId = ifindex &    */
/* 0xFFFF, ruleId = results[i] >> 8 & 0xFFFF, action = 1, pad = 0, pktLength =   */
/* len & 0xFFFF}, then the frame's first captured = min(len, 256) bytes, then   */
/* zeros to the end of the slot — the layout of infw_events_capture.  Frames     */
/* are found as infw_classify_xdp_host finds them (aligned or unaligned mode).  */
/* *count = the ring's events, also those past `cap` (perf's lost samples).     */
/* Pure host function: no context or device.  0, or -EINVAL.                    */
int infw_xdp_host_events(const uint8_t *umem, const struct infw_xdp_desc *descs, uint64_t n, uint32_t ifindex,
                         const uint32_t *results, struct infw_event_sample *samples, uint64_t cap,
                         uint64_t *count);

/* ------------------------------------------------------------------------ */
/* DPDK-style bursts (SURVEY.md §8f-3 "AF_XDP/DPDK-style NIC feed"): frames  */
/* anywhere in host memory, one pointer per frame — an rte_mbuf burst's       */
/* rte_pktmbuf_mtod(m) with data_len (the first segment's bytes: the linear   */
/* part the program can read) and pkt_len (the whole frame, every segment:    */
/* bpf_xdp_get_buff_len) — or frames a capture file or any other source holds. */
/* One burst = one port = one ifindex.                                        */
/* ------------------------------------------------------------------------ */
struct infw_frame_burst {
    const uint8_t *const *frames;  /* frames[i]: the frame's first byte                            */
    const uint32_t *linear_len;    /* bytes readable at frames[i] (data_len)                       */
    const uint32_t *pkt_len;       /* whole-frame length (pkt_len), or NULL: = linear_len          */
    uint64_t n;
    uint32_t ifindex;
    uint32_t flags;                /* 0                                                           */
    uint32_t *results;             /* n result words, or NULL                                     */
    uint8_t *verdicts;             /* n XDP verdicts, or NULL                                     */
};
/* infw_classify_xdp_host for bursts: the context's packer threads read each  */
/* frame's header window through its pointer (bytes at or past linear_len[i]  */
/* read as 0, as kernel.c's data_end checks make them) and the packed tuples  */
/* are pipelined through the device exactly as for AF_XDP rings (same chunks, */
/* same options, same results as infw_classify_frames on the same frames).    */
/* Synchronous; the whole call reads one table epoch.  Hand many bursts to    */
/* one call (every port's rx bursts of a poll round): the call copies none   */
/* of the array (two passes over it, split over up to 8 threads for a call   */
/* of many bursts); result arrays that continue one                           */
/* another (slices of one array) come back in one copy per run, arrays of     */
/* their own are staged per chunk and scattered by the calling thread.        */
/* -EINVAL for a burst with flags set or a null frames / linear_len array     */
/* (nothing classified), -ENODEV for a host-only context.                     */
int infw_classify_bursts_host(infw_ctx *ctx, int dev, const struct infw_frame_burst *bursts, uint32_t n_bursts,
                              uint64_t chunk);
/* The burst packer alone on the calling thread (family-compact streams, as   */
/* infw_pack_xdp_host writes them; out->ifindex may be NULL).  Pure host.     */
int infw_pack_burst_host(const struct infw_frame_burst *burst, const struct infw_batch_soa_c_out *out);
/* Deny-event perf samples of one burst from its result words, as             */
/* infw_xdp_host_events (captured = min(pkt_len, 256); bytes at or past       */
/* linear_len — other mbuf segments — written as zeros, as infw_events_capture */
/* writes them for frames in HBM).  Pure host.  0, or -EINVAL.                */
int infw_burst_host_events(const struct infw_frame_burst *burst, const uint32_t *results,
                           struct infw_event_sample *samples, uint64_t cap, uint64_t *count);

#ifdef __cplusplus
}
#endif

#endif /* INFW_HOST_H */
