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

#ifdef __cplusplus
}
#endif

#endif /* INFW_HOST_H */
