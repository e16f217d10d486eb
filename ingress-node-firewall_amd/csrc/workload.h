// workload.h — synthetic workloads of BASELINE.json configs[0..4] (bench/test
// infrastructure, libinfw_workload.so; not part of the classifier ABI).
#pragma once
#include <stdint.h>

#include "../../include/infw.h"
#include "infw_gen.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct infw_wl infw_wl;

enum {
    INFW_WL_CFG0_DEMO = 0,       // config/samples demo-1 ingress[0] on ifindex 1, 1M packets
    INFW_WL_CFG1_V4_10K = 1,     // 10k IPv4 /16-/32 x 10 rules
    INFW_WL_CFG2_MIXED_1M = 2,   // 1M mixed v4/v6 BGP-like x 99 rules, 4 ifindexes, Zipf(1.1)
    INFW_WL_CFG4_ADVERSARIAL = 4 // /128 deepest hits, last-slot ICMPv6, cross-family aliasing
};

// n_prefixes / n_templates = 0 -> the config's defaults.
int infw_wl_create(infw_wl **out, int cfg, uint64_t seed, uint32_t n_prefixes, uint32_t n_templates);
void infw_wl_destroy(infw_wl *wl);

uint64_t infw_wl_n_entries(const infw_wl *wl);
const struct lpm_ip_key_st *infw_wl_keys(const infw_wl *wl);
const uint32_t *infw_wl_val_index(const infw_wl *wl);
uint32_t infw_wl_n_templates(const infw_wl *wl);
const struct rulesVal_st *infw_wl_templates(const infw_wl *wl);
// Host-side generator parameters (pointers into wl).
const struct infw_gen_params *infw_wl_params(const infw_wl *wl);
// Sources drawn uniformly over the prefixes instead of the config's Zipf law (tables unchanged).
void infw_wl_uniform_sources(infw_wl *wl);
// Overwrite the packet seed (tables unchanged).
void infw_wl_set_packet_seed(infw_wl *wl, uint64_t seed);

// Frames [start, start+n): header snapshots (INFW_HDR_SNAP B each), linear
// length, frame length, ifindex.  nthreads workers.
int infw_wl_frames(const infw_wl *wl, uint64_t start, uint64_t n, uint8_t *hdr, uint32_t *caplen,
                   uint32_t *pkt_len, uint32_t *ifindex, int nthreads);
// Tuples [start, start+n) on the host (n x 8 u32: saddr[4], ifindex, pkt_len, meta, l4word).
int infw_wl_tuples(const infw_wl *wl, uint64_t start, uint64_t n, uint32_t *tuples, int nthreads);
// Pack arbitrary frame header snapshots into tuples (host).
int infw_wl_pack(const uint8_t *hdr, const uint32_t *caplen, const uint32_t *pkt_len,
                 const uint32_t *ifindex, uint64_t n, uint32_t *tuples);

// Device generator: copies prefixes / CDF to device `hip_device` once, then
// writes SoA tuples of packets [start, start+n) straight into HBM.
int infw_wl_upload(infw_wl *wl, int hip_device);
int infw_wl_gen_soa(infw_wl *wl, uint64_t start, uint64_t n, uint8_t *saddr, uint32_t *ifindex,
                    uint32_t *pkt_len, uint32_t *meta, uint32_t *l4word, void *stream);
// Device generator of raw frames (an infw_frame_batch at a fixed stride >= INFW_HDR_SNAP): frame i holds the
// header snapshot infw_wl_frames gives for packet start+i; linear_len = min(linear length, INFW_HDR_SNAP).
int infw_wl_gen_frames(infw_wl *wl, uint64_t start, uint64_t n, uint8_t *frames, uint64_t stride,
                       uint32_t *linear_len, uint32_t *pkt_len, uint32_t *ifindex, void *stream);

#ifdef __cplusplus
}
#endif
