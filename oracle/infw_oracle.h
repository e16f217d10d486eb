/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference hot path, used as the parity checker by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Nothing in
 * the product (ingress-node-firewall_amd/) links, loads or calls this code.
 *
 * What it restates (reference = pbmoses/ingress-node-firewall @ 2025-01-14):
 *   - bpf/ingress_node_firewall_kernel.c:95-457   the XDP data path, byte for
 *     byte over raw frames (parse, LPM lookup, first-match scan, stats);
 *   - the LPM_TRIE map semantics the program relies on (kernel.c:50-57;
 *     Linux kernel/bpf/lpm_trie.c of the host kernel, 6.18 — a third-party
 *     dependency outside /root/reference): update / delete / longest-prefix
 *     lookup / get_next_key post-order, -ENOSPC on a full map;
 *   - the PERCPU_ARRAY statistics map (kernel.c:36-41): one slot per worker
 *     thread, summed like pkg/metrics/statistics.go:126-157.
 *
 * Pinning: the reference's prebuilt eBPF object is not loaded (task rule: no
 * prebuilt machine code shipped inside the reference is run) and the C source
 * cannot be rebuilt here (no BPF target in this image's clang).  The oracle is
 * pinned against the reference's own test fixtures and the survey's recorded
 * BPF_PROG_TEST_RUN observations (tests/golden/).
 *
 * Structs are restated here (not included from the product) on purpose.
 */
#ifndef INFW_ORACLE_H
#define INFW_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_TARGETS 1024          /* ingress_node_firewall.h:13 */
#define ORC_MAX_RULES 100             /* ingress_node_firewall.h:14 */
#define ORC_VALUE_SIZE 1200           /* sizeof(struct rulesVal_st) */
#define ORC_KEY_SIZE 24               /* sizeof(struct lpm_ip_key_st) */
#define ORC_MAX_PREFIXLEN 160         /* lpm_trie max_prefixlen = 8 * data_size(20) */

struct orc_stats {                    /* ruleStatistics_st, ingress_node_firewall.h:45-54 */
    uint64_t allow_packets, allow_bytes, deny_packets, deny_bytes;
};

struct orc_event {                    /* event_hdr_st (ingress_node_firewall.h:58-64) + packet index */
    uint64_t pkt_index;
    uint16_t ifId, ruleId;
    uint8_t action, pad;
    uint16_t pktLength;
    uint16_t captured;                /* min(len, MAX_EVENT_DATA): bytes attached to the perf record */
};

typedef struct orc_map orc_map;

orc_map *orc_map_create(uint32_t max_entries);
void orc_map_destroy(orc_map *m);
/* key: 24 B lpm_ip_key_st, val: 1200 B rulesVal_st.  bpf(2) error codes. */
int orc_map_update(orc_map *m, const uint8_t *key, const uint8_t *val, uint64_t flags);
int orc_map_delete(orc_map *m, const uint8_t *key);
int orc_map_lookup(const orc_map *m, const uint8_t *key, uint8_t *val_out);
int orc_map_get_next_key(const orc_map *m, const uint8_t *key /*NULL ok*/, uint8_t *next);
uint64_t orc_map_count(const orc_map *m);

/*
 * One XDP invocation (ingress_node_firewall_main, kernel.c:412-457).
 *   data/linear_len: the linear frame bytes (xdp data .. data_end)
 *   buff_len:        bpf_xdp_get_buff_len(ctx) (== linear_len without frags)
 *   stats:           this worker's per-CPU slot (1024 entries), may be NULL
 *   result_out:      the `result` word (0 when the frame never reaches a lookup)
 *   ev_out:          filled when a DENY event would be emitted (kernel.c:392-399)
 * returns the XDP action (1 DROP / 2 PASS).
 */
int orc_xdp_run(const orc_map *m, struct orc_stats *stats, const uint8_t *data,
                uint32_t linear_len, uint32_t buff_len, uint32_t ifindex,
                uint32_t *result_out, int *event_out);

/*
 * Batch over frames with nthreads workers (one stats slot per worker, summed
 * into stats_sum[1024]).  frame i = frames[offsets[i] .. offsets[i]+caplen[i]),
 * with linear length min(caplen[i], pkt_len[i]) and buff_len pkt_len[i]
 * (callers may store only the first caplen bytes of long frames: the program
 * never reads past byte 74).  results/verdicts may be NULL.
 * Returns elapsed seconds of the classification (wall clock).
 */
double orc_classify_frames(const orc_map *m, const uint8_t *frames, const uint64_t *offsets,
                           const uint32_t *caplen, const uint32_t *pkt_len,
                           const uint32_t *ifindex, uint64_t n, uint32_t *results,
                           uint8_t *verdicts, struct orc_stats *stats_sum, int nthreads);

/* Valid rules (ruleId != 0) the reference's first-match loop examines over a batch,
 * up to and including each packet's first match (x 12 B = rule bytes). */
uint64_t orc_rules_examined(const orc_map *m, const uint8_t *frames, const uint64_t *offsets,
                            const uint32_t *caplen, const uint32_t *pkt_len, const uint32_t *ifindex,
                            uint64_t n);

/* Events of a batch: fills up to max_events DENY events in packet order. */
uint64_t orc_collect_events(const orc_map *m, const uint8_t *frames, const uint64_t *offsets,
                            const uint32_t *caplen, const uint32_t *pkt_len,
                            const uint32_t *ifindex, uint64_t n, struct orc_event *events,
                            uint64_t max_events);

/* One event's perf sample (272-B slot: u32 raw size, event_hdr_st, min(len, 256) frame bytes, zero pad). */
uint32_t orc_perf_sample(const uint8_t *frame, uint32_t linear, const struct orc_event *e, uint8_t *out);

/* Debug lookup keys (24-B lpm_ip_key_st images) in packet order, duplicates included. */
uint64_t orc_collect_lookup_keys(const uint8_t *frames, const uint64_t *offsets, const uint32_t *caplen,
                                 const uint32_t *pkt_len, const uint32_t *ifindex, uint64_t n,
                                 uint8_t *keys_out, uint64_t n_max);

#ifdef __cplusplus
}
#endif
#endif
