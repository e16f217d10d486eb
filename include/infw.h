/*
 * infw.h — C ABI of the MI355X-native batched ingress-firewall classifier.
 *
 * This is the drop-in boundary for the hot path of pbmoses/ingress-node-firewall:
 * the XDP program bpf/ingress_node_firewall_kernel.c and the map-population API
 * of pkg/ebpf (cilium *ebpf.Map calls on ingress_node_firewall_table_map and
 * ingress_node_firewall_statistics_map).  A cgo build of pkg/ebpf binds these
 * symbols; every entry point below names the reference
 * interface it replaces.
 *
 * Conventions (mirroring bpf(2), which is what the reference's Go code sees):
 *   - return 0 on success or a negative errno (-EINVAL, -ENOENT, -EEXIST,
 *     -ENOSPC, -ENOMEM, -ENODEV, -EIO);
 *   - opaque handle, caller-owned buffers, no callbacks;
 *   - threads: control-plane calls (infw_table_*, infw_table_commit,
 *     infw_table_import/export, infw_stats_reset, infw_set_option,
 *     infw_set_launch, infw_debug_lookup_set, infw_debug_keys_clear) are
 *     externally serialised, like ebpfsyncer.go:62,72-73 (e.mu).  The data
 *     path and the readers — infw_classify*, infw_pack_frames*,
 *     infw_events_capture, infw_stats_read*, infw_table_info,
 *     infw_debug_walk, infw_debug_keys_read, infw_classify_variant — may run
 *     on any number of other threads concurrently with them and with each
 *     other; each batch observes exactly one committed table epoch;
 *   - the library reads no environment variable: everything that selects a
 *     table form or a kernel is a per-context option (infw_set_option), and
 *     no option changes a result word, a verdict or a counter.
 *
 * No torch types, no HIP types: device buffers and streams are plain pointers.
 */
#ifndef INFW_H
#define INFW_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* Constants — bpf/ingress_node_firewall.h:4-23                              */
/* ------------------------------------------------------------------------ */
#define INFW_MAX_TARGETS 1024          /* ingress_node_firewall.h:13 (stats map size)   */
#define INFW_MAX_RULES_PER_TARGET 100  /* ingress_node_firewall.h:14                    */
#define INFW_MAX_EVENT_DATA 256        /* ingress_node_firewall.h:15                    */
#define INFW_INVALID_RULE_ID 0         /* ingress_node_firewall.h:16                    */
#define INFW_XDP_ABORTED 0             /* UNDEF, ingress_node_firewall.h:10             */
#define INFW_XDP_DROP 1                /* DENY,  ingress_node_firewall.h:11             */
#define INFW_XDP_PASS 2                /* ALLOW, ingress_node_firewall.h:12             */
#define INFW_MAX_PREFIXLEN 160         /* 8 * sizeof(ifindex + ip_data): LPM data bits   */

/* BPF map update flags (uapi/linux/bpf.h), accepted by infw_table_update.   */
#define INFW_BPF_ANY 0
#define INFW_BPF_NOEXIST 1
#define INFW_BPF_EXIST 2

/* Result word: ingress_node_firewall.h:18-23 (SET_ACTIONRULE_RESPONSE).     */
#define INFW_RESULT(action, rule_id) \
    ((uint32_t)((((uint32_t)(rule_id)) & 0xFFFFFFu) << 8 | ((action) & 0xFFu)))
#define INFW_GET_ACTION(r) ((uint8_t)((r) & 0xFFu))
#define INFW_GET_RULE_ID(r) ((uint16_t)(((r) >> 8) & 0xFFFFFFu))

/* ------------------------------------------------------------------------ */
/* Struct ABI — byte-identical to bpf/ingress_node_firewall.h:45-91 and to   */
/* the bpf2go mirrors pkg/ebpf/bpf_bpfel.go:16-51 as marshalled by           */
/* cilium/ebpf sysenc (packed, little-endian).  Skipped if the reference     */
/* header was included first.                                                */
/* ------------------------------------------------------------------------ */
#ifndef __INGRESS_NODE_FIREWALL__
struct ruleStatistics_st {            /* ingress_node_firewall.h:45-54, 32 B */
    struct allow_stats_st {
        uint64_t packets;
        uint64_t bytes;
    } allow_stats;
    struct deny_stats_st {
        uint64_t packets;
        uint64_t bytes;
    } deny_stats;
};

struct event_hdr_st {                 /* ingress_node_firewall.h:58-64, 8 B  */
    uint16_t ifId;
    uint16_t ruleId;
    uint8_t action;
    uint8_t pad;
    uint16_t pktLength;
} __attribute__((packed));

struct ruleType_st {                  /* ingress_node_firewall.h:69-77, 12 B */
    uint32_t ruleId;
    uint8_t protocol;
    uint16_t dstPortStart;
    uint16_t dstPortEnd;
    uint8_t icmpType;
    uint8_t icmpCode;
    uint8_t action;
} __attribute__((packed));

struct lpm_ip_key_st {                /* ingress_node_firewall.h:83-87, 24 B */
    uint32_t prefixLen;
    uint32_t ingress_ifindex;
    uint8_t ip_data[16];
} __attribute__((packed));

struct rulesVal_st {                  /* ingress_node_firewall.h:89-91, 1200 B */
    struct ruleType_st rules[INFW_MAX_RULES_PER_TARGET];
} __attribute__((packed));
#endif /* __INGRESS_NODE_FIREWALL__ */

/* ------------------------------------------------------------------------ */
/* Packet batch: struct-of-arrays header tuples, 32 B per packet.            */
/* One tuple carries exactly the frame bytes kernel.c reads                  */
/* (ingress_node_firewall_main :412-457, ip_extract_l4info :95-174):         */
/*   saddr   16 B  frame[26..29] (IPv4, bytes 4..15 ignored) or frame[22..37] */
/*   ifindex  4 B  xdp_md.ingress_ifindex                                     */
/*   pkt_len  4 B  bpf_xdp_get_buff_len(ctx) (stats byte count)               */
/*   meta     4 B  bits 0..15 ethertype (frame[12]<<8|frame[13]),             */
/*                 bits 16..23 L3 next-proto (frame[23] v4 / frame[20] v6),   */
/*                 bits 24..31 min(linear length, 255) (truncation checks)    */
/*   l4word   4 B  frame[L4..L4+3] little-endian, L4 = 34 (v4) / 54 (v6),     */
/*                 bytes past the linear length read as 0                     */
/* All pointers are device pointers on the device the batch is classified on. */
/* saddr must be 16-byte aligned.                                             */
/* ------------------------------------------------------------------------ */
struct infw_batch_soa {
    const uint8_t *saddr;
    const uint32_t *ifindex;
    const uint32_t *pkt_len;
    const uint32_t *meta;
    const uint32_t *l4word;
};

#define INFW_META(ethertype, proto, caplen)                                    \
    ((uint32_t)((ethertype) & 0xFFFFu) | ((uint32_t)((proto) & 0xFFu) << 16) | \
     ((uint32_t)((caplen) > 255u ? 255u : (caplen)) << 24))

/* Raw frames in device memory (NIC -> HBM ingestion): frame i */
/* starts at frames + (offsets ? offsets[i] : i * stride); only its first     */
/* linear_len[i] bytes are read (xdp data .. data_end).                       */
struct infw_frame_batch {
    const uint8_t *frames;
    const uint64_t *offsets;      /* NULL: fixed-stride chunks (AF_XDP umem style)   */
    uint64_t stride;
    const uint32_t *linear_len;   /* data_end - data                                  */
    const uint32_t *pkt_len;      /* bpf_xdp_get_buff_len(); NULL: = linear_len       */
    const uint32_t *ifindex;
};
/* Writable SoA destination of infw_pack_frames (same layout as infw_batch_soa). */
struct infw_batch_soa_out {
    uint8_t *saddr;
    uint32_t *ifindex;
    uint32_t *pkt_len;
    uint32_t *meta;
    uint32_t *l4word;
};

/* Family-compact layout of the same bytes (infw_classify_c): the 12 address   */
/* bytes only IPv6 packets have are stored only for them.                     */
/*   saddr4   4 B per packet: frame[26..29] (IPv4) or frame[22..25] (IPv6)     */
/*   v6tail   per group g of INFW_V6_GROUP packets, a 12*INFW_V6_GROUP-byte   */
/*            block at g * 12 * INFW_V6_GROUP: frame[26..37] of the group's    */
/*            packets whose meta ethertype is 0x86DD, in packet order, packed */
/*            from the start of the block (4-byte aligned)                     */
/*   ifindex, pkt_len, meta, l4word as in infw_batch_soa                       */
/* A reader touches only the first 12 * (IPv6 packets of the group) bytes of  */
/* a block: 4 + 12 * (IPv6 share) address bytes per packet instead of 16.      */
#define INFW_V6_GROUP 64
struct infw_batch_soa_c {
    const uint32_t *saddr4;
    const uint8_t *v6tail;
    const uint32_t *ifindex;
    const uint32_t *pkt_len;
    const uint32_t *meta;
    const uint32_t *l4word;
};

/* Writable family-compact destination of infw_pack_frames_c.                */
struct infw_batch_soa_c_out {
    uint32_t *saddr4;
    uint8_t *v6tail;
    uint32_t *ifindex;
    uint32_t *pkt_len;
    uint32_t *meta;
    uint32_t *l4word;
};

typedef struct infw_ctx infw_ctx;

/* ------------------------------------------------------------------------ */
/* Lifecycle — replaces NewIngNodeFwController (loader.go:56-112) and Close */
/* (loader.go:306-333) for the table + statistics maps.                      */
/* ------------------------------------------------------------------------ */
/* hip_devices: HIP device ordinals the context replicates its tables onto;   */
/* NULL/n_dev=0 means {current device}.  max_entries: LPM capacity (the       */
/* reference's MAX_TARGETS=1024 at kernel.c:54; 0 selects 1<<22).            */
/* Without INFW_F_HOST_ONLY, -ENODEV when no HIP device is visible: there is   */
/* no CPU classification path.                                                */
#define INFW_F_HOST_ONLY 0x1u   /* control plane only: map API + compile, no    */
                                /* device tables; infw_classify -> -ENODEV     */
#define INFW_F_KEEP_HOST_IMAGE 0x2u /* accepted for compatibility: the host    */
                                    /* image is always kept (incremental       */
                                    /* commits patch it; infw_debug_walk reads) */
#define INFW_F_FULL_COMMIT 0x4u     /* every commit recompiles the whole epoch  */
int infw_create(infw_ctx **out, const int *hip_devices, int n_dev,
                uint32_t max_entries, uint32_t flags);
void infw_destroy(infw_ctx *ctx);
int infw_num_devices(const infw_ctx *ctx);

/* ------------------------------------------------------------------------ */
/* Table map — ingress_node_firewall_table_map (kernel.c:50-57, LPM_TRIE     */
/* key 24 B / value 1200 B).  Calls edit the PENDING set with the kernel's   */
/* LPM-trie map semantics; infw_table_commit publishes it to the GPUs.       */
/* ------------------------------------------------------------------------ */
/* Map.Update(key, val, flags)   loader.go:203  (addOrUpdateRules)           */
/*   -EINVAL prefixLen>160, flags>BPF_EXIST; -EEXIST / -ENOENT per NOEXIST  */
/*           / EXIST.  prefixLen<32 (a partial ifindex, never produced by     */
/*           BuildEBPFKey, loader.go:543) is accepted like lpm_trie does: it  */
/*           covers every ifindex whose key bytes start with its bits, below  */
/*           the interface's own entries (commits with one are full compiles) */
/*   -ENOSPC when a new key would exceed max_entries.                        */
int infw_table_update(infw_ctx *ctx, const struct lpm_ip_key_st *key,
                      const struct rulesVal_st *val, uint64_t flags);
/* Batch form (BPF_MAP_UPDATE_BATCH): val_index==NULL -> keys[i]:vals[i],     */
/* else keys[i]:vals[val_index[i]].  Stops at the first error; *done (may be  */
/* NULL) receives the number of keys applied.                                 */
int infw_table_update_batch(infw_ctx *ctx, const struct lpm_ip_key_st *keys,
                            const struct rulesVal_st *vals, const uint32_t *val_index,
                            uint64_t n, uint64_t flags, uint64_t *done);
/* Map.Delete(key)               loader.go:640  (purgeKeys): exact prefix.    */
int infw_table_delete(infw_ctx *ctx, const struct lpm_ip_key_st *key);
/* Batch form (BPF_MAP_DELETE_BATCH): stops at the first error (-ENOENT for a */
/* key not in the map); *done (may be NULL) receives the keys deleted.         */
int infw_table_delete_batch(infw_ctx *ctx, const struct lpm_ip_key_st *keys, uint64_t n, uint64_t *done);
/* Map.Iterate() key walk        loader.go:293,558 (getStaleKeys,            */
/* GetBPFMapContentForTest): key==NULL or absent -> first key; -ENOENT at end. */
/* Order is the LPM trie's post-order (children before parents, 0-bit first). */
int infw_table_get_next_key(infw_ctx *ctx, const struct lpm_ip_key_st *key,
                            struct lpm_ip_key_st *next);
/* Map.Lookup(key, &val): longest-prefix match over entries with              */
/* prefixLen <= key->prefixLen (BPF LPM trie lookup semantics).               */
int infw_table_lookup(infw_ctx *ctx, const struct lpm_ip_key_st *key,
                      struct rulesVal_st *val);
int infw_table_count(infw_ctx *ctx, uint64_t *n_entries);
/* End of IngressNodeFwRulesLoader (loader.go:189-193): publish the pending   */
/* set as the next epoch; in-flight batches finish on the old one.            */
/* Incremental by default: only the keys edited since the   */
/* last commit are turned into table bytes (DIR-24-8 words / tbl8 groups,     */
/* IPv6 buckets, appended rule lists), copied into the device's spare image,  */
/* which then becomes live — each device keeps two images, so a batch always  */
/* reads exactly one epoch.  Layout changes (new ifindex, overflowed IPv6     */
/* groups, > 1/4 of the keys edited, ...) fall back to a full compile;        */
/* infw_table_info reports which one ran and why.                             */
int infw_table_commit(infw_ctx *ctx);

/* ------------------------------------------------------------------------ */
/* Data path — replaces the per-frame XDP entry ingress_node_firewall_process */
/* (kernel.c:459-462) with one batched launch.                                */
/*   result_words[i] = the `result` of ingress_node_firewall_main (:418-442): */
/*                     (ruleId & 0xFFFFFF) << 8 | action, 0 = UNDEF;          */
/*   xdp_verdicts[i] = XDP return code (1 DROP / 2 PASS);                     */
/*   statistics      = per-rule allow/deny packets+bytes added on the device  */
/*                     (kernel.c:361-390), one slot per device.               */
/* Either output may be NULL.  stream: hipStream_t (NULL = default stream).   */
/* The call is asynchronous with respect to the host.                         */
/* ------------------------------------------------------------------------ */
int infw_classify(infw_ctx *ctx, int dev, const struct infw_batch_soa *in, uint64_t n,
                  uint32_t *result_words, uint8_t *xdp_verdicts, void *stream);
/* infw_classify over the family-compact layout (identical results).          */
int infw_classify_c(infw_ctx *ctx, int dev, const struct infw_batch_soa_c *in, uint64_t n,
                    uint32_t *result_words, uint8_t *xdp_verdicts, void *stream);
/* Standard -> family-compact address layout on the device: saddr4 (n words) */
/* and v6tail (ceil(n / INFW_V6_GROUP) blocks); the other streams are shared.  */
int infw_soa_compact(infw_ctx *ctx, int dev, const struct infw_batch_soa *in, uint64_t n,
                     uint32_t *saddr4, uint8_t *v6tail, void *stream);

/* Launch shape of the classify kernel (default 768 / 0 / 2 = 24 waves per CU). */
/* scan_group 0 = first-match decision tables in one of the shapes           */
/* (block x blocks_per_cu) 768x2, 512x2, 512x3, 512x4, 256x6; scan_group      */
/* 1|4|8 = the one-lane-per-rule ballot scan (kernel.c:222-258 in rule order) */
/* with that many packets in flight, 512x3 or 256x6.  -EINVAL for any other   */
/* shape.  The family-compact layout runs non-default shapes as decision       */
/* tables 512x3; frames and sideband launches have fixed shapes.               */
int infw_set_launch(infw_ctx *ctx, int block, int scan_group, int blocks_per_cu);
/* The launch shape infw_classify uses (default or set above; bench reporting). */
int infw_get_launch(infw_ctx *ctx, int *block, int *scan_group, int *blocks_per_cu);

/* Per-context options.  Each selects among bit-exact forms of the same table */
/* epoch (full compiles read them), how the classify launch reads it, or      */
/* tracing — results, verdicts and counters never depend on them.  value -1   */
/* means "chosen per epoch" where an option has that.  -EINVAL for an unknown */
/* name or a value out of range (nothing changes then).                       */
/*   short_table      -1 auto (DIR-24-8 while ifindexes x 128 MiB <= 4 GiB),   */
/*                    0 DIR-24-8, 1 compressed 16-8-8 (next full compile)      */
/*   d16              -1 auto, 0 off, 1 on: /16 words in front of DIR-24-8      */
/*   dt_half          -1 auto, 0 off, 1 on: half-first decision-line reads      */
/*   dt_parts         0 auto, or 1|2|4|8|16 value parts per (list, class)        */
/*   dt_adapt         1 per-list part counts (<= 4096 lists), 0 uniform parts    */
/*   dt_budget_mb     64..1048576 (2048): entry lines of one image at most        */
/*   compile_threads  0 hardware threads (<= 16), or 1..16                        */
/*   split            -1 auto, 0 off, 1 on: two-phase classify (many lists)       */
/*   split_min_mb     0..1048576 (1024): auto splits past this many MiB of lines  */
/*   stat_flush_tiles 1..1024 (1024): LDS counter flush period in tiles           */
/*   trace            bit mask to stderr: 1 compile, 2 incremental patch,          */
/*                    4 commit timing, 8 infw_classify_xdp_host pipeline timing    */
/*   host_threads     0 the CPUs the process may run on (affinity mask, cgroup     */
/*                    CPU quota; <= 16), or 1..64: infw_classify_xdp_host packers  */
int infw_set_option(infw_ctx *ctx, const char *name, int64_t value);
int infw_get_option(infw_ctx *ctx, const char *name, int64_t *value);
/* Name of option i (0-based), NULL past the last.                             */
const char *infw_option_name(int i);

/* Which kernel instantiation(s) a launch would run (introspection; nothing is */
/* launched, no device needed — host-only contexts answer from their image).  */
/* input: INFW_INPUT_* (XDP: infw_classify_xdp); flags: INFW_VARIANT_EVENTS   */
/* for an infw_classify_ex event stream (not with COMPACT or XDP); the debug   */
/* sideband follows infw_debug_lookup_set.  name is a registry name           */
/* (infw_kernel_variant_name); two-phase launches name both kernels joined by */
/* '+'.  -ERANGE when cap is too small.                                        */
#define INFW_INPUT_SOA 0
#define INFW_INPUT_COMPACT 1
#define INFW_INPUT_FRAMES 2
#define INFW_INPUT_XDP 3
#define INFW_VARIANT_EVENTS 0x1u
int infw_classify_variant(infw_ctx *ctx, int dev, int input, uint32_t flags, char *name, size_t cap);
/* Registry of every kernel instantiation the library launches: name of entry */
/* i (0-based), NULL past the last.                                            */
const char *infw_kernel_variant_name(int i);
/* Launch counters of device slot `dev` since infw_create: counts[0] two-phase */
/* launches (phase 1 + decide), counts[1] launches the selector made two-phase */
/* that ran the fused kernel because the scratch could not be allocated (no    */
/* pool, or the pool out of memory) — results are the same either way.        */
int infw_launch_counts(infw_ctx *ctx, int dev, uint64_t counts[2]);

/* Frame headers -> SoA tuples on the device (the packer of the batch format  */
/* above, run as a kernel over frames already in HBM).  Asynchronous.          */
int infw_pack_frames(infw_ctx *ctx, int dev, const struct infw_frame_batch *frames, uint64_t n,
                     const struct infw_batch_soa_out *out, void *stream);
/* infw_pack_frames into the family-compact layout (the production feed of     */
/* infw_classify_c): v6tail blocks of groups with fewer IPv6 packets are only  */
/* written up to their last tail.                                             */
int infw_pack_frames_c(infw_ctx *ctx, int dev, const struct infw_frame_batch *frames, uint64_t n,
                       const struct infw_batch_soa_c_out *out, void *stream);

/* infw_classify straight from the frames (no SoA batch written or read: the  */
/* kernel builds infw_pack_header()'s tuple from each frame's bytes [10, 58)  */
/* in LDS — the XDP program's own input, kernel.c:412-462 per frame).          */
/* Identical results and counters to infw_pack_frames + infw_classify.        */
/* Reads are whole 16-byte aligned blocks that hold a byte of                  */
/* [frame + 10, frame + min(linear_len, 58)): no block outside a frame's own   */
/* bytes' blocks is touched (the packer's rule, infw_pack_frames).             */
int infw_classify_frames(infw_ctx *ctx, int dev, const struct infw_frame_batch *frames, uint64_t n,
                         uint32_t *result_words, uint8_t *xdp_verdicts, void *stream);

/* An AF_XDP socket's RX ring as the feed (the NIC side of   */
/* the frames path): descriptors as the kernel writes them into the ring      */
/* (linux/if_xdp.h struct xdp_desc), frames in the socket's umem.  Frame i's  */
/* bytes start at umem + (addr & (2^48 - 1)) + (addr >> 48) — aligned mode,    */
/* and unaligned mode's offset in bits 48..63 (XSK_UNALIGNED_BUF_OFFSET_SHIFT) */
/* — and len is both its linear length (xdp data .. data_end) and             */
/* bpf_xdp_get_buff_len(): single-buffer frames (a multi-buffer frame's first */
/* descriptor is classified on its own bytes and length).  One ring belongs  */
/* to one interface queue, so every frame carries `ifindex`.  umem and descs  */
/* must be device-accessible: HBM, or pinned host memory (hipHostMalloc), which */
/* the kernel reads in place over PCIe — one 64-B header window and one 16-B  */
/* descriptor per frame.  descs 16-byte aligned.  Identical results and       */
/* counters to infw_classify_frames over the same frames.  Asynchronous.      */
struct infw_xdp_desc {
    uint64_t addr;
    uint32_t len;
    uint32_t options;
};
/* umem and descs are checked with hipPointerGetAttributes: -EFAULT when either */
/* is ordinary (pageable, unregistered) host memory, which the GPU cannot read  */
/* — register such a mapping with infw_host_register first, or use            */
/* infw_classify_xdp_host, which reads it on the CPU.                          */
int infw_classify_xdp(infw_ctx *ctx, int dev, const uint8_t *umem, const struct infw_xdp_desc *descs, uint64_t n,
                      uint32_t ifindex, uint32_t *result_words, uint8_t *xdp_verdicts, void *stream);

/* AF_XDP RX rings over a HOST umem, read by the CPU (the host-fed path): the */
/* context's packer threads (option host_threads) read each frame's header    */
/* window where the NIC left it and write the family-compact tuple            */
/* (infw_batch_soa_c, without the ifindex stream: one ring = one interface)    */
/* into pinned slots, which go to the device in bulk copies — ~28 B per packet */
/* over PCIe instead of one 64-B read request per frame.  Pipelined per chunk  */
/* of `chunk` descriptors (0 = 512K; rounded up to 512): packing of chunk k+1  */
/* || H2D of k || classify of k-1 || D2H of k-2, chunks running on from one    */
/* ring into the next.  umem and descs may be any memory the process can read  */
/* (the socket's mmapped RX ring and umem as they are); results / verdicts are */
/* host memory (pinned or infw_host_register'ed for the full rate), per ring   */
/* in descriptor order, either may be NULL.  Frames are read exactly as        */
/* infw_classify_xdp reads them (same result words, verdicts and counters).    */
/* Synchronous; the whole call reads one table epoch.  One call at a time per  */
/* device (concurrent calls queue).                                            */
struct infw_xdp_ring {
    const uint8_t *umem;                 /* frame i at umem + (addr & (2^48-1)) + (addr >> 48) */
    const struct infw_xdp_desc *descs;   /* n RX descriptors                                    */
    uint64_t n;
    uint32_t ifindex;                    /* the interface the socket is bound to                 */
    uint32_t flags;                      /* 0                                                    */
    uint32_t *results;                   /* n result words, or NULL                              */
    uint8_t *verdicts;                   /* n XDP verdicts, or NULL                              */
};
int infw_classify_xdp_host(infw_ctx *ctx, int dev, const struct infw_xdp_ring *rings, uint32_t n_rings,
                           uint64_t chunk);
/* The host packer of infw_classify_xdp_host alone, on the calling thread: one */
/* ring's frames -> the family-compact streams in host memory (the layout       */
/* infw_classify_c reads; out->ifindex may be NULL, else it is filled with      */
/* `ifindex`), for a caller that moves the tuples itself.  Pure host function:  */
/* no context or device.  Every stream 4-byte aligned.                          */
int infw_pack_xdp_host(const uint8_t *umem, const struct infw_xdp_desc *descs, uint64_t n, uint32_t ifindex,
                       const struct infw_batch_soa_c_out *out);

/* ------------------------------------------------------------------------ */
/* Sidebands of the data path, opt-in per batch (infw_classify_ex).          */
/*  - Deny events (kernel.c:392-399, ingress_node_firewall_events_map): one  */
/*    record per DROP-by-rule packet: the 8-B event_hdr_st the program       */
/*    emits plus where the min(len, 256) packet bytes of the perf record     */
/*    live (the batch index).  Records are appended with one atomic per      */
/*    wave; order across waves is unspecified, like perf records across      */
/*    CPUs; *events_count counts every event, also those beyond events_cap   */
/*    (perf "lost samples").                                                  */
/* ------------------------------------------------------------------------ */
struct infw_event_rec {
    struct event_hdr_st hdr;      /* ifId, ruleId, action (1), pad, pktLength (u16 truncations) */
    uint32_t captured;            /* min(pkt_len, INFW_MAX_EVENT_DATA)                          */
    uint32_t reserved;
    uint64_t pkt_index;           /* batch index of the packet the record belongs to             */
};

struct infw_classify_ex {
    uint32_t size;                /* sizeof(struct infw_classify_ex)                              */
    uint32_t flags;               /* reserved, 0                                                 */
    struct infw_event_rec *events;   /* device buffer, or NULL: no event stream                  */
    uint64_t events_cap;
    uint64_t *events_count;       /* device u64, incremented by the kernel                       */
};

int infw_classify_ex(infw_ctx *ctx, int dev, const struct infw_batch_soa *in, uint64_t n,
                     uint32_t *result_words, uint8_t *xdp_verdicts,
                     const struct infw_classify_ex *ex, void *stream);
/* infw_classify_frames with the sidebands: the event records' pkt_index is   */
/* the frame's index in the batch, so infw_events_capture over the same       */
/* frames writes the perf samples.                                            */
int infw_classify_frames_ex(infw_ctx *ctx, int dev, const struct infw_frame_batch *frames, uint64_t n,
                            uint32_t *result_words, uint8_t *xdp_verdicts,
                            const struct infw_classify_ex *ex, void *stream);

/*  - Deny-event payload: the perf sample each record stands for, as the      */
/*    reader receives it (kernel.c:392-399: bpf_perf_event_output(ctx, map,   */
/*    BPF_F_CURRENT_CPU | min(len, 256) << 32, &hdr, 8); events.go:77-96       */
/*    reads perf.Record.RawSample).  Slot k of `samples` belongs to record k    */
/*    of the event ring: `size` is perf's raw-size field,                       */
/*    round_up(8 + captured + 4, 8) - 4, and raw[0 .. size) is event_hdr_st,    */
/*    then the frame's first `captured` bytes, then perf's alignment pad        */
/*    (written as zeros; the kernel leaves stale ring bytes there).  Frame     */
/*    bytes past the frame's linear length (XDP multi-buffer frags, which HBM  */
/*    frames do not carry) are written as zeros.  Bytes past `size` are zero.  */
#define INFW_EVENT_SAMPLE_BYTES 272   /* 4 + round_up(8 + 256 + 4, 8) - 4       */
struct infw_event_sample {
    uint32_t size;
    uint8_t raw[INFW_EVENT_SAMPLE_BYTES - 4];
};
/* Fill samples[k] for k < min(*events_count, events_cap) — the records       */
/* infw_classify_ex wrote — from the n_frames frames the batch was packed     */
/* from (record.pkt_index = frame index; a record whose index is >= n_frames  */
/* gets its header and no frame bytes).  Stream-ordered after the classify: the */
/* count is read on the device, no host synchronisation.  samples: device     */
/* memory of events_cap slots.                                                 */
int infw_events_capture(infw_ctx *ctx, int dev, const struct infw_frame_batch *frames, uint64_t n_frames,
                        const struct infw_event_rec *events, uint64_t events_cap,
                        const uint64_t *events_count, struct infw_event_sample *samples, void *stream);

/* Host-resident batch: the SoA streams, result words and verdicts live in   */
/* host memory (as a cgo caller hands them over).  The batch goes through    */
/* the device in chunks of `chunk` packets (0 = 4M) with three HIP streams:  */
/* the H2D copy of chunk k+1 and the D2H copy of chunk k-1 overlap the       */
/* kernel on chunk k; two sets of chunk buffers per device are owned by the  */
/* context.  The whole batch reads one table epoch.  Synchronous: returns    */
/* when every result is in host memory.  Full PCIe rate needs pinned or      */
/* registered host memory (hipHostMalloc / infw_host_register); pageable     */
/* memory is correct but staged by the HIP runtime.  Statistics accumulate   */
/* in the device's slot exactly as for infw_classify.                         */
int infw_classify_host(infw_ctx *ctx, int dev, const struct infw_batch_soa *host_in, uint64_t n,
                       uint32_t *host_results, uint8_t *host_verdicts, uint64_t chunk);
/* Page-lock (hipHostRegister) / release a host range for infw_classify_host. */
int infw_host_register(infw_ctx *ctx, void *ptr, uint64_t bytes);
int infw_host_unregister(infw_ctx *ctx, void *ptr);

/* ------------------------------------------------------------------------ */
/* Statistics — ingress_node_firewall_statistics_map (kernel.c:36-41,        */
/* PERCPU_ARRAY[1024] of ruleStatistics_st).  One slot per device plays the  */
/* role of one per-CPU slot; readers sum slots like statistics.go:126-157.   */
/*                                                                          */
/* Where the multi-GPU sum happens — the library never runs a collective:   */
/*  - one process, one context over N devices (the node daemon's shape):    */
/*    each device slot counts its own batches; infw_stats_read returns the  */
/*    N per-slot values (the []BpfRuleStatisticsSt of one per-CPU lookup)   */
/*    and the caller sums them, as statistics.go:132-156 does;              */
/*    infw_stats_read_all returns that sum (u64 wrap-around) for all rules; */
/*  - one process per GPU (torch.distributed / RCCL ranks): each rank's     */
/*    context has one slot; a caller that wants node totals binds the slot  */
/*    to its own device buffer (infw_stats_bind) and all-reduces it with    */
/*    its communicator (bench.py: an async RCCL all-reduce), or reads each  */
/*    rank's slot and sums on the host — the per-CPU sum again.             */
/* Reads are snapshots: a lookup copies the slot on a stream of its own and  */
/* waits for nothing queued on other streams (batches in flight keep adding,*/
/* like XDP on other CPUs while statistics.go polls).                       */
/* ------------------------------------------------------------------------ */
/* Map.Lookup(uint32(rule), &[]BpfRuleStatisticsSt)  statistics.go:127       */
/* per_slot must hold infw_num_devices() entries; -ENOENT for rule >= 1024.   */
int infw_stats_read(infw_ctx *ctx, uint32_t rule_id, struct ruleStatistics_st *per_slot,
                    int *n_slots);
/* All 1024 rules summed over slots (u64 wrap-around like the kernel).        */
int infw_stats_read_all(infw_ctx *ctx, struct ruleStatistics_st out[INFW_MAX_TARGETS]);
int infw_stats_reset(infw_ctx *ctx);
/* Redirect device `dev`'s statistics slot to caller-owned device memory of   */
/* 1024*32 B (e.g. a tensor that an RCCL all-reduce then sums across GPUs).   */
/* NULL restores the context-owned slot.  Contents are not copied.            */
int infw_stats_bind(infw_ctx *ctx, int dev, uint64_t *device_stats);
/* Device pointer of device `dev`'s current statistics slot.                  */
int infw_stats_device_ptr(infw_ctx *ctx, int dev, uint64_t **device_stats);

/* ------------------------------------------------------------------------ */
/* Debug lookup capture — ingress_node_firewall_dbg_map (kernel.c:59-64,     */
/* HASH of lpm_ip_key_st -> lpm_ip_key_st, 16384 entries) filled with        */
/* bpf_map_update_elem(key, key, BPF_NOEXIST) for every lookup key while the */
/* load-time constant debug_lookup != 0 (kernel.c:78, :214-216, :297-299;    */
/* loader.go:72-83 sets it from ENABLE_EBPF_LPM_LOOKUP_DBG).                 */
/* Key inserted: packets whose L4 header was extracted (not UNDEF), before   */
/* the LPM: {prefixLen 64, ifindex, saddr, 12 zero bytes} for IPv4,          */
/* {160, ifindex, saddr[16]} for IPv6.  Existing keys are left alone; once   */
/* INFW_DBG_MAX_ENTRIES distinct keys are held, new keys are dropped.        */
/* One set per device (like one map per node); reads return their union,    */
/* capped at INFW_DBG_MAX_ENTRIES.  Keys are deduplicated on the device by a */
/* 64-bit fingerprint of the 24-B key.  Which keys fill the last places when */
/* more arrive at once is decided by the device's atomic order (the          */
/* reference's by the CPUs' order).                                          */
/* ------------------------------------------------------------------------ */
#define INFW_DBG_MAX_ENTRIES 16384
/* debug_lookup rewrite at load (loader.go:72-83).  Non-zero allocates the   */
/* per-device key sets on first use; 0 stops capturing (keys are kept).      */
int infw_debug_lookup_set(infw_ctx *ctx, uint32_t debug_lookup);
/* Map iteration of the dbg map: copies up to cap keys, *n = keys held.       */
/* Waits for work queued on the devices.                                      */
int infw_debug_keys_read(infw_ctx *ctx, struct lpm_ip_key_st *keys, uint32_t cap, uint32_t *n);
/* Delete every key of the dbg map (all devices).                             */
int infw_debug_keys_clear(infw_ctx *ctx);

/* ------------------------------------------------------------------------ */
/* Control-plane encoders — the Go helpers whose byte output is the contract */
/* of the table map.  Pure host functions (no device needed).                */
/* ------------------------------------------------------------------------ */
/* BuildEBPFKey(ifID, cidr)  loader.go:530-547.  -EINVAL on a bad CIDR.      */
int infw_build_ebpf_key(uint32_t if_id, const char *cidr, struct lpm_ip_key_st *key);
/* One IngressNodeFirewallProtocolRule -> rulesVal_st slot [order]            */
/* (makeIngressFwRulesMap loader.go:435-515, utils.go:13-60).                 */
/*   protocol: "TCP","UDP","SCTP","ICMP","ICMPv6" or "" (no protocolConfig)   */
/*   ports:    "N" or "A-B" (TCP/UDP/SCTP), NULL/"" otherwise                 */
/*   action:   "Allow" or "Deny"                                              */
/* -EINVAL for the cases the Go code rejects; -E2BIG for order >= 100 (the Go */
/* code panics on an out-of-range array index there, loader.go:437).          */
int infw_make_rule(struct rulesVal_st *val, uint32_t order, const char *protocol,
                   const char *ports, uint8_t icmp_type, uint8_t icmp_code,
                   const char *action);

/* ------------------------------------------------------------------------ */
/* Introspection for tests and the bench.                                     */
/* ------------------------------------------------------------------------ */
struct infw_table_info {
    uint64_t epoch;            /* number of successful commits                */
    uint64_t n_entries;        /* committed LPM entries                       */
    uint32_t n_if_slots;       /* distinct ingress ifindexes                  */
    uint32_t n_lists;          /* interned rule lists                         */
    uint64_t n_rules;          /* GPU rule records over all lists/classes     */
    uint64_t n_tbl8_groups;    /* DIR-24-8 second-level groups                */
    uint32_t n_long_levels;    /* distinct IPv6 prefix lengths > /32          */
    uint64_t n_long_entries;   /* long-prefix hash entries incl. markers      */
    uint64_t device_bytes;     /* table bytes resident per device             */
    double compile_ms;         /* host compile time of the last commit        */
    double upload_ms;          /* H2D time of the last commit                 */
    uint64_t n_v6_groups;      /* (ifindex, /32) groups of IPv6 long prefixes */
    uint64_t n_v6_overflow;    /* groups in the Waldvogel table (> 3 long      */
                               /* prefixes; > 2 in the two-choice slot form)  */
    uint32_t commit_mode;      /* INFW_COMMIT_*: how the last commit ran      */
    uint32_t dt_parts;         /* value parts per (list, class) decision table */
    uint64_t patch_bytes;      /* bytes copied to the devices by it           */
    uint64_t dead_lists;       /* compiled lists no entry references (GC'd by */
                               /* the next full compile)                      */
    char full_reason[48];      /* why the last full compile was needed        */
    uint64_t reserved0;        /* zero (ABI 3: the removed two-choice IPv6     */
                               /* slot form)                                   */
    uint32_t short_mode;       /* <= /32 key space: 0 DIR-24-8, 1 compressed   */
                               /* 16-8-8, 2 none                               */
    uint32_t reserved1;        /* zero (ABI 3: the removed range form)         */
    /* ABI 3: commit timing per device slot (the slots upload / patch in        */
    /* parallel, one host thread each) and room to grow without another break.  */
    double device_ms_max;      /* slowest slot's upload / patch of the last     */
                               /* commit (wall, host thread of that slot)      */
    uint32_t n_device_slots;   /* slots the last commit published to            */
    uint32_t imported;         /* 1: the epoch came from infw_table_import      */
    uint32_t d16;              /* 1: /16 words in front of DIR-24-8 (sparse     */
                               /* short tables; chosen per full compile)       */
    uint32_t d16_permille;     /* of the /16s holding a prefix longer than /16, */
                               /* those a /16 word answers alone               */
    uint32_t split;            /* 1: the epoch classifies in two phases (LPM   */
                               /* -> decision-line address per packet, then   */
                               /* the decision lines as independent gathers):  */
                               /* many distinct rule lists (option split)      */
    uint32_t dt_half_reads;    /* 1: decision lines read half-first (nearly all */
                               /* compact leaves of <= 9 segments; dt_half)    */
    uint64_t reserved[12];     /* zero; future fields come out of this         */
};
#define INFW_COMMIT_FULL 0u        /* compile + upload of a fresh image           */
#define INFW_COMMIT_INCREMENTAL 1u /* patched ranges copied into the spare image  */
#define INFW_COMMIT_REUPLOAD 2u    /* patched host image, re-uploaded (grew)     */
int infw_table_info(infw_ctx *ctx, struct infw_table_info *info);
/* Verification hook for tests/ only — never called by infw_classify: walks     */
/* the last committed HOST table image (INFW_F_HOST_ONLY or                      */
/* INFW_F_KEEP_HOST_IMAGE contexts) with the same lookup code the kernel runs,   */
/* so the table compiler can be checked against the oracle on a CPU-only box.   */
/* tuples: n x 8 u32 {saddr[4], ifindex, pkt_len, meta, l4word}.                */
/* out: result words (same meaning as infw_classify's).  -ENODATA w/o image.    */
int infw_debug_walk(infw_ctx *ctx, const uint32_t *tuples, uint64_t n, uint32_t *out);
/* Last error string of this thread (static storage).                          */
const char *infw_last_error(void);
/* ABI version (bumped on incompatible change).  3: struct infw_table_info     */
/* grew (and now ends in reserved space), infw_build_id, table export/import. */
/* 4: per-context options replace environment variables, infw_set_launch      */
/* accepts only the registered shapes, kernel-variant introspection.          */
#define INFW_ABI_VERSION 4
int infw_abi_version(void);
/* Identity of the code this library was built from: a hash of the kernel and */
/* table-layout sources and the flags they were compiled with (Makefile).       */
/* Profiles taken on one build are only valid for the same build id.           */
const char *infw_build_id(void);

/* ------------------------------------------------------------------------ */
/* Compiled-epoch images: compile once, install on many contexts.  The        */
/* reference has one daemon per node driving one map (ebpfsyncer.go:70-125);  */
/* here one process per GPU each holds a context, and instead of every rank    */
/* compiling the same 1M-entry set, one exports its committed epoch (the      */
/* entry set, the compiled host tables and the incremental-commit state) and  */
/* the others import it.                                                       */
/* ------------------------------------------------------------------------ */
/* Serialise the last committed epoch.  buf == NULL: *size = bytes needed.     */
/* -EBUSY when the pending set has uncommitted edits, -ENOSPC when cap is too  */
/* small (*size says how much is needed).                                      */
int infw_table_export(infw_ctx *ctx, void *buf, uint64_t cap, uint64_t *size);
/* Install an exported epoch into a context whose map is empty: the entries    */
/* become the committed set (get_next_key / lookup / later incremental commits */
/* work as after a commit) and every device slot gets the image — no compile.  */
/* -EBUSY: the context holds entries or uncommitted edits (one whose entries   */
/* were all removed and committed counts as empty); -EINVAL: not an image of  */
/* this library build (infw_build_id), truncated, a payload that does not     */
/* match the header's XXH64, or compiled tables that fail the structural      */
/* checks (an index outside its buffer, a probe table without a free slot) —  */
/* nothing is installed or uploaded then; -ENOSPC: more entries than          */
/* max_entries.                                                               */
int infw_table_import(infw_ctx *ctx, const void *buf, uint64_t size);

#ifdef __cplusplus
}
#endif
#endif /* INFW_H */
