/*
 * xdp_demo.c — the AF_XDP side of the boundary driven from plain C, the way a node daemon would
 * (INTEGRATION.md §1.1.2): the umem is the daemon's own memory (posix_memalign, as it would hand it to
 * XDP_UMEM_REG), page-locked for the GPU with infw_host_register; the RX ring's descriptors name frames in it;
 * infw_classify_xdp reads the frames and the descriptors in place over PCIe and writes the result words and verdicts
 * into the daemon's (registered) host arrays.  One ring per interface queue: the frames of ifindex 7 and of ifindex
 * 8 are two calls.  Then the same frames through the host-fed path, infw_classify_xdp_host, with the memory as the
 * daemon allocated it (pageable, unregistered — the form a socket's mmapped ring has): both rings in one call.  Before
 * any registration, infw_classify_xdp must refuse that memory with -EFAULT rather than let the GPU fault on it.
 * Last, the same packets as a DPDK poll loop hands them over (infw_classify_bursts_host): every frame in a buffer of
 * its own (an mbuf's data room), one pointer, data_len and pkt_len per frame — one frame split over two segments —
 * one burst per port, the bursts' result words slices of one array; and the burst's deny events.
 *
 *   the XDP entry per frame (kernel.c:459-462, ethertype / L4 extraction :95-174, :412-440)
 *   statsMap.Lookup (statistics.go:127):  infw_stats_read
 *
 * Built by tests/test_c_abi.py (gcc against include/infw.h and the HIP runtime's header for the stream sync).
 * `xdp_demo host` runs without a GPU: an INFW_F_HOST_ONLY context, whose infw_classify_xdp must refuse (-ENODEV).
 * Prints "xdp_demo OK ..." and exits 0 when every verdict and counter is the expected one.
 */
#define _POSIX_C_SOURCE 200112L /* posix_memalign */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "infw.h"
#include "infw_host.h"

#define CHECK(call)                                                                                 \
    do {                                                                                            \
        int rc_ = (call);                                                                           \
        if (rc_ < 0) {                                                                              \
            fprintf(stderr, "%s failed: %d (%s)\n", #call, rc_, infw_last_error());                 \
            return 1;                                                                               \
        }                                                                                           \
    } while (0)

enum { CHUNK = 2048, HEADROOM = 256, N = 6, CHUNKS = 16 };

/* An Ethernet + IPv4 + TCP/UDP frame of `len` bytes at f: the bytes kernel.c reads (ethertype, protocol, saddr,
 * destination port at L4 offset 34). */
static void put_frame(uint8_t *f, const uint8_t ip[4], uint8_t proto, uint16_t dport, uint32_t len) {
    memset(f, 0, len);
    f[12] = 0x08, f[13] = 0x00;     /* ETH_P_IP */
    f[14] = 0x45;                   /* version 4, IHL 5 */
    f[16] = (uint8_t)((len - 14) >> 8), f[17] = (uint8_t)(len - 14);
    f[22] = 64, f[23] = proto;      /* ttl, protocol */
    memcpy(f + 26, ip, 4);          /* saddr */
    f[30] = 198, f[31] = 51, f[32] = 100, f[33] = 1;
    f[34] = 40000 >> 8, f[35] = 40000 & 0xFF;  /* source port */
    f[36] = dport >> 8, f[37] = dport & 0xFF;  /* destination port */
}

int main(int argc, char **argv) {
    const int host_only = argc > 1 && strcmp(argv[1], "host") == 0;
    infw_ctx *ctx = NULL;
    CHECK(infw_create(&ctx, NULL, 0, 1024, host_only ? INFW_F_HOST_ONLY : 0));

    /* eth0 (ifindex 7): 10.0.0.0/8 -> [order 1: TCP 80 Deny, order 2: TCP 1-1024 Allow]; 192.0.2.0/24 -> UDP 53 Allow */
    struct lpm_ip_key_st key;
    struct rulesVal_st val;
    memset(&val, 0, sizeof(val));
    CHECK(infw_build_ebpf_key(7, "10.0.0.0/8", &key));
    CHECK(infw_make_rule(&val, 1, "TCP", "80", 0, 0, "Deny"));
    CHECK(infw_make_rule(&val, 2, "TCP", "1-1024", 0, 0, "Allow"));
    CHECK(infw_table_update(ctx, &key, &val, INFW_BPF_ANY));
    memset(&val, 0, sizeof(val));
    CHECK(infw_build_ebpf_key(7, "192.0.2.0/24", &key));
    CHECK(infw_make_rule(&val, 3, "UDP", "53", 0, 0, "Allow"));
    CHECK(infw_table_update(ctx, &key, &val, INFW_BPF_ANY));
    CHECK(infw_table_commit(ctx));

    /* the daemon's umem and ring memory, page-aligned as XDP_UMEM_REG wants it */
    uint8_t *umem = NULL;
    struct infw_xdp_desc *rx = NULL;
    uint32_t *results = NULL;
    uint8_t *verdicts = NULL;
    if (posix_memalign((void **)&umem, 4096, CHUNKS * CHUNK) || posix_memalign((void **)&rx, 4096, 4096) ||
        posix_memalign((void **)&results, 4096, 4096) || posix_memalign((void **)&verdicts, 4096, 4096)) {
        fprintf(stderr, "posix_memalign failed\n");
        return 1;
    }
    memset(umem, 0, CHUNKS * CHUNK);
    const uint8_t a[4] = {10, 1, 2, 3}, b[4] = {192, 0, 2, 9}, c[4] = {11, 0, 0, 1};
    /* packet i in chunk 2i+1 (a fill ring hands chunks out in any order), frame at chunk + headroom;
     * the last one arrives on the other interface's queue */
    const struct { const uint8_t *ip; uint8_t proto; uint16_t dport; uint32_t len; } pk[N] = {
        {a, 6, 80, 100},   /* rule 1: DROP  */
        {a, 6, 443, 200},  /* rule 2: PASS  */
        {a, 6, 2000, 300}, /* no rule: PASS */
        {b, 17, 53, 400},  /* rule 3: PASS  */
        {c, 6, 80, 500},   /* no prefix     */
        {a, 6, 80, 600},   /* ifindex 8: no entry */
    };
    for (int i = 0; i < N; i++) {
        const uint64_t at = (uint64_t)(2 * i + 1) * CHUNK + HEADROOM;
        put_frame(umem + at, pk[i].ip, pk[i].proto, pk[i].dport, pk[i].len);
        rx[i].addr = at;
        rx[i].len = pk[i].len;
        rx[i].options = 0;
    }
    /* the two interface rings as infw_classify_xdp_host takes them (one call) */
    const struct infw_xdp_ring rings[2] = {{umem, rx, N - 1, 7, 0, results, verdicts},
                                           {umem, rx + N - 1, 1, 8, 0, results + N - 1, verdicts + N - 1}};
    if (host_only) {
        int rc = infw_classify_xdp(ctx, 0, umem, rx, N - 1, 7, results, verdicts, NULL);
        if (rc != -ENODEV) {
            fprintf(stderr, "host-only classify_xdp returned %d, want -ENODEV\n", rc);
            return 1;
        }
        rc = infw_classify_xdp_host(ctx, 0, rings, 2, 0);
        if (rc != -ENODEV) {
            fprintf(stderr, "host-only classify_xdp_host returned %d, want -ENODEV\n", rc);
            return 1;
        }
        /* the host packer alone needs no device: frame 0's tuple as kernel.c reads it */
        uint32_t s4[N], ifx[N], plen[N], meta[N], l4[N];
        uint8_t tail[768];
        const struct infw_batch_soa_c_out o = {s4, tail, ifx, plen, meta, l4};
        CHECK(infw_pack_xdp_host(umem, rx, N, 7, &o));
        if (s4[0] != (10u | 1u << 8 | 2u << 16 | 3u << 24) || ifx[0] != 7 || plen[0] != 100 ||
            meta[0] != (0x0800u | 6u << 16 | 100u << 24) || l4[0] != (40000u >> 8 | (40000u & 0xFF) << 8 | 80u << 24)) {
            fprintf(stderr, "pack_xdp_host: frame 0 packed as %08x %u %u %08x %08x\n", s4[0], ifx[0], plen[0], meta[0],
                    l4[0]);
            return 1;
        }
        /* the event builder needs no device either: result words as a classify would have returned them */
        const uint32_t words[N] = {INFW_RESULT(INFW_XDP_DROP, 1), INFW_RESULT(INFW_XDP_PASS, 2), 0, 0, 0, 0};
        struct infw_event_sample ev[1];
        uint64_t n_ev = 0;
        CHECK(infw_xdp_host_events(umem, rx, N, 7, words, ev, 1, &n_ev));
        if (n_ev != 1 || ev[0].size != 108 || memcmp(ev[0].raw + 8, umem + rx[0].addr, 100) != 0) {
            fprintf(stderr, "host events: %llu events, size %u\n", (unsigned long long)n_ev, ev[0].size);
            return 1;
        }
        const uint8_t *fp[N];
        uint32_t fl[N];
        for (int i = 0; i < N; i++) fp[i] = umem + rx[i].addr, fl[i] = rx[i].len;
        const struct infw_frame_burst hb = {fp, fl, NULL, N - 1, 7, 0, results, NULL};
        rc = infw_classify_bursts_host(ctx, 0, &hb, 1, 0);
        if (rc != -ENODEV) {
            fprintf(stderr, "host-only classify_bursts_host returned %d, want -ENODEV\n", rc);
            return 1;
        }
        uint32_t s4b[N], plb[N], mb[N], l4b[N];
        uint8_t tailb[768];
        const struct infw_batch_soa_c_out ob = {s4b, tailb, NULL, plb, mb, l4b};
        CHECK(infw_pack_burst_host(&hb, &ob));
        for (int i = 0; i < N - 1; i++)
            if (s4b[i] != s4[i] || plb[i] != plen[i] || mb[i] != meta[i] || l4b[i] != l4[i]) {
                fprintf(stderr, "pack_burst_host: frame %d differs from pack_xdp_host\n", i);
                return 1;
            }
        infw_destroy(ctx);
        printf("xdp_demo OK (host): classify_xdp, classify_xdp_host and classify_bursts_host refused without a device, "
               "the host packers alone packed %d frames (rings and bursts alike), ABI %d\n", N, infw_abi_version());
        return 0;
    }
    {
        const int rc = infw_classify_xdp(ctx, 0, umem, rx, N - 1, 7, results, verdicts, NULL);
        if (rc != -EFAULT) {
            fprintf(stderr, "classify_xdp on pageable memory returned %d, want -EFAULT\n", rc);
            return 1;
        }
    }
    CHECK(infw_host_register(ctx, umem, CHUNKS * CHUNK));
    CHECK(infw_host_register(ctx, rx, 4096));
    CHECK(infw_host_register(ctx, results, 4096));
    CHECK(infw_host_register(ctx, verdicts, 4096));
    memset(results, 0xFF, 4 * N);
    memset(verdicts, 7, N);
    /* ring of ifindex 7: descriptors 0..4; ring of ifindex 8: descriptor 5 (NULL stream: the default one) */
    CHECK(infw_classify_xdp(ctx, 0, umem, rx, N - 1, 7, results, verdicts, NULL));
    CHECK(infw_classify_xdp(ctx, 0, umem, rx + N - 1, 1, 8, results + N - 1, verdicts + N - 1, NULL));
    if (hipDeviceSynchronize() != hipSuccess) {
        fprintf(stderr, "hipDeviceSynchronize failed\n");
        return 1;
    }
    const uint32_t want_r[N] = {INFW_RESULT(INFW_XDP_DROP, 1), INFW_RESULT(INFW_XDP_PASS, 2), 0,
                                INFW_RESULT(INFW_XDP_PASS, 3), 0, 0};
    const uint8_t want_v[N] = {INFW_XDP_DROP, INFW_XDP_PASS, INFW_XDP_PASS, INFW_XDP_PASS, INFW_XDP_PASS, INFW_XDP_PASS};
    for (int i = 0; i < N; i++)
        if (verdicts[i] != want_v[i] || results[i] != want_r[i]) {
            fprintf(stderr, "frame %d: verdict %u result 0x%x, want %u 0x%x\n", i, verdicts[i], results[i],
                    want_v[i], want_r[i]);
            return 1;
        }
    /* per-rule counters (bytes = the descriptor's frame length, bpf_xdp_get_buff_len) */
    struct ruleStatistics_st st[8];
    int slots = 0;
    uint64_t allow = 0, deny = 0, allow_b = 0, deny_b = 0;
    for (uint32_t rule = 1; rule < 100; rule++) {
        CHECK(infw_stats_read(ctx, rule, st, &slots));
        for (int s = 0; s < slots; s++) {
            allow += st[s].allow_stats.packets;
            allow_b += st[s].allow_stats.bytes;
            deny += st[s].deny_stats.packets;
            deny_b += st[s].deny_stats.bytes;
        }
    }
    if (allow != 2 || allow_b != 600 || deny != 1 || deny_b != 100) {
        fprintf(stderr, "counters: allow %llu/%llu deny %llu/%llu\n", (unsigned long long)allow,
                (unsigned long long)allow_b, (unsigned long long)deny, (unsigned long long)deny_b);
        return 1;
    }
    CHECK(infw_host_unregister(ctx, umem));
    CHECK(infw_host_unregister(ctx, rx));
    CHECK(infw_host_unregister(ctx, results));
    CHECK(infw_host_unregister(ctx, verdicts));

    /* the host-fed path over the same memory, now ordinary pageable memory again: the library's packer threads read
     * the frames on the CPU; both rings in one synchronous call; same verdicts, counters doubled */
    memset(results, 0xFF, 4 * N);
    memset(verdicts, 7, N);
    CHECK(infw_classify_xdp_host(ctx, 0, rings, 2, 0));
    for (int i = 0; i < N; i++)
        if (verdicts[i] != want_v[i] || results[i] != want_r[i]) {
            fprintf(stderr, "host-fed frame %d: verdict %u result 0x%x, want %u 0x%x\n", i, verdicts[i], results[i],
                    want_v[i], want_r[i]);
            return 1;
        }
    struct ruleStatistics_st all[INFW_MAX_TARGETS];
    CHECK(infw_stats_read_all(ctx, all));
    uint64_t allow2 = 0, deny2 = 0, allow2_b = 0, deny2_b = 0;
    for (int rule = 1; rule < 100; rule++) {
        allow2 += all[rule].allow_stats.packets, allow2_b += all[rule].allow_stats.bytes;
        deny2 += all[rule].deny_stats.packets, deny2_b += all[rule].deny_stats.bytes;
    }
    if (allow2 != 2 * allow || allow2_b != 2 * allow_b || deny2 != 2 * deny || deny2_b != 2 * deny_b) {
        fprintf(stderr, "host-fed counters: allow %llu/%llu deny %llu/%llu\n", (unsigned long long)allow2,
                (unsigned long long)allow2_b, (unsigned long long)deny2, (unsigned long long)deny2_b);
        return 1;
    }
    /* the ring's deny events for the events reader (kernel.c:392-399), built on the host from the frames and the
     * result words: frame 0 (rule 1, 100 B) is the one denied packet of ring 7 */
    struct infw_event_sample ev[2];
    uint64_t n_ev = 0;
    CHECK(infw_xdp_host_events(umem, rx, N - 1, 7, results, ev, 2, &n_ev));
    const struct event_hdr_st *eh = (const struct event_hdr_st *)ev[0].raw;
    if (n_ev != 1 || ev[0].size != ((8 + 100 + 4 + 7) & ~7) - 4 || eh->ifId != 7 || eh->ruleId != 1 || eh->action != 1 ||
        eh->pktLength != 100 || memcmp(ev[0].raw + 8, umem + rx[0].addr, 100) != 0) {
        fprintf(stderr, "host events: %llu events, size %u\n", (unsigned long long)n_ev, ev[0].size);
        return 1;
    }

    /* DPDK-style: each frame in a buffer of its own (an mbuf's data room, at a 128-B headroom); packet 1's frame split
     * over two segments after 60 B (data_len 60 < pkt_len 200: kernel.c reads only the linear part, and its bytes are
     * all inside it); one burst per port; result words as slices of one array, verdicts not wanted */
    uint8_t *mbuf[N];
    const uint8_t *ptr[N];
    uint32_t dlen[N], plen2[N], res[N];
    for (int i = 0; i < N; i++) {
        if (posix_memalign((void **)&mbuf[i], 64, 2048)) return 1;
        memset(mbuf[i], 0, 2048);
        memcpy(mbuf[i] + 128, umem + rx[i].addr, pk[i].len);
        ptr[i] = mbuf[i] + 128, plen2[i] = pk[i].len, dlen[i] = i == 1 ? 60 : pk[i].len;
    }
    memset(res, 0xFF, sizeof(res));
    const struct infw_frame_burst bursts[2] = {{ptr, dlen, plen2, N - 1, 7, 0, res, NULL},
                                               {ptr + N - 1, dlen + N - 1, plen2 + N - 1, 1, 8, 0, res + N - 1, NULL}};
    CHECK(infw_classify_bursts_host(ctx, 0, bursts, 2, 0));
    for (int i = 0; i < N; i++)
        if (res[i] != want_r[i]) {
            fprintf(stderr, "burst frame %d: result 0x%x, want 0x%x\n", i, res[i], want_r[i]);
            return 1;
        }
    CHECK(infw_stats_read_all(ctx, all));
    uint64_t allow3 = 0, deny3 = 0;
    for (int rule = 1; rule < 100; rule++) allow3 += all[rule].allow_stats.packets, deny3 += all[rule].deny_stats.packets;
    if (allow3 != 3 * allow || deny3 != 3 * deny) {
        fprintf(stderr, "burst counters: allow %llu deny %llu\n", (unsigned long long)allow3, (unsigned long long)deny3);
        return 1;
    }
    n_ev = 0;
    CHECK(infw_burst_host_events(&bursts[0], res, ev, 2, &n_ev));
    if (n_ev != 1 || ev[0].size != ((8 + 100 + 4 + 7) & ~7) - 4 || memcmp(ev[0].raw + 8, ptr[0], 100) != 0) {
        fprintf(stderr, "burst events: %llu events, size %u\n", (unsigned long long)n_ev, ev[0].size);
        return 1;
    }
    for (int i = 0; i < N; i++) free(mbuf[i]);
    infw_destroy(ctx);
    free(umem), free(rx), free(results), free(verdicts);
    printf("xdp_demo OK: %d frames in 2 rings, allow %llu (%llu B), deny %llu (%llu B); pageable memory refused by the "
           "device read (-EFAULT) and classified by the host-fed path, its deny event built on the host; the same "
           "frames as DPDK-style bursts (one split over two segments) give the same words and event, ABI %d\n", N,
           (unsigned long long)allow, (unsigned long long)allow_b, (unsigned long long)deny,
           (unsigned long long)deny_b, infw_abi_version());
    return 0;
}
