/*
 * abi_demo.c — the drop-in boundary driven from plain C, the way a cgo build of pkg/ebpf would
 * (INTEGRATION.md): no Python, no torch, host-resident batches through infw_classify_host.
 *
 *   IngressNodeFwRulesLoader (loader.go:130-194):  infw_build_ebpf_key + infw_make_rule -> infw_table_update,
 *                                                  infw_table_commit
 *   the XDP entry per frame (kernel.c:459-462):    infw_classify_host over a SoA batch in host memory
 *   statsMap.Lookup (statistics.go:127):           infw_stats_read
 *
 * Built by tests/test_c_abi.py (gcc, linked against lib/libinfw.so); run on the GPU by its -m gpu test.
 * `abi_demo host` runs on a box without a GPU: an INFW_F_HOST_ONLY context, whose infw_classify_host must refuse
 * (-ENODEV: there is no CPU path), checked instead through the tests-only infw_debug_walk over the host image.
 * Prints "abi_demo OK ..." and exits 0 when every verdict and counter is the expected one.
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "infw.h"

#define CHECK(call)                                                                                 \
    do {                                                                                            \
        int rc_ = (call);                                                                           \
        if (rc_ < 0) {                                                                              \
            fprintf(stderr, "%s failed: %d (%s)\n", #call, rc_, infw_last_error());                 \
            return 1;                                                                               \
        }                                                                                           \
    } while (0)

/* One packet of the batch: an IPv4 TCP/UDP frame's tuple (include/infw.h, struct infw_batch_soa). */
static void put_v4(uint8_t *saddr, uint32_t *ifindex, uint32_t *pkt_len, uint32_t *meta, uint32_t *l4word, int i,
                   const uint8_t ip[4], uint32_t ifx, uint8_t proto, uint16_t dport, uint32_t len) {
    memset(saddr + 16 * i, 0, 16);
    memcpy(saddr + 16 * i, ip, 4);
    ifindex[i] = ifx;
    pkt_len[i] = len;
    meta[i] = INFW_META(0x0800u, proto, len);
    /* frame[34..37]: source port (big endian), destination port (big endian), little-endian word */
    const uint16_t sport = 40000;
    l4word[i] = (uint32_t)(sport >> 8) | (uint32_t)(sport & 0xFF) << 8 | (uint32_t)(dport >> 8) << 16 |
                (uint32_t)(dport & 0xFF) << 24;
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

    enum { N = 6 };
    uint8_t saddr[16 * N];
    uint32_t ifindex[N], pkt_len[N], meta[N], l4word[N], results[N];
    uint8_t verdicts[N];
    const uint8_t a[4] = {10, 1, 2, 3}, b[4] = {192, 0, 2, 9}, c[4] = {11, 0, 0, 1};
    put_v4(saddr, ifindex, pkt_len, meta, l4word, 0, a, 7, 6, 80, 100);   /* rule 1: DROP  */
    put_v4(saddr, ifindex, pkt_len, meta, l4word, 1, a, 7, 6, 443, 200);  /* rule 2: PASS  */
    put_v4(saddr, ifindex, pkt_len, meta, l4word, 2, a, 7, 6, 2000, 300); /* no rule: PASS */
    put_v4(saddr, ifindex, pkt_len, meta, l4word, 3, b, 7, 17, 53, 400);  /* rule 3: PASS  */
    put_v4(saddr, ifindex, pkt_len, meta, l4word, 4, c, 7, 6, 80, 500);   /* no prefix     */
    put_v4(saddr, ifindex, pkt_len, meta, l4word, 5, a, 8, 6, 80, 600);   /* other iface   */
    const struct infw_batch_soa in = {saddr, ifindex, pkt_len, meta, l4word};
    const uint32_t want_r[N] = {INFW_RESULT(INFW_XDP_DROP, 1), INFW_RESULT(INFW_XDP_PASS, 2), 0,
                                INFW_RESULT(INFW_XDP_PASS, 3), 0, 0};
    if (host_only) {
        const int rc = infw_classify_host(ctx, 0, &in, N, results, verdicts, 0);
        if (rc != -ENODEV) {
            fprintf(stderr, "host-only classify returned %d, want -ENODEV\n", rc);
            return 1;
        }
        uint32_t tuples[8 * N];
        for (int i = 0; i < N; i++) {
            memcpy(tuples + 8 * i, saddr + 16 * i, 16);
            tuples[8 * i + 4] = ifindex[i];
            tuples[8 * i + 5] = pkt_len[i];
            tuples[8 * i + 6] = meta[i];
            tuples[8 * i + 7] = l4word[i];
        }
        CHECK(infw_debug_walk(ctx, tuples, N, results));
        for (int i = 0; i < N; i++)
            if (results[i] != want_r[i]) {
                fprintf(stderr, "packet %d: result 0x%x, want 0x%x\n", i, results[i], want_r[i]);
                return 1;
            }
        struct rulesVal_st got;
        CHECK(infw_build_ebpf_key(7, "10.9.9.9/32", &key));
        CHECK(infw_table_lookup(ctx, &key, &got));
        if (got.rules[1].ruleId != 1 || got.rules[1].action != INFW_XDP_DROP || got.rules[2].dstPortEnd != 1024) {
            fprintf(stderr, "lookup of 10.9.9.9 did not return the /8's rules\n");
            return 1;
        }
        infw_destroy(ctx);
        printf("abi_demo OK (host): %d packets walked, ABI %d\n", N, infw_abi_version());
        return 0;
    }
    CHECK(infw_classify_host(ctx, 0, &in, N, results, verdicts, 0));

    const uint8_t want_v[N] = {INFW_XDP_DROP, INFW_XDP_PASS, INFW_XDP_PASS, INFW_XDP_PASS, INFW_XDP_PASS, INFW_XDP_PASS};
    for (int i = 0; i < N; i++)
        if (verdicts[i] != want_v[i] || results[i] != want_r[i]) {
            fprintf(stderr, "packet %d: verdict %u result 0x%x, want %u 0x%x\n", i, verdicts[i], results[i],
                    want_v[i], want_r[i]);
            return 1;
        }

    /* per-rule counters: one slot per device, summed like statistics.go:126-157 */
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
    /* Map.Delete + a commit: the /8 goes away, packet 0 falls through */
    CHECK(infw_build_ebpf_key(7, "10.0.0.0/8", &key));
    CHECK(infw_table_delete(ctx, &key));
    CHECK(infw_table_commit(ctx));
    CHECK(infw_classify_host(ctx, 0, &in, 1, results, verdicts, 0));
    if (verdicts[0] != INFW_XDP_PASS || results[0] != 0) {
        fprintf(stderr, "after delete: verdict %u result 0x%x\n", verdicts[0], results[0]);
        return 1;
    }
    infw_destroy(ctx);
    printf("abi_demo OK: %d packets, allow %llu (%llu B), deny %llu (%llu B), ABI %d\n", N, (unsigned long long)allow,
           (unsigned long long)allow_b, (unsigned long long)deny, (unsigned long long)deny_b, infw_abi_version());
    return 0;
}
