/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see infw_oracle.h for scope and pinning).
 *
 * Plain C restatement of pbmoses/ingress-node-firewall's XDP hot path
 * (bpf/ingress_node_firewall_kernel.c) and of the LPM-trie map semantics it
 * runs against.  Written to be obviously correct, not fast:
 *   - frames are parsed byte by byte at the program's fixed offsets;
 *   - the LPM is a hash set per (prefixLen, masked data) probed from the
 *     longest candidate length down, which is the definition of longest-prefix
 *     match that kernel/bpf/lpm_trie.c implements with a path-compressed trie;
 *   - rules are read from the packed 1200-byte value exactly as the program
 *     reads rulesVal_st.
 */
#define _GNU_SOURCE
#include "infw_oracle.h"

#include <errno.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* kernel.c / ingress_node_firewall.h constants */
#define ETH_HLEN 14              /* sizeof(struct ethhdr)   vmlinux.h:31465 */
#define IPV4_HLEN 20             /* sizeof(struct iphdr)    vmlinux.h:31739 */
#define IPV6_HLEN 40             /* sizeof(struct ipv6hdr)  vmlinux.h:31761 */
#define TCP_HLEN 20              /* sizeof(struct tcphdr)   */
#define UDP_HLEN 8               /* sizeof(struct udphdr)   */
#define SCTP_HLEN 12             /* sizeof(struct sctphdr)  */
#define ICMP_HLEN 8              /* sizeof(struct icmphdr)  */
#define ICMP6_HLEN 8             /* sizeof(struct icmp6hdr) */
#define XDP_ABORTED 0
#define XDP_DROP 1
#define XDP_PASS 2
#define UNDEF XDP_ABORTED        /* ingress_node_firewall.h:10 */
#define DENY XDP_DROP            /* :11 */
#define ALLOW XDP_PASS           /* :12 */
#define INVALID_RULE_ID 0        /* :16 */
#define IPPROTO_ICMP 1
#define IPPROTO_TCP 6
#define IPPROTO_UDP 17
#define IPPROTO_ICMPV6 58        /* ingress_node_firewall.h:8 */
#define IPPROTO_SCTP 132
#define BPF_ANY 0
#define BPF_NOEXIST 1
#define BPF_EXIST 2
#define MAX_EVENT_DATA 256       /* :15 */

/* ingress_node_firewall.h:18-23 */
#define GET_ACTION(a) ((uint8_t)((a)&0xFF))
#define SET_ACTION(a) ((uint32_t)(((uint32_t)(a)) & 0xFF))
#define GET_RULE_ID(r) ((uint16_t)(((r) >> 8) & 0xFFFFFF))
#define SET_ACTIONRULE_RESPONSE(a, r) ((uint32_t)((((uint32_t)(r)) & 0xFFFFFF) << 8 | ((a)&0xFF)))

static inline uint32_t rd_le32(const uint8_t *p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}
static inline uint16_t rd_le16(const uint8_t *p) { return (uint16_t)(p[0] | p[1] << 8); }
static inline void wr_le32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

static uint64_t hash_bytes(const uint8_t *p, size_t n, uint64_t seed) {
    uint64_t h = seed ^ (n * 0x9E3779B97F4A7C15ull);
    for (size_t i = 0; i < n; i++) {
        h ^= p[i];
        h *= 0x100000001B3ull;
    }
    h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33;
    return h;
}

/* ------------------------------------------------------------------------ */
/* Interned 1200-byte values (many keys share one rule list).               */
/* ------------------------------------------------------------------------ */
typedef struct {
    uint8_t **slots;
    uint64_t cap, n;
} val_pool;

static const uint8_t *pool_intern(val_pool *vp, const uint8_t *val) {
    if ((vp->n + 1) * 2 > vp->cap) {
        uint64_t ncap = vp->cap ? vp->cap * 2 : 1024;
        uint8_t **ns = (uint8_t **)calloc(ncap, sizeof(uint8_t *));
        for (uint64_t i = 0; i < vp->cap; i++) {
            if (!vp->slots[i]) continue;
            uint64_t h = hash_bytes(vp->slots[i], ORC_VALUE_SIZE, 7) & (ncap - 1);
            while (ns[h]) h = (h + 1) & (ncap - 1);
            ns[h] = vp->slots[i];
        }
        free(vp->slots);
        vp->slots = ns;
        vp->cap = ncap;
    }
    uint64_t h = hash_bytes(val, ORC_VALUE_SIZE, 7) & (vp->cap - 1);
    while (vp->slots[h]) {
        if (memcmp(vp->slots[h], val, ORC_VALUE_SIZE) == 0) return vp->slots[h];
        h = (h + 1) & (vp->cap - 1);
    }
    uint8_t *c = (uint8_t *)malloc(ORC_VALUE_SIZE);
    memcpy(c, val, ORC_VALUE_SIZE);
    vp->slots[h] = c;
    vp->n++;
    return c;
}

/* ------------------------------------------------------------------------ */
/* LPM trie map (kernel.c:50-57).  Trie data = key bytes [4..24):            */
/* ingress_ifindex (LE) then ip_data, compared MSB-first (lpm_trie.c).      */
/* ------------------------------------------------------------------------ */
typedef struct {
    uint32_t plen;       /* prefixLen; UINT32_MAX = empty, UINT32_MAX-1 = tombstone */
    uint8_t mdata[20];   /* data masked to plen bits (identity of the node)  */
    uint8_t data[20];    /* data as written by the last update (host bits kept) */
    const uint8_t *val;
} map_ent;

#define ENT_EMPTY 0xFFFFFFFFu
#define ENT_TOMB 0xFFFFFFFEu

struct orc_map {
    map_ent *tab;
    uint64_t cap, n, used;  /* used = live + tombstones */
    uint32_t max_entries;
    uint32_t len_count[ORC_MAX_PREFIXLEN + 1];
    val_pool pool;
};

static void mask_data(const uint8_t *in, uint32_t plen, uint8_t *out) {
    for (uint32_t i = 0; i < 20; i++) {
        uint32_t bit0 = i * 8;
        if (plen >= bit0 + 8) out[i] = in[i];
        else if (plen <= bit0) out[i] = 0;
        else out[i] = (uint8_t)(in[i] & (0xFFu << (8 - (plen - bit0))));
    }
}

static uint64_t ent_hash(uint32_t plen, const uint8_t *mdata) {
    return hash_bytes(mdata, 20, 0x51ED27ull + plen);
}

static map_ent *map_find(const orc_map *m, uint32_t plen, const uint8_t *mdata) {
    uint64_t h = ent_hash(plen, mdata) & (m->cap - 1);
    for (;;) {
        map_ent *e = &m->tab[h];
        if (e->plen == ENT_EMPTY) return NULL;
        if (e->plen == plen && memcmp(e->mdata, mdata, 20) == 0) return e;
        h = (h + 1) & (m->cap - 1);
    }
}

static void map_rehash(orc_map *m, uint64_t ncap) {
    map_ent *old = m->tab;
    uint64_t ocap = m->cap;
    m->tab = (map_ent *)malloc(ncap * sizeof(map_ent));
    for (uint64_t i = 0; i < ncap; i++) m->tab[i].plen = ENT_EMPTY;
    m->cap = ncap;
    m->used = m->n;
    for (uint64_t i = 0; i < ocap; i++) {
        if (old[i].plen >= ENT_TOMB) continue;
        uint64_t h = ent_hash(old[i].plen, old[i].mdata) & (ncap - 1);
        while (m->tab[h].plen != ENT_EMPTY) h = (h + 1) & (ncap - 1);
        m->tab[h] = old[i];
    }
    free(old);
}

orc_map *orc_map_create(uint32_t max_entries) {
    orc_map *m = (orc_map *)calloc(1, sizeof(orc_map));
    m->max_entries = max_entries;
    m->cap = 1024;
    m->tab = (map_ent *)malloc(m->cap * sizeof(map_ent));
    for (uint64_t i = 0; i < m->cap; i++) m->tab[i].plen = ENT_EMPTY;
    return m;
}

void orc_map_destroy(orc_map *m) {
    if (!m) return;
    for (uint64_t i = 0; i < m->pool.cap; i++) free(m->pool.slots[i]);
    free(m->pool.slots);
    free(m->tab);
    free(m);
}

uint64_t orc_map_count(const orc_map *m) { return m->n; }

/* trie_update_elem (lpm_trie.c, 6.18): flags check, prefixlen check, replace
 * in place when the exact prefix exists (also when the map is full),
 * NOEXIST/EXIST, then -ENOSPC for a new node on a full map. */
int orc_map_update(orc_map *m, const uint8_t *key, const uint8_t *val, uint64_t flags) {
    if (flags > BPF_EXIST) return -EINVAL;
    uint32_t plen = rd_le32(key);
    if (plen > ORC_MAX_PREFIXLEN) return -EINVAL;
    uint8_t md[20];
    mask_data(key + 4, plen, md);
    map_ent *e = map_find(m, plen, md);
    if (e) {
        if (flags == BPF_NOEXIST) return -EEXIST;
        memcpy(e->data, key + 4, 20);
        e->val = pool_intern(&m->pool, val);
        return 0;
    }
    if (flags == BPF_EXIST) return -ENOENT;
    if (m->n == m->max_entries) return -ENOSPC;
    if ((m->used + 1) * 2 > m->cap) map_rehash(m, m->n * 4 > m->cap ? m->cap * 2 : m->cap);
    uint64_t h = ent_hash(plen, md) & (m->cap - 1);
    while (m->tab[h].plen < ENT_TOMB) h = (h + 1) & (m->cap - 1);
    if (m->tab[h].plen == ENT_EMPTY) m->used++;
    map_ent *ne = &m->tab[h];
    ne->plen = plen;
    memcpy(ne->mdata, md, 20);
    memcpy(ne->data, key + 4, 20);
    ne->val = pool_intern(&m->pool, val);
    m->n++;
    m->len_count[plen]++;
    return 0;
}

/* trie_delete_elem: exact prefixlen + prefix bits, host bits ignored. */
int orc_map_delete(orc_map *m, const uint8_t *key) {
    uint32_t plen = rd_le32(key);
    if (plen > ORC_MAX_PREFIXLEN) return -EINVAL;
    uint8_t md[20];
    mask_data(key + 4, plen, md);
    map_ent *e = map_find(m, plen, md);
    if (!e) return -ENOENT;
    e->plen = ENT_TOMB;
    m->n--;
    m->len_count[plen]--;
    return 0;
}

/* Longest prefix match over entries with prefixlen <= key prefixlen. */
static const map_ent *map_lpm(const orc_map *m, uint32_t key_plen, const uint8_t *data) {
    if (key_plen > ORC_MAX_PREFIXLEN) key_plen = ORC_MAX_PREFIXLEN;
    uint8_t md[20];
    for (int L = (int)key_plen; L >= 0; L--) {
        if (!m->len_count[L]) continue;
        mask_data(data, (uint32_t)L, md);
        const map_ent *e = map_find(m, (uint32_t)L, md);
        if (e) return e;
    }
    return NULL;
}

int orc_map_lookup(const orc_map *m, const uint8_t *key, uint8_t *val_out) {
    const map_ent *e = map_lpm(m, rd_le32(key), key + 4);
    if (!e) return -ENOENT;
    if (val_out) memcpy(val_out, e->val, ORC_VALUE_SIZE);
    return 0;
}

static int bit_at(const uint8_t *d, uint32_t i) { return (d[i >> 3] >> (7 - (i & 7))) & 1; }

/* Post-order of the trie: a node's subtree before the node, child[0] before
 * child[1] (trie_get_next_key). */
static int postorder_cmp(const map_ent *a, const map_ent *b) {
    uint32_t mn = a->plen < b->plen ? a->plen : b->plen;
    for (uint32_t i = 0; i < mn; i++) {
        int x = bit_at(a->mdata, i), y = bit_at(b->mdata, i);
        if (x != y) return x < y ? -1 : 1;
    }
    if (a->plen == b->plen) return 0;
    return a->plen > b->plen ? -1 : 1; /* longer (descendant) first */
}

int orc_map_get_next_key(const orc_map *m, const uint8_t *key, uint8_t *next) {
    const map_ent *best = NULL;   /* smallest entry > key (or overall smallest) */
    map_ent probe;
    int have_key = 0;
    if (key && rd_le32(key) <= ORC_MAX_PREFIXLEN) {
        probe.plen = rd_le32(key);
        mask_data(key + 4, probe.plen, probe.mdata);
        have_key = map_find(m, probe.plen, probe.mdata) != NULL;
    }
    for (uint64_t i = 0; i < m->cap; i++) {
        const map_ent *e = &m->tab[i];
        if (e->plen >= ENT_TOMB) continue;
        if (have_key && postorder_cmp(e, &probe) <= 0) continue;
        if (!best || postorder_cmp(e, best) < 0) best = e;
    }
    if (!best) return -ENOENT;
    wr_le32(next, best->plen);
    memcpy(next + 4, best->data, 20);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* The XDP program, kernel.c:95-457.                                         */
/* ------------------------------------------------------------------------ */

/* ip_extract_l4info, kernel.c:95-174 */
static int ip_extract_l4info(const uint8_t *data, uint32_t data_end, uint8_t *proto,
                             uint16_t *dstPort, uint8_t *icmpType, uint8_t *icmpCode,
                             int is_v4) {
    uint32_t dataStart = ETH_HLEN;
    if (is_v4) {
        dataStart += IPV4_HLEN;                       /* :104 — IHL is not consulted */
        if (dataStart > data_end) return -1;
        *proto = data[ETH_HLEN + 9];                  /* iph->protocol */
    } else {
        dataStart += IPV6_HLEN;                       /* :111 — no extension headers */
        if (dataStart > data_end) return -1;
        *proto = data[ETH_HLEN + 6];                  /* iph->nexthdr */
    }
    switch (*proto) {
    case IPPROTO_TCP:
        if (dataStart + TCP_HLEN > data_end) return -1;
        *dstPort = (uint16_t)(data[dataStart + 2] | data[dataStart + 3] << 8); /* tcph->dest, network order */
        break;
    case IPPROTO_UDP:
        if (dataStart + UDP_HLEN > data_end) return -1;
        *dstPort = (uint16_t)(data[dataStart + 2] | data[dataStart + 3] << 8);
        break;
    case IPPROTO_SCTP:
        if (dataStart + SCTP_HLEN > data_end) return -1;
        *dstPort = (uint16_t)(data[dataStart + 2] | data[dataStart + 3] << 8);
        break;
    case IPPROTO_ICMP:
        if (dataStart + ICMP_HLEN > data_end) return -1;
        *icmpType = data[dataStart];
        *icmpCode = data[dataStart + 1];
        break;
    case IPPROTO_ICMPV6:
        if (dataStart + ICMP6_HLEN > data_end) return -1;
        *icmpType = data[dataStart];
        *icmpCode = data[dataStart + 1];
        break;
    default:
        return -1;
    }
    return 0;
}

static inline uint16_t bpf_ntohs(uint16_t x) { return (uint16_t)((x >> 8) | (x << 8)); }

/* The first-match loop shared by ipv4_firewall_lookup (:222-258) and
 * ipv6_firewall_lookup (:306-340); they differ only in the ICMP protocol
 * number honoured (IPPROTO_ICMP on the v4 path, IPPROTO_ICMPV6 on v6). */
/* examined (may be NULL): += the valid rules (ruleId != 0) looked at, up to and
 * including the first match (SURVEY.md §8d "rule bytes examined" = 12 B each). */
static uint32_t scan_rules(const uint8_t *rulesVal, uint8_t proto, uint16_t dstPort,
                           uint8_t icmpType, uint8_t icmpCode, uint8_t icmp_proto, uint64_t *examined) {
    for (int i = 0; i < ORC_MAX_RULES; ++i) {
        const uint8_t *r = rulesVal + 12 * i;
        uint32_t ruleId = rd_le32(r);
        uint8_t protocol = r[4];
        uint16_t dstPortStart = rd_le16(r + 5);
        uint16_t dstPortEnd = rd_le16(r + 7);
        uint8_t rIcmpType = r[9], rIcmpCode = r[10], action = r[11];
        if (ruleId == INVALID_RULE_ID) continue;
        if (examined) ++*examined;
        if (protocol != 0 && protocol == proto) {
            if (protocol == IPPROTO_TCP || protocol == IPPROTO_UDP || protocol == IPPROTO_SCTP) {
                if (dstPortEnd == 0) {
                    if (dstPortStart == bpf_ntohs(dstPort))
                        return SET_ACTIONRULE_RESPONSE(action, ruleId);
                } else {
                    if (bpf_ntohs(dstPort) >= dstPortStart && bpf_ntohs(dstPort) < dstPortEnd)
                        return SET_ACTIONRULE_RESPONSE(action, ruleId);
                }
            }
            if (protocol == icmp_proto) {
                if (rIcmpType == icmpType && rIcmpCode == icmpCode)
                    return SET_ACTIONRULE_RESPONSE(action, ruleId);
            }
        }
        if (protocol == 0) return SET_ACTIONRULE_RESPONSE(action, ruleId);
    }
    return SET_ACTION(UNDEF);
}

/* ipv4_firewall_lookup, kernel.c:189-262 */
static uint32_t ipv4_firewall_lookup(const orc_map *m, const uint8_t *data, uint32_t data_end,
                                     uint32_t ifId, uint64_t *examined) {
    uint16_t dstPort = 0;
    uint8_t icmpCode = 0, icmpType = 0, proto = 0;
    if (ip_extract_l4info(data, data_end, &proto, &dstPort, &icmpType, &icmpCode, 1) < 0)
        return SET_ACTION(UNDEF);
    uint8_t kd[20] = {0};
    wr_le32(kd, ifId);                                /* key.ingress_ifindex */
    memcpy(kd + 4, data + ETH_HLEN + 12, 4);          /* key.ip_data[0..3] = saddr bytes */
    const map_ent *e = map_lpm(m, 64, kd);            /* key.prefixLen = 64 (:207) */
    if (!e) return SET_ACTION(UNDEF);
    return scan_rules(e->val, proto, dstPort, icmpType, icmpCode, IPPROTO_ICMP, examined);
}

/* ipv6_firewall_lookup, kernel.c:277-344 */
static uint32_t ipv6_firewall_lookup(const orc_map *m, const uint8_t *data, uint32_t data_end,
                                     uint32_t ifId, uint64_t *examined) {
    uint16_t dstPort = 0;
    uint8_t icmpCode = 0, icmpType = 0, proto = 0;
    if (ip_extract_l4info(data, data_end, &proto, &dstPort, &icmpType, &icmpCode, 0) < 0)
        return SET_ACTION(UNDEF);
    uint8_t kd[20];
    wr_le32(kd, ifId);
    memcpy(kd + 4, data + ETH_HLEN + 8, 16);          /* iph->saddr */
    const map_ent *e = map_lpm(m, 160, kd);           /* key.prefixLen = 160 (:293) */
    if (!e) return SET_ACTION(UNDEF);
    return scan_rules(e->val, proto, dstPort, icmpType, icmpCode, IPPROTO_ICMPV6, examined);
}

/* generate_event_and_update_statistics, kernel.c:361-400 (statistics part;
 * the perf record is reported through *event_out). */
static void update_statistics(struct orc_stats *stats, uint64_t packet_len, uint8_t action,
                              uint16_t ruleId) {
    uint32_t key = ruleId;
    if (!stats || key >= ORC_MAX_TARGETS) return;  /* PERCPU_ARRAY lookup fails, update fails */
    switch (action) {
    case ALLOW:
        stats[key].allow_packets += 1;
        stats[key].allow_bytes += packet_len;
        break;
    case DENY:
        stats[key].deny_packets += 1;
        stats[key].deny_bytes += packet_len;
        break;
    }
}

/* ingress_node_firewall_main, kernel.c:412-457 */
static int xdp_run(const orc_map *m, struct orc_stats *stats, const uint8_t *data, uint32_t linear_len,
                   uint32_t buff_len, uint32_t ifindex, uint32_t *result_out, int *event_out,
                   uint64_t *examined) {
    uint32_t result = UNDEF;
    if (result_out) *result_out = 0;
    if (event_out) *event_out = 0;
    if (ETH_HLEN > linear_len) return XDP_DROP;       /* :423-426 */
    uint16_t h_proto = (uint16_t)(data[12] << 8 | data[13]);
    switch (h_proto) {
    case 0x0800: result = ipv4_firewall_lookup(m, data, linear_len, ifindex, examined); break;
    case 0x86DD: result = ipv6_firewall_lookup(m, data, linear_len, ifindex, examined); break;
    default: return XDP_PASS;                         /* :436-438 */
    }
    if (result_out) *result_out = result;
    uint16_t ruleId = GET_RULE_ID(result);
    uint8_t action = GET_ACTION(result);
    switch (action) {
    case DENY:
        update_statistics(stats, buff_len, DENY, ruleId);
        if (event_out) *event_out = 1;
        return XDP_DROP;
    case ALLOW:
        update_statistics(stats, buff_len, ALLOW, ruleId);
        return XDP_PASS;
    default:
        return XDP_PASS;
    }
}

int orc_xdp_run(const orc_map *m, struct orc_stats *stats, const uint8_t *data,
                uint32_t linear_len, uint32_t buff_len, uint32_t ifindex, uint32_t *result_out,
                int *event_out) {
    return xdp_run(m, stats, data, linear_len, buff_len, ifindex, result_out, event_out, NULL);
}

uint64_t orc_rules_examined(const orc_map *m, const uint8_t *frames, const uint64_t *offsets,
                            const uint32_t *caplen, const uint32_t *pkt_len, const uint32_t *ifindex,
                            uint64_t n) {
    uint64_t ex = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint32_t lin = caplen[i] < pkt_len[i] ? caplen[i] : pkt_len[i];
        uint32_t res;
        xdp_run(m, NULL, frames + offsets[i], lin, pkt_len[i], ifindex[i], &res, NULL, &ex);
    }
    return ex;
}

/* ------------------------------------------------------------------------ */
/* Batch driver: one worker per CPU with its own stats slot (PERCPU_ARRAY). */
/* ------------------------------------------------------------------------ */
typedef struct {
    const orc_map *m;
    const uint8_t *frames;
    const uint64_t *offsets;
    const uint32_t *caplen, *pkt_len, *ifindex;
    uint64_t begin, end;
    uint32_t *results;
    uint8_t *verdicts;
    struct orc_stats *stats;
} worker_arg;

static void *worker(void *p) {
    worker_arg *a = (worker_arg *)p;
    for (uint64_t i = a->begin; i < a->end; i++) {
        uint32_t lin = a->caplen[i] < a->pkt_len[i] ? a->caplen[i] : a->pkt_len[i];
        uint32_t res;
        int v = orc_xdp_run(a->m, a->stats, a->frames + a->offsets[i], lin, a->pkt_len[i],
                            a->ifindex[i], &res, NULL);
        if (a->results) a->results[i] = res;
        if (a->verdicts) a->verdicts[i] = (uint8_t)v;
    }
    return NULL;
}

double orc_classify_frames(const orc_map *m, const uint8_t *frames, const uint64_t *offsets,
                           const uint32_t *caplen, const uint32_t *pkt_len,
                           const uint32_t *ifindex, uint64_t n, uint32_t *results,
                           uint8_t *verdicts, struct orc_stats *stats_sum, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if ((uint64_t)nthreads > n && n > 0) nthreads = (int)n;
    worker_arg *args = (worker_arg *)calloc((size_t)nthreads, sizeof(worker_arg));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    struct orc_stats *slots =
        (struct orc_stats *)calloc((size_t)nthreads * ORC_MAX_TARGETS, sizeof(struct orc_stats));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < nthreads; t++) {
        worker_arg *a = &args[t];
        a->m = m; a->frames = frames; a->offsets = offsets; a->caplen = caplen;
        a->pkt_len = pkt_len; a->ifindex = ifindex; a->results = results; a->verdicts = verdicts;
        a->begin = n * (uint64_t)t / (uint64_t)nthreads;
        a->end = n * (uint64_t)(t + 1) / (uint64_t)nthreads;
        a->stats = slots + (size_t)t * ORC_MAX_TARGETS;
        if (nthreads == 1) worker(a);
        else pthread_create(&th[t], NULL, worker, a);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (stats_sum) {
        /* statistics.go:126-157 sums slots (u64 wrap, overflow only logged) */
        for (int t = 0; t < nthreads; t++)
            for (int k = 0; k < ORC_MAX_TARGETS; k++) {
                const struct orc_stats *s = &slots[(size_t)t * ORC_MAX_TARGETS + k];
                stats_sum[k].allow_packets += s->allow_packets;
                stats_sum[k].allow_bytes += s->allow_bytes;
                stats_sum[k].deny_packets += s->deny_packets;
                stats_sum[k].deny_bytes += s->deny_bytes;
            }
    }
    free(slots); free(th); free(args);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

uint64_t orc_collect_events(const orc_map *m, const uint8_t *frames, const uint64_t *offsets,
                            const uint32_t *caplen, const uint32_t *pkt_len,
                            const uint32_t *ifindex, uint64_t n, struct orc_event *events,
                            uint64_t max_events) {
    uint64_t ne = 0;
    for (uint64_t i = 0; i < n && ne < max_events; i++) {
        uint32_t lin = caplen[i] < pkt_len[i] ? caplen[i] : pkt_len[i];
        uint32_t res;
        int ev;
        orc_xdp_run(m, NULL, frames + offsets[i], lin, pkt_len[i], ifindex[i], &res, &ev);
        if (!ev) continue;
        /* kernel.c:369-373, 393 */
        struct orc_event *e = &events[ne++];
        e->pkt_index = i;
        e->ruleId = GET_RULE_ID(res);
        e->action = GET_ACTION(res);
        e->pad = 0;
        e->pktLength = (uint16_t)pkt_len[i];
        e->ifId = (uint16_t)ifindex[i];
        e->captured = (uint16_t)(pkt_len[i] < MAX_EVENT_DATA ? pkt_len[i] : MAX_EVENT_DATA);
    }
    return ne;
}

/* The perf sample of one DENY event as the reader receives it (perf.Record.RawSample, events.go:64-96):
 * bpf_perf_event_output(ctx, map, BPF_F_CURRENT_CPU | headerSize << 32, &hdr, sizeof(hdr)) (kernel.c:392-399)
 * emits a raw record of two fragments — the 8-B event_hdr_st, then headerSize = min(len, MAX_EVENT_DATA) bytes
 * copied from the start of the XDP frame (bpf_xdp_copy: linear data, then frags) — and the perf core sizes it
 * round_up(8 + headerSize + sizeof(u32), 8) - sizeof(u32), the tail being alignment pad (perf_prepare_sample).
 * out (272 B): u32 raw size, raw bytes, zeros after.  Frame bytes past `linear` (frags, which a snapshot of the
 * linear part does not hold) and the pad are written as zeros.  Returns the raw size. */
uint32_t orc_perf_sample(const uint8_t *frame, uint32_t linear, const struct orc_event *e, uint8_t *out) {
    const uint32_t hs = e->captured, size = ((8u + hs + 4u + 7u) & ~7u) - 4u;
    memset(out, 0, 272);
    memcpy(out, &size, 4);
    memcpy(out + 4, &e->ifId, 2);
    memcpy(out + 6, &e->ruleId, 2);
    out[8] = e->action;
    out[9] = e->pad;
    memcpy(out + 10, &e->pktLength, 2);
    memcpy(out + 12, frame, hs < linear ? hs : linear);
    return size;
}

/* Debug lookup keys (kernel.c:205-216, :291-299): the key each frame would insert
 * into ingress_node_firewall_dbg_map when debug_lookup != 0 — formed after the L4
 * extraction succeeded and before the LPM lookup — in packet order, duplicates
 * included.  keys_out: n_max x 24 B lpm_ip_key_st images. */
uint64_t orc_collect_lookup_keys(const uint8_t *frames, const uint64_t *offsets, const uint32_t *caplen,
                                 const uint32_t *pkt_len, const uint32_t *ifindex, uint64_t n,
                                 uint8_t *keys_out, uint64_t n_max) {
    uint64_t nk = 0;
    for (uint64_t i = 0; i < n && nk < n_max; i++) {
        const uint8_t *data = frames + offsets[i];
        uint32_t lin = caplen[i] < pkt_len[i] ? caplen[i] : pkt_len[i];
        if (ETH_HLEN > lin) continue;                                     /* :423-426 */
        uint16_t h_proto = (uint16_t)(data[12] << 8 | data[13]);
        int v4 = h_proto == 0x0800;
        if (!v4 && h_proto != 0x86DD) continue;                           /* :436-438 */
        uint16_t dstPort = 0;
        uint8_t icmpCode = 0, icmpType = 0, proto = 0;
        if (ip_extract_l4info(data, lin, &proto, &dstPort, &icmpType, &icmpCode, v4) < 0) continue;
        uint8_t *k = keys_out + 24 * nk++;
        memset(k, 0, 24);                                                 /* memset(&key, 0, ...) */
        wr_le32(k, v4 ? 64u : 160u);                                      /* :207 / :293 */
        wr_le32(k + 4, ifindex[i]);
        if (v4) memcpy(k + 8, data + ETH_HLEN + 12, 4);                    /* :208-211 */
        else memcpy(k + 8, data + ETH_HLEN + 8, 16);                       /* :294 */
    }
    return nk;
}
