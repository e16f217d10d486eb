// workload.hip — synthetic tables and packets for BASELINE.json configs
// (SURVEY.md §8d).  Bench / test infrastructure: libinfw_workload.so.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "workload.h"

struct infw_wl {
    int cfg = 0;
    std::vector<lpm_ip_key_st> keys;
    std::vector<uint32_t> val_index;
    std::vector<rulesVal_st> templates;
    std::vector<infw_gen_prefix> prefixes;  // popularity rank order
    std::vector<uint64_t> cdf;
    infw_gen_params params{};
    // device copies
    int dev = -1;
    infw_gen_prefix *d_prefixes = nullptr;
    uint64_t *d_cdf = nullptr;
};

namespace {

struct Rng {  // host-side sequential generator for tables (splitmix64)
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() { return infw_mix64(s += 0x9E3779B97F4A7C15ull); }
    uint32_t below(uint32_t n) { return infw_below(next(), n); }
    bool chance(uint32_t permille) { return below(1000) < permille; }
};

void set_rule(ruleType_st &r, uint32_t id, uint8_t proto, uint16_t ps, uint16_t pe, uint8_t it,
              uint8_t ic, uint8_t action) {
    r.ruleId = id;
    r.protocol = proto;
    r.dstPortStart = ps;
    r.dstPortEnd = pe;
    r.icmpType = it;
    r.icmpCode = ic;
    r.action = action;
}

const uint16_t kServicePorts[16] = {22, 53, 80, 123, 179, 443, 2049, 3306, 5432, 6379, 6443, 8000, 8080, 8443, 9100, 12345};
const uint16_t kIcmpTc[8] = {0x0000, 0x0301, 0x0800, 0x0B00, 0x8000, 0x8100, 0x8700, 0x8800};

// A random transport/ICMP rule at slot `order` drawn from the service-port pool.
void random_rule(Rng &g, ruleType_st &r, uint32_t order) {
    uint32_t k = g.below(100);
    uint8_t act = g.chance(500) ? INFW_XDP_PASS : INFW_XDP_DROP;
    if (k < 82) {
        uint8_t proto = k < 34 ? 6 : k < 64 ? 17 : 132;
        uint16_t base = g.chance(600) ? kServicePorts[g.below(16)] : (uint16_t)(1 + g.below(65534));
        if (g.chance(500)) set_rule(r, order, proto, base, 0, 0, 0, act);  // exact port
        else {
            uint32_t end = (uint32_t)base + 1 + g.below(64);
            if (end > 65535) end = 65535;
            set_rule(r, order, proto, base, (uint16_t)end, 0, 0, act);       // end-exclusive range
        }
    } else {
        uint16_t tc = kIcmpTc[g.below(8)];
        set_rule(r, order, k < 91 ? 1 : 58, 0, 0, (uint8_t)(tc >> 8), (uint8_t)tc, act);
    }
}

void common_mix(infw_gen_params &p) {
    p.p_tcp = 600;
    p.p_udp = 250;
    p.p_icmp = 100;
    p.p_sctp = 30;  // remaining 20: GRE (unsupported -> UNDEF)
    p.n_icmp = 8;
    for (int i = 0; i < 8; i++) p.icmp_tc[i] = kIcmpTc[i];
    p.len_min = 54;
    p.len_max = 1514;
    p.p_nonip = 5;
    p.p_trunc = 5;
}

void push_prefix(infw_wl &w, uint32_t ifx, const uint8_t *addr, uint32_t plen_bits, int fam) {
    infw_gen_prefix gp;
    memset(&gp, 0, sizeof(gp));
    memcpy(gp.addr, addr, fam == 4 ? 4 : 16);
    gp.ifindex = ifx;
    gp.plen = (uint8_t)plen_bits;
    gp.family = (uint8_t)fam;
    w.prefixes.push_back(gp);
    lpm_ip_key_st k;
    memset(&k, 0, sizeof(k));
    k.prefixLen = plen_bits + 32;
    k.ingress_ifindex = ifx;
    memcpy(k.ip_data, addr, fam == 4 ? 4 : 16);
    w.keys.push_back(k);
}

void random_addr(Rng &g, uint8_t *a, int fam) {
    uint64_t x = g.next(), y = g.next();
    memcpy(a, &x, 8);
    memcpy(a + 8, &y, 8);
    if (fam == 6) a[0] = (uint8_t)(0x20 | (a[0] & 0x1F));  // 2000::/3
}

void zipf_cdf(std::vector<uint64_t> &cdf, uint32_t n, double s) {
    cdf.resize(n);
    long double H = 0;
    for (uint32_t k = 1; k <= n; k++) H += 1.0L / powl((long double)k, (long double)s);
    long double cum = 0;
    for (uint32_t k = 1; k <= n; k++) {
        cum += 1.0L / powl((long double)k, (long double)s);
        long double f = cum / H * 18446744073709551616.0L;
        cdf[k - 1] = f >= 18446744073709551615.0L ? ~0ull : (uint64_t)f;
    }
    cdf[n - 1] = ~0ull;
}

void build_cfg0(infw_wl &w) {
    // config/samples/ingressnodefirewall-demo-1.yaml:12-27 (ingress[0]) on ifindex 1
    rulesVal_st v;
    memset(&v, 0, sizeof(v));
    set_rule(v.rules[10], 10, 6, 100, 200, 0, 0, INFW_XDP_PASS);
    set_rule(v.rules[20], 20, 17, 8000, 0, 0, 0, INFW_XDP_PASS);
    w.templates.push_back(v);
    const uint8_t a4[4] = {1, 1, 1, 1};
    uint8_t a6[16] = {0x01, 0x00, 0x00, 0x01};
    a6[15] = 1;
    push_prefix(w, 1, a4, 24, 4);
    push_prefix(w, 1, a6, 64, 6);
    w.val_index.assign(2, 0);
    infw_gen_params &p = w.params;
    common_mix(p);
    p.hit_permille = 700;
    p.v6_permille = 500;
    p.p_special = 500;
    const uint16_t sp[10] = {99, 100, 101, 150, 199, 200, 201, 7999, 8000, 8001};
    p.n_special = 10;
    for (int i = 0; i < 10; i++) p.special_ports[i] = sp[i];
    p.n_ifindex = 2;
    p.ifindexes[0] = 1;
    p.ifindexes[1] = 2;
}

void build_cfg1(infw_wl &w, Rng &g, uint32_t n) {
    w.templates.resize(n);
    w.val_index.resize(n);
    for (uint32_t i = 0; i < n; i++) {
        rulesVal_st &v = w.templates[i];
        memset(&v, 0, sizeof(v));
        for (uint32_t o = 1; o <= 9; o++) random_rule(g, v.rules[o], o);
        set_rule(v.rules[10], 10, 0, 0, 0, 0, 0, INFW_XDP_DROP);  // catch-all Deny
        w.val_index[i] = i;
        uint8_t a[16];
        random_addr(g, a, 4);
        push_prefix(w, 1, a, 16 + g.below(17), 4);
    }
    infw_gen_params &p = w.params;
    common_mix(p);
    p.hit_permille = 900;
    p.v6_permille = 0;
    p.p_special = 500;
    p.n_special = 16;
    for (int i = 0; i < 16; i++) p.special_ports[i] = kServicePorts[i];
    p.n_ifindex = 1;
    p.ifindexes[0] = 1;
}

uint32_t v4_len_bgp(Rng &g) {
    uint32_t r = g.below(100);
    if (r < 60) return 24;
    if (r < 75) return 22 + g.below(2);
    if (r < 90) return 16 + g.below(6);
    return 25 + g.below(8);
}
uint32_t v6_len_mix(Rng &g) {
    uint32_t r = g.below(100);
    if (r < 45) return 48;
    if (r < 80) return 32 + g.below(13);
    if (r < 95) return 56 + g.below(9);
    return 128;
}

void build_cfg2(infw_wl &w, Rng &g, uint32_t n, uint32_t n_tmpl) {
    w.templates.resize(n_tmpl);
    for (uint32_t t = 0; t < n_tmpl; t++) {
        rulesVal_st &v = w.templates[t];
        memset(&v, 0, sizeof(v));
        for (uint32_t o = 1; o <= 98; o++) random_rule(g, v.rules[o], o);
        set_rule(v.rules[99], 99, 0, 0, 0, 0, 0, (t & 1) ? INFW_XDP_PASS : INFW_XDP_DROP);
    }
    const uint32_t ifx[4] = {2, 3, 4, 5};
    w.val_index.resize(n);
    for (uint32_t i = 0; i < n; i++) {
        int fam = g.chance(600) ? 4 : 6;
        uint8_t a[16];
        random_addr(g, a, fam);
        uint32_t len = fam == 4 ? v4_len_bgp(g) : v6_len_mix(g);
        push_prefix(w, ifx[g.below(4)], a, len, fam);
        const uint32_t t = g.below(n_tmpl);
        // distinct-lists variant (n_templates >= n_prefixes): every key carries its own 1200-B value, as
        // makeIngressFwRulesMap produces one value per key (loader.go:158-161) — no interning in the workload
        w.val_index[i] = n_tmpl >= n ? i : t;
    }
    zipf_cdf(w.cdf, n, 1.1);
    infw_gen_params &p = w.params;
    common_mix(p);
    p.hit_permille = 950;
    p.v6_permille = 400;
    p.p_special = 500;
    p.n_special = 16;
    for (int i = 0; i < 16; i++) p.special_ports[i] = kServicePorts[i];
    p.n_ifindex = 4;
    for (int i = 0; i < 4; i++) p.ifindexes[i] = ifx[i];
}

void build_cfg4(infw_wl &w, Rng &g, uint32_t n, uint32_t n_tmpl) {
    // every list: 98 rules no adversarial packet matches, last slot ICMPv6 128/0
    w.templates.resize(n_tmpl);
    for (uint32_t t = 0; t < n_tmpl; t++) {
        rulesVal_st &v = w.templates[t];
        memset(&v, 0, sizeof(v));
        for (uint32_t o = 1; o <= 98; o++) {
            uint32_t k = g.below(4);
            uint8_t act = (o & 1) ? INFW_XDP_PASS : INFW_XDP_DROP;
            if (k == 0) set_rule(v.rules[o], o, 58, 0, 0, 128, (uint8_t)(2 + g.below(200)), act);  // wrong code
            else if (k == 1) set_rule(v.rules[o], o, 58, 0, 0, (uint8_t)(130 + g.below(100)), 0, act);
            else if (k == 2) set_rule(v.rules[o], o, 1, 0, 0, 128, 0, act);  // ICMP on the v6 path: ignored
            else set_rule(v.rules[o], o, 6, (uint16_t)(1 + g.below(1000)), 0, 0, 0, act);
        }
        set_rule(v.rules[99], 99, 58, 0, 0, 128, 0, (t & 1) ? INFW_XDP_PASS : INFW_XDP_DROP);
    }
    const uint32_t ifx[2] = {7, 8};
    w.val_index.clear();
    uint32_t n_alias = n / 50;
    for (uint32_t i = 0; i < n; i++) {
        uint8_t a[16];
        uint32_t r = g.below(100);
        int fam;
        uint32_t len;
        if (r < 50) { fam = 6; len = 128; }              // deepest-prefix hits
        else if (r < 80) { fam = 6; len = 48 + g.below(17); }
        else { fam = 4; len = 16 + g.below(17); }
        random_addr(g, a, fam);
        push_prefix(w, ifx[g.below(2)], a, len, fam);
        w.val_index.push_back(g.below(n_tmpl));
        // a covering /64 below every /128 so the long search has to go deep
        if (len == 128 && g.chance(500)) {
            push_prefix(w, w.prefixes.back().ifindex, a, 64, 6);
            w.val_index.push_back(g.below(n_tmpl));
        }
    }
    // cross-family aliasing: an IPv6 /16 with the bits of an IPv4 /16 (same key)
    for (uint32_t i = 0; i < n_alias; i++) {
        uint8_t a[16];
        random_addr(g, a, 4);
        push_prefix(w, ifx[i & 1], a, 16, 4);
        w.val_index.push_back(g.below(n_tmpl));
        uint8_t b[16] = {0};
        b[0] = a[0];
        b[1] = a[1];
        push_prefix(w, ifx[i & 1], b, 16, 6);
        w.val_index.push_back(g.below(n_tmpl));
    }
    // identical-key IPv4 0.0.0.0/0 and IPv6 ::/0 on one interface: last writer wins
    uint8_t z[16] = {0};
    push_prefix(w, ifx[0], z, 0, 4);
    w.val_index.push_back(0);
    push_prefix(w, ifx[0], z, 0, 6);
    w.val_index.push_back(1 % n_tmpl);
    infw_gen_params &p = w.params;
    common_mix(p);
    p.p_tcp = 200;
    p.p_udp = 100;
    p.p_icmp = 650;
    p.p_sctp = 30;
    p.n_icmp = 3;
    p.icmp_tc[0] = 0x8000;  // 128/0 matches the last slot
    p.icmp_tc[1] = 0x8100;  // 129/0 falls through
    p.icmp_tc[2] = 0x8001;  // 128/1 falls through
    p.hit_permille = 900;
    p.v6_permille = 700;
    p.cross_permille = 100;
    p.p_special = 0;
    p.n_ifindex = 2;
    p.ifindexes[0] = ifx[0];
    p.ifindexes[1] = ifx[1];
}

template <class F>
void parallel_for(uint64_t n, int nthreads, F f) {
    if (nthreads <= 1 || n < 4096) {
        f(0, n);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; t++) {
        uint64_t b = n * (uint64_t)t / (uint64_t)nthreads, e = n * (uint64_t)(t + 1) / (uint64_t)nthreads;
        th.emplace_back([=] { f(b, e); });
    }
    for (auto &x : th) x.join();
}

__global__ void gen_soa_kernel(infw_gen_params p, uint64_t start, uint64_t n, uint4 *saddr,
                               uint32_t *ifindex, uint32_t *pkt_len, uint32_t *meta, uint32_t *l4word) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        infw_tuple t;
        infw_gen_tuple(&p, start + i, &t);
        saddr[i] = make_uint4(t.saddr[0], t.saddr[1], t.saddr[2], t.saddr[3]);
        ifindex[i] = t.ifindex;
        pkt_len[i] = t.pkt_len;
        meta[i] = t.meta;
        l4word[i] = t.l4word;
    }
}

// Frames of packets [start, start+n) at a fixed stride (AF_XDP-style chunks): the 80-B header snapshot of the
// host frame builder, the linear length of the snapshot's valid bytes, the frame length, the ifindex.
__global__ void gen_frames_kernel(infw_gen_params p, uint64_t start, uint64_t n, uint8_t *frames, uint64_t stride,
                                  uint32_t *linear_len, uint32_t *pkt_len, uint32_t *ifindex) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t h[INFW_HDR_SNAP / 4];
        uint32_t cap, plen, ifx;
        infw_gen_header(&p, start + i, reinterpret_cast<uint8_t *>(h), &cap, &plen, &ifx);
        uint32_t *f = reinterpret_cast<uint32_t *>(frames + i * stride);
        for (int k = 0; k < INFW_HDR_SNAP / 4; k++) f[k] = h[k];
        linear_len[i] = cap < INFW_HDR_SNAP ? cap : INFW_HDR_SNAP;
        pkt_len[i] = plen;
        ifindex[i] = ifx;
    }
}

// ---- random-line and stream rates of the device, measured inside the bench's own process just before its timed
// loop (bench.py random_line_model; tools/micro/gather.hip is the standalone microbenchmark they come from): the
// rate of independent random 16-B lookups that hit the L2 (a 1-MiB table), of ones that miss it (a 2-GiB table:
// every lookup a distinct line beyond the XCD L2s and the 256-MB Infinity Cache), and the read bandwidth of a
// coalesced stream of 16-B non-temporal loads (the tuple stream's access pattern) over the same 2 GiB.
typedef unsigned int lr_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t lr_mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    return x ^ (x >> 16);
}
__global__ __launch_bounds__(512) void lr_gather(const lr_u32x4 *__restrict__ tab, uint32_t mask, int iters,
                                                 uint32_t *__restrict__ out) {
    const uint32_t tid = blockIdx.x * 512 + threadIdx.x;
    uint32_t acc = 0;
    const uint32_t idx = lr_mix(tid);
    for (int it = 0; it < iters; it++) {
        const lr_u32x4 v = tab[lr_mix(idx + (uint32_t)it * 0x9E3779B9u) & mask];
        acc += v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    out[tid] = acc;
}
__global__ __launch_bounds__(512) void lr_stream(const lr_u32x4 *__restrict__ buf, uint64_t n16, uint32_t *__restrict__ out) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 512 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 512) {
        const lr_u32x4 v = __builtin_nontemporal_load(buf + i);
        acc += v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    out[blockIdx.x * 512 + threadIdx.x] = acc;
}

}  // namespace

extern "C" {

// out[0] L2-hit lookups G/s, out[1] L2-miss lookups G/s, out[2] streamed read GB/s (device `dev`; ~0.3 s, 2 GiB of
// scratch freed before returning).
int infw_wl_line_rates(int dev, double *out) {
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (!out || hipSetDevice(dev) != hipSuccess) return -ENODEV;
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint32_t grid = (uint32_t)(cus > 0 ? cus : 256) * 4;  // gathers: grid blocks, the stream: 2 * grid blocks
    const uint64_t big = 2ull << 30;
    const size_t sink_words = (size_t)2 * grid * 512;            // one word per thread of the largest launch
    lr_u32x4 *tab = nullptr;
    uint32_t *sink = nullptr;
    hipEvent_t a = nullptr, b = nullptr;
    int rc = 0;
    if (hipMalloc(&tab, big) != hipSuccess || hipMalloc(&sink, sink_words * 4) != hipSuccess ||
        hipMemset(tab, 1, big) != hipSuccess || hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
        rc = -ENOMEM;
        (void)hipGetLastError();  // the failed allocation's sticky error must not surface in the caller's next check
    }
    auto timed = [&](auto launch, int reps) -> double {  // ms per launch after one untimed launch
        launch();
        (void)hipEventRecord(a, 0);
        for (int r = 0; r < reps; r++) launch();
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, a, b);
        return ms / reps;
    };
    const int iters = 64;
    if (!rc) {
        const double lookups = (double)grid * 512 * iters;
        const double hit_ms = timed([&] { lr_gather<<<grid, 512>>>(tab, (1u << 20) / 16 - 1, iters, sink); }, 10);
        const double miss_ms = timed([&] { lr_gather<<<grid, 512>>>(tab, (uint32_t)(big / 16 - 1), iters, sink); }, 5);
        const double st_ms = timed([&] { lr_stream<<<grid * 2, 512>>>(tab, big / 16, sink); }, 5);
        out[0] = lookups / (hit_ms * 1e-3) / 1e9;
        out[1] = lookups / (miss_ms * 1e-3) / 1e9;
        out[2] = (double)big / (st_ms * 1e-3) / 1e9;
        if (hipGetLastError() != hipSuccess) rc = -EIO;
    }
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
    if (tab) (void)hipFree(tab);
    if (sink) (void)hipFree(sink);
    (void)hipSetDevice(prev);
    return rc;
}

int infw_wl_create(infw_wl **out, int cfg, uint64_t seed, uint32_t n_prefixes, uint32_t n_templates) {
    if (!out) return -EINVAL;
    infw_wl *w = new infw_wl();
    w->cfg = cfg;
    Rng g(seed ^ 0x7AB1E5ull);
    switch (cfg) {
    case INFW_WL_CFG0_DEMO: build_cfg0(*w); break;
    case INFW_WL_CFG1_V4_10K: build_cfg1(*w, g, n_prefixes ? n_prefixes : 10000); break;
    case INFW_WL_CFG2_MIXED_1M:
        build_cfg2(*w, g, n_prefixes ? n_prefixes : 1000000, n_templates ? n_templates : 4096);
        break;
    case INFW_WL_CFG4_ADVERSARIAL:
        build_cfg4(*w, g, n_prefixes ? n_prefixes : 100000, n_templates ? n_templates : 256);
        break;
    default:
        delete w;
        return -EINVAL;
    }
    w->params.seed = seed;
    w->params.prefixes = w->prefixes.data();
    w->params.n_prefixes = (uint32_t)w->prefixes.size();
    w->params.zipf_cdf = w->cdf.empty() ? nullptr : w->cdf.data();
    *out = w;
    return 0;
}

void infw_wl_destroy(infw_wl *w) {
    if (!w) return;
    if (w->dev >= 0) {
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(w->dev);
        if (w->d_prefixes) (void)hipFree(w->d_prefixes);
        if (w->d_cdf) (void)hipFree(w->d_cdf);
        (void)hipSetDevice(prev);
    }
    delete w;
}

void infw_wl_uniform_sources(infw_wl *w) {
    if (w->d_cdf) {
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(w->dev);
        (void)hipFree(w->d_cdf);
        (void)hipSetDevice(prev);
        w->d_cdf = nullptr;
    }
    w->cdf.clear();
    w->params.zipf_cdf = nullptr;
}

uint64_t infw_wl_n_entries(const infw_wl *w) { return w->keys.size(); }
const lpm_ip_key_st *infw_wl_keys(const infw_wl *w) { return w->keys.data(); }
const uint32_t *infw_wl_val_index(const infw_wl *w) { return w->val_index.data(); }
uint32_t infw_wl_n_templates(const infw_wl *w) { return (uint32_t)w->templates.size(); }
const rulesVal_st *infw_wl_templates(const infw_wl *w) { return w->templates.data(); }
const infw_gen_params *infw_wl_params(const infw_wl *w) { return &w->params; }
void infw_wl_set_packet_seed(infw_wl *w, uint64_t seed) { w->params.seed = seed; }

int infw_wl_frames(const infw_wl *w, uint64_t start, uint64_t n, uint8_t *hdr, uint32_t *caplen,
                   uint32_t *pkt_len, uint32_t *ifindex, int nthreads) {
    const infw_gen_params p = w->params;
    parallel_for(n, nthreads, [&](uint64_t b, uint64_t e) {
        for (uint64_t i = b; i < e; i++)
            infw_gen_header(&p, start + i, hdr + i * INFW_HDR_SNAP, &caplen[i], &pkt_len[i], &ifindex[i]);
    });
    return 0;
}

int infw_wl_tuples(const infw_wl *w, uint64_t start, uint64_t n, uint32_t *tuples, int nthreads) {
    const infw_gen_params p = w->params;
    parallel_for(n, nthreads, [&](uint64_t b, uint64_t e) {
        for (uint64_t i = b; i < e; i++) infw_gen_tuple(&p, start + i, reinterpret_cast<infw_tuple *>(tuples + 8 * i));
    });
    return 0;
}

int infw_wl_pack(const uint8_t *hdr, const uint32_t *caplen, const uint32_t *pkt_len,
                 const uint32_t *ifindex, uint64_t n, uint32_t *tuples) {
    for (uint64_t i = 0; i < n; i++)
        infw_pack_header(hdr + i * INFW_HDR_SNAP, caplen[i], pkt_len[i], ifindex[i],
                         reinterpret_cast<infw_tuple *>(tuples + 8 * i));
    return 0;
}

int infw_wl_upload(infw_wl *w, int dev) {
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(dev) != hipSuccess) return -ENODEV;
    int rc = 0;
    if (hipMalloc(&w->d_prefixes, std::max<size_t>(1, w->prefixes.size()) * sizeof(infw_gen_prefix)) != hipSuccess ||
        hipMemcpy(w->d_prefixes, w->prefixes.data(), w->prefixes.size() * sizeof(infw_gen_prefix),
                  hipMemcpyHostToDevice) != hipSuccess)
        rc = -EIO;
    if (!rc && !w->cdf.empty() &&
        (hipMalloc(&w->d_cdf, w->cdf.size() * sizeof(uint64_t)) != hipSuccess ||
         hipMemcpy(w->d_cdf, w->cdf.data(), w->cdf.size() * sizeof(uint64_t), hipMemcpyHostToDevice) != hipSuccess))
        rc = -EIO;
    w->dev = dev;
    (void)hipSetDevice(prev);
    return rc;
}

int infw_wl_gen_soa(infw_wl *w, uint64_t start, uint64_t n, uint8_t *saddr, uint32_t *ifindex,
                    uint32_t *pkt_len, uint32_t *meta, uint32_t *l4word, void *stream) {
    if (w->dev < 0) return -ENODEV;
    if (n == 0) return 0;
    infw_gen_params p = w->params;
    p.prefixes = w->d_prefixes;
    p.zipf_cdf = w->cdf.empty() ? nullptr : w->d_cdf;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(gen_soa_kernel, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, p, start, n,
                       reinterpret_cast<uint4 *>(saddr), ifindex, pkt_len, meta, l4word);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int infw_wl_gen_frames(infw_wl *w, uint64_t start, uint64_t n, uint8_t *frames, uint64_t stride,
                       uint32_t *linear_len, uint32_t *pkt_len, uint32_t *ifindex, void *stream) {
    if (w->dev < 0) return -ENODEV;
    if (n == 0) return 0;
    if (stride < INFW_HDR_SNAP || (stride & 3) || ((uintptr_t)frames & 3)) return -EINVAL;
    infw_gen_params p = w->params;
    p.prefixes = w->d_prefixes;
    p.zipf_cdf = w->cdf.empty() ? nullptr : w->d_cdf;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(gen_frames_kernel, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, p, start, n,
                       frames, stride, linear_len, pkt_len, ifindex);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

}  // extern "C"
