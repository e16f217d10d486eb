// hostfeed.cpp — the host packer threads of infw_classify_xdp_host (infw_hostfeed.h).
#include "infw_hostfeed.h"

#include <errno.h>
#include <string.h>

#include "../../include/infw_host.h"

#include <sched.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <system_error>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

// The packer's prefetch distance (frames) and store kind (non-temporal or not): build-time knobs for same-box A/Bs
// of two libraries (tools/hostfeed_ab.sh); the shipped library uses the defaults.
#ifndef INFW_PACK_PF
#define INFW_PACK_PF 16
#endif
#ifndef INFW_PACK_NT
#define INFW_PACK_NT 0
#endif

namespace infw {

void Signal::set(uint64_t v) {
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (v <= v_.load(std::memory_order_relaxed)) return;
        v_.store(v, std::memory_order_release);
    }
    cv_.notify_all();
}

void Signal::wait_at_least(uint64_t target) {
    // ~50 us of spinning covers the gap between two chunks of one call; past that the waiter sleeps
    for (int i = 0; i < 4096; i++) {
        if (get() >= target) return;
#if defined(__x86_64__)
        _mm_pause();
#endif
    }
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return get() >= target; });
}

HostPackPool::HostPackPool(int threads) : n_threads_(threads) {
    workers_.reserve(threads);
    for (int t = 0; t < threads; t++) workers_.emplace_back([this] { work(); });
}

HostPackPool::~HostPackPool() {
    quit_.store(true);
    job_.set(gen_ + 1);
    for (auto &w : workers_) w.join();
}

void HostPackPool::begin(const std::vector<XdpChunk> *chunks, const HostFedSrc *src, uint64_t released) {
    // closed_ is set: no worker reads the fields below while they are written
    chunks_ = chunks;
    src_ = src;
    const size_t K = chunks->size();
    unit_base_.assign(K + 1, 0);
    for (size_t k = 0; k < K; k++)
        unit_base_[k + 1] = unit_base_[k] + std::max<uint64_t>(1, ((*chunks)[k].n + kPackUnit - 1) / kPackUnit);
    done_.reset(new std::atomic<uint32_t>[std::max<size_t>(K, 1)]());
    next_unit_.store(0);
    frontier_ = 0;
    abort_.store(false);
    pack_ns_.store(0);
    release_wait_ns_.store(0);
    released_.set(base_ + released);
    closed_.store(false, std::memory_order_seq_cst);  // publishes the job to workers that check it
    if (unit_base_.back() > 2) job_.set(++gen_);        // a call of one or two units wakes no worker
}

void HostPackPool::end(bool abort) {
    if (abort) {
        abort_.store(true);
        released_.set(base_ + chunks_->size());
    }
    closed_.store(true, std::memory_order_seq_cst);
    // a worker inside the job finishes at most the unit it holds; one that arrives now sees closed_ and leaves
    for (int i = 0; active_.load(std::memory_order_seq_cst) != 0; i++) {
        if (i < 4096) {
#if defined(__x86_64__)
            _mm_pause();
#endif
        } else {
            std::this_thread::yield();
        }
    }
    base_ += chunks_->size();
    chunks_ = nullptr;
    src_ = nullptr;
}

void HostPackPool::advance_frontier() {
    std::lock_guard<std::mutex> lk(frontier_mu_);
    const uint64_t K = chunks_->size(), f0 = frontier_;
    while (frontier_ < K &&
           done_[frontier_].load(std::memory_order_acquire) == unit_base_[frontier_ + 1] - unit_base_[frontier_])
        frontier_++;
    if (frontier_ != f0) packed_.set(base_ + frontier_);
}

void HostPackPool::pack_unit(uint64_t u, uint64_t k) {
    const XdpChunk &c = (*chunks_)[k];
    const uint64_t a = std::min(c.n, (u - unit_base_[k]) * kPackUnit), b = std::min(c.n, a + kPackUnit);
    if (a < b && !abort_.load(std::memory_order_relaxed)) pack_chunk_range(c, *src_, a, b);
}

bool HostPackPool::claim_and_pack(bool coordinator) {
    using clk = std::chrono::steady_clock;
    const uint64_t U = unit_base_.back();
    uint64_t u, k;
    auto chunk_of = [&](uint64_t unit) {
        return (uint64_t)(std::upper_bound(unit_base_.begin(), unit_base_.end(), unit) - unit_base_.begin()) - 1;
    };
    auto t0 = clk::now();
    if (coordinator) {  // only units of released chunks: the coordinator is the one that releases
        u = next_unit_.load(std::memory_order_relaxed);
        for (;;) {
            if (u >= U) return false;
            k = chunk_of(u);
            if (base_ + k + 1 > released_.get()) return false;
            if (next_unit_.compare_exchange_weak(u, u + 1, std::memory_order_relaxed)) break;
        }
    } else {
        u = next_unit_.fetch_add(1, std::memory_order_relaxed);
        if (u >= U) return false;
        k = chunk_of(u);
        released_.wait_at_least(base_ + k + 1);
    }
    const auto t1 = clk::now();
    pack_unit(u, k);
    const auto t2 = clk::now();
    release_wait_ns_.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count(),
                               std::memory_order_relaxed);
    pack_ns_.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count(), std::memory_order_relaxed);
    if (done_[k].fetch_add(1, std::memory_order_acq_rel) + 1 == unit_base_[k + 1] - unit_base_[k]) advance_frontier();
    return true;
}

void HostPackPool::help_until_packed(uint64_t k) {
    const uint64_t target = base_ + k + 1;
    while (packed_.get() < target)
        if (!claim_and_pack(true)) {
            packed_.wait_at_least(target);  // the last units are on workers
            return;
        }
}

void HostPackPool::work() {
    uint64_t seen = 0;
    for (;;) {
        job_.wait_at_least(seen + 1);
        seen = job_.get();
        if (quit_.load()) return;
        active_.fetch_add(1, std::memory_order_seq_cst);
        if (!closed_.load(std::memory_order_seq_cst))
            while (claim_and_pack(false)) {
            }
        active_.fetch_sub(1, std::memory_order_seq_cst);
    }
}

void hostpack_burst(const uint8_t *const *frames, const uint32_t *linear_len, const uint32_t *pkt_len, uint64_t n,
                    uint32_t ifindex, const infw_hostpack_out &o) {
    constexpr uint64_t kPF = 16;  // frames ahead (infw_hostpack.h: the headers are DRAM misses)
    uint32_t rank = 0;
    uint32_t *tail = nullptr;
    for (uint64_t i = 0; i < n; i++) {
        if (i + kPF < n) {
            __builtin_prefetch(frames[i + kPF] + 10);
            __builtin_prefetch(frames[i + kPF] + 57);
        }
        if ((i & (INFW_V6_GROUP - 1)) == 0) {
            rank = 0;
            tail = reinterpret_cast<uint32_t *>(o.v6tail + (i / INFW_V6_GROUP) * (12ull * INFW_V6_GROUP));
        }
        const uint8_t *f = frames[i];
        const uint32_t lin = linear_len[i], plen = pkt_len ? pkt_len[i] : lin;
        uint32_t s0, s1, s2, s3, l4, meta;
        if (__builtin_expect(lin >= 58, 1)) {  // every field in place: infw_hostpack_xdp's branch-free form
            const uint32_t et = (uint32_t)f[12] << 8 | f[13];
            const bool v4 = et == 0x0800, v6 = et == 0x86DD;
            const uint32_t ip = (v4 || v6) ? ~0u : 0u;
            const uint32_t proto = f[v6 ? 20 : 23] & ip;
            s0 = infw_ld32(f + (v6 ? 22 : 26)) & ip;
            l4 = infw_ld32(f + (v6 ? 54 : 34)) & ip;
            s1 = infw_ld32(f + 26);
            s2 = infw_ld32(f + 30);
            s3 = infw_ld32(f + 34);
            meta = et | proto << 16 | (lin > 255u ? 255u : lin) << 24;
        } else {
            infw_tuple t;
            infw_pack_header(f, lin, plen, ifindex, &t);
            s0 = t.saddr[0], s1 = t.saddr[1], s2 = t.saddr[2], s3 = t.saddr[3];
            l4 = t.l4word;
            meta = t.meta;
        }
        const bool is6 = (meta & 0xFFFFu) == 0x86DDu;
        tail[3 * rank] = s1, tail[3 * rank + 1] = s2, tail[3 * rank + 2] = s3;
        rank += is6;
        o.saddr4[i] = s0;
        if (o.ifindex) o.ifindex[i] = ifindex;
        o.pkt_len[i] = plen;
        o.meta[i] = meta;
        o.l4word[i] = l4;
    }
}

uint32_t HostFedSrc::at(uint64_t pos) const {
    return (uint32_t)(std::upper_bound(start, start + count + 1, pos) - start) - 1;
}

uint64_t chunk_positions(uint64_t total, uint64_t chunk, bool auto_chunk) {
    if (auto_chunk && total < 4 * chunk)
        return std::min(chunk, std::max<uint64_t>(32768, ((total + 3) / 4 + 4095) & ~4095ull));
    return chunk;
}

namespace {

// Source i's fields; false for a source with flags set or a null array it needs.
inline bool source_fields(const infw_xdp_ring *rings, const infw_frame_burst *bursts, uint32_t i, uint64_t &n,
                          uint32_t &ifx, uint32_t *&res, uint8_t *&ver) {
    if (rings) {
        const infw_xdp_ring &g = rings[i];
        n = g.n, ifx = g.ifindex, res = g.results, ver = g.verdicts;
        return !(g.flags || (g.n && (!g.umem || !g.descs)));
    }
    const infw_frame_burst &g = bursts[i];
    n = g.n, ifx = g.ifindex, res = g.results, ver = g.verdicts;
    return !(g.flags || (g.n && (!g.frames || !g.linear_len)));
}

// A copy appended to a chunk's copies [first, end) of one kind: merged into the last one when the destinations
// continue one another.
inline void append_copy(std::vector<XdpCopy> &v, uint32_t first, uint32_t &end, const XdpCopy &q, uint64_t bytes) {
    if (end > first && v[end - 1].pos + v[end - 1].n == q.pos && v[end - 1].dst + bytes * v[end - 1].n == q.dst) {
        v[end - 1].n += q.n;
        return;
    }
    v.push_back(q);
    end++;
}

// A staged chunk keeps no copies (they are the last ones of their vectors).
inline void seal(XdpChunk &c, std::vector<XdpCopy> &rc, std::vector<XdpCopy> &vc) {
    if (!c.staged) return;
    rc.resize(c.r0), vc.resize(c.v0);
    c.r1 = c.r0, c.v1 = c.v0;
}

// One thread's share of the sources [lo, hi): its pieces of chunks (a chunk's positions this share holds, its copies
// in the share's own vectors), merged in order afterwards.
struct CutPart {
    uint32_t lo = 0, hi = 0;
    uint64_t base = 0, sum = 0;
    bool bad = false;
    std::vector<XdpChunk> pieces;
    std::vector<uint32_t> first_if;  // per piece: its first source's ifindex
    std::vector<XdpCopy> rc, vc;
};

void part_count(CutPart &p, const infw_xdp_ring *rings, const infw_frame_burst *bursts) {
    uint64_t n;
    uint32_t ifx, *res;
    uint8_t *ver;
    for (uint32_t i = p.lo; i < p.hi; i++) {
        if (!source_fields(rings, bursts, i, n, ifx, res, ver)) {
            p.bad = true;
            return;
        }
        p.sum += n;
    }
}

void part_cut(CutPart &p, const infw_xdp_ring *rings, const infw_frame_burst *bursts, uint64_t ce, uint64_t *start) {
    p.pieces.clear(), p.first_if.clear(), p.rc.clear(), p.vc.clear();
    uint64_t pos = p.base, n;
    uint32_t ifx, *res;
    uint8_t *ver;
    for (uint32_t i = p.lo; i < p.hi; i++) {
        (void)source_fields(rings, bursts, i, n, ifx, res, ver);
        start[i] = pos;
        for (uint64_t a = 0; a < n;) {  // the chunks this source's frames fall in (one, for a small burst)
            const uint64_t k = (pos + a) / ce, in = pos + a - k * ce;  // chunk, position in it
            if (p.pieces.empty() || p.pieces.back().begin != k * ce) {
                if (!p.pieces.empty()) seal(p.pieces.back(), p.rc, p.vc);
                const uint32_t r = (uint32_t)p.rc.size(), v = (uint32_t)p.vc.size();
                p.pieces.push_back({k * ce, 0, i, i + 1, false, false, false, false, r, r, v, v, {}});
                p.first_if.push_back(ifx);
            }
            XdpChunk &c = p.pieces.back();
            const uint64_t take = std::min(ce - in, n - a);
            c.mixed |= ifx != p.first_if.back();
            c.src1 = i + 1;
            c.n += take;
            c.any_res |= res != nullptr, c.any_ver |= ver != nullptr;
            if (!c.staged) {
                if (res) append_copy(p.rc, c.r0, c.r1, {in, take, reinterpret_cast<uint8_t *>(res + a)}, 4);
                if (ver) append_copy(p.vc, c.v0, c.v1, {in, take, ver + a}, 1);
                c.staged = (c.r1 - c.r0) + (c.v1 - c.v0) > kXdpMaxCopies;
            }
            a += take;
        }
        pos += n;
    }
    if (!p.pieces.empty()) seal(p.pieces.back(), p.rc, p.vc);
}

// Runs f(t) for t in [0, T): T - 1 helper threads and the calling thread, which also runs the shares of helpers the
// system would not start (the result does not depend on which thread ran a share).
template <class F>
void run_parts(int T, F &&f) {
    std::vector<std::thread> th;
    int started = 1;
    try {
        for (; started < T; started++) th.emplace_back([&f, t = started] { f(t); });
    } catch (const std::system_error &) {
    }
    for (int t = started; t < T; t++) f(t);
    f(0);
    for (auto &x : th) x.join();
}

}  // namespace

int cut_chunks(const infw_xdp_ring *rings, const infw_frame_burst *bursts, uint32_t count, uint64_t chunk,
               bool auto_chunk, int threads, CutPlan &plan) {
    constexpr uint32_t kPerThread = 32768;  // sources per thread below which a helper costs more than it saves
    const int T = (int)std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)std::max(threads, 1), count / kPerThread));
    // the calling thread's shares (their vectors keep their capacity from call to call); the helpers reach them through
    // this reference — a thread_local named inside the lambdas would be each helper's own, empty, instance
    thread_local std::vector<CutPart> tl_parts;
    std::vector<CutPart> &parts = tl_parts;
    parts.resize(T);
    for (int t = 0; t < T; t++) {  // (each share's vectors keep their capacity from call to call)
        parts[t].base = parts[t].sum = 0, parts[t].bad = false;
        parts[t].lo = (uint32_t)((uint64_t)count * t / T), parts[t].hi = (uint32_t)((uint64_t)count * (t + 1) / T);
    }
    run_parts(T, [&](int t) { part_count(parts[t], rings, bursts); });
    uint64_t total = 0;
    for (CutPart &p : parts) {
        if (p.bad) return -EINVAL;
        p.base = total, total += p.sum;
    }
    plan.start.resize((size_t)count + 1);
    plan.start[count] = total;
    plan.src = HostFedSrc{rings, bursts, plan.start.data(), count};
    plan.ce = chunk_positions(total, chunk, auto_chunk);
    run_parts(T, [&](int t) { part_cut(parts[t], rings, bursts, plan.ce, plan.start.data()); });
    // the pieces in order: a chunk shared by two shares is merged (its copies continued, ifindexes compared)
    std::vector<XdpChunk> &chunks = plan.chunks;
    std::vector<XdpCopy> &rc = plan.rcopies, &vc = plan.vcopies;
    chunks.clear(), rc.clear(), vc.clear();
    uint32_t g_first_if = 0;
    for (CutPart &p : parts)
        for (size_t j = 0; j < p.pieces.size(); j++) {
            const XdpChunk &c = p.pieces[j];
            if (chunks.empty() || chunks.back().begin != c.begin) {
                const uint32_t r = (uint32_t)rc.size(), v = (uint32_t)vc.size();
                chunks.push_back({c.begin, 0, c.src0, c.src1, c.mixed, c.staged, c.any_res, c.any_ver, r, r, v, v, {}});
                g_first_if = p.first_if[j];
            } else {
                XdpChunk &g = chunks.back();
                g.mixed |= c.mixed || p.first_if[j] != g_first_if;
                g.src1 = c.src1;
                g.staged |= c.staged;
                g.any_res |= c.any_res, g.any_ver |= c.any_ver;
            }
            XdpChunk &g = chunks.back();
            g.n += c.n;
            if (!g.staged) {
                for (uint32_t q = c.r0; q < c.r1; q++) append_copy(rc, g.r0, g.r1, p.rc[q], 4);
                for (uint32_t q = c.v0; q < c.v1; q++) append_copy(vc, g.v0, g.v1, p.vc[q], 1);
                g.staged = (g.r1 - g.r0) + (g.v1 - g.v0) > kXdpMaxCopies;
            }
            seal(g, rc, vc);
        }
    return 0;
}

void pack_chunk_range(const XdpChunk &c, const HostFedSrc &src, uint64_t a, uint64_t b) {
    constexpr uint64_t G = INFW_V6_GROUP;
    const uint64_t A = c.begin + a, B = c.begin + b;  // call positions
    for (uint32_t i = src.at(A); i < src.count && src.start[i] < B; i++) {
        const uint64_t s0 = std::max(A, src.start[i]), s1 = std::min(B, src.start[i + 1]);
        if (s0 >= s1) continue;  // (an empty source)
        const uint32_t ifx = src.ifindex(i);
        const infw_frame_burst *bu = src.bursts ? &src.bursts[i] : nullptr;
        if (bu && i + 1 < src.count && s1 == src.start[i + 1]) {
            // a burst's first frames are not prefetched by its own loop (which runs 16 frames ahead of itself): issue
            // the next burst's while this one packs, so rx_burst-sized bursts keep as many misses in flight
            const infw_frame_burst &nx = src.bursts[i + 1];
            for (uint64_t q = 0, m = std::min<uint64_t>(nx.n, 16); q < m; q++) {
                __builtin_prefetch(nx.frames[q] + 10);
                __builtin_prefetch(nx.frames[q] + 57);
            }
        }
        for (uint64_t p = s0 - c.begin, e1 = s1 - c.begin; p < e1;) {  // chunk positions
            const uint64_t g0 = p & ~(G - 1);
            uint32_t rank = 0;  // IPv6 packets an earlier source put into this group: they hold its first tail slots
            uint64_t e = e1;
            if (p != g0) {  // (the same thread packed them: units start on group boundaries)
                for (uint64_t q = g0; q < p; q++) rank += (c.out.meta[q] & 0xFFFFu) == 0x86DDu;
                e = std::min(e1, g0 + G);  // up to the group's end, so the packer's group boundaries stay aligned
            }
            const infw_hostpack_out o{c.out.saddr4 + p, c.out.v6tail + g0 / G * (12 * G) + 12 * rank,
                                      c.mixed ? c.out.ifindex + p : nullptr, c.out.pkt_len + p, c.out.meta + p,
                                      c.out.l4word + p};
            const uint64_t off = c.begin + p - src.start[i];  // the source's frame / descriptor index
            if (bu)
                hostpack_burst(bu->frames + off, bu->linear_len + off, bu->pkt_len ? bu->pkt_len + off : nullptr, e - p,
                               ifx, o);
            else
                infw_hostpack_xdp<INFW_PACK_PF, INFW_PACK_NT != 0>(src.rings[i].umem, src.rings[i].descs + off, e - p,
                                                                   ifx, o);
            p = e;
        }
    }
}

int host_threads_auto() {
    int n = 0;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
    if (n <= 0) n = (int)std::thread::hardware_concurrency();
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {  // cgroup v2 "quota period" (or "max period")
        long long quota = 0, period = 0;
        if (fscanf(f, "%lld %lld", &quota, &period) == 2 && quota > 0 && period > 0)
            n = std::min<int>(n, (int)((quota + period - 1) / period));
        fclose(f);
    }
    return std::max(1, std::min(n, 16));
}

}  // namespace infw

extern "C" int infw_xdp_host_events(const uint8_t *umem, const struct infw_xdp_desc *descs, uint64_t n,
                                    uint32_t ifindex, const uint32_t *results, struct infw_event_sample *samples,
                                    uint64_t cap, uint64_t *count);

// Shared by the two event builders: sample k of a denied packet (kernel.c:392-399, infw_events_capture's layout).
static void infw_fill_sample(infw_event_sample &s, const uint8_t *f, uint32_t linear, uint32_t plen, uint32_t ifindex,
                             uint32_t r) {
    const uint32_t captured = plen < INFW_MAX_EVENT_DATA ? plen : INFW_MAX_EVENT_DATA;
    s.size = ((8u + captured + 4u + 7u) & ~7u) - 4u;
    memset(s.raw, 0, sizeof s.raw);
    event_hdr_st h{};
    h.ifId = (uint16_t)ifindex;
    h.ruleId = (uint16_t)(r >> 8);
    h.action = INFW_XDP_DROP;
    h.pktLength = (uint16_t)plen;
    memcpy(s.raw, &h, sizeof h);
    memcpy(s.raw + sizeof h, f, captured < linear ? captured : linear);  // past the linear part: zeros
}

extern "C" int infw_burst_host_events(const struct infw_frame_burst *b, const uint32_t *results,
                                      struct infw_event_sample *samples, uint64_t cap, uint64_t *count) {
    if (!b || !count || (b->n && (!b->frames || !b->linear_len || !results)) || (cap && !samples)) return -EINVAL;
    uint64_t k = 0;
    for (uint64_t i = 0; i < b->n; i++) {
        if ((results[i] & 0xFFu) != INFW_XDP_DROP) continue;
        if (k < cap)
            infw_fill_sample(samples[k], b->frames[i], b->linear_len[i], b->pkt_len ? b->pkt_len[i] : b->linear_len[i],
                             b->ifindex, results[i]);
        k++;
    }
    *count = k;
    return 0;
}

extern "C" int infw_pack_burst_host(const struct infw_frame_burst *b, const struct infw_batch_soa_c_out *out) {
    if (!b || !out) return -EINVAL;
    if (b->n == 0) return 0;
    bool ok = b->frames && b->linear_len && out->saddr4 && out->v6tail && out->pkt_len && out->meta && out->l4word;
    for (const void *q : {(const void *)out->saddr4, (const void *)out->v6tail, (const void *)out->ifindex,
                          (const void *)out->pkt_len, (const void *)out->meta, (const void *)out->l4word})
        ok = ok && ((uintptr_t)q & 3) == 0;
    if (!ok) return -EINVAL;
    infw::hostpack_burst(b->frames, b->linear_len, b->pkt_len, b->n, b->ifindex,
                         {out->saddr4, out->v6tail, out->ifindex, out->pkt_len, out->meta, out->l4word});
    return 0;
}

extern "C" int infw_xdp_host_events(const uint8_t *umem, const struct infw_xdp_desc *descs, uint64_t n,
                                    uint32_t ifindex, const uint32_t *results, struct infw_event_sample *samples,
                                    uint64_t cap, uint64_t *count) {
    if (!count || (n && (!umem || !descs || !results)) || (cap && !samples)) return -EINVAL;
    uint64_t k = 0;
    for (uint64_t i = 0; i < n; i++) {
        if ((results[i] & 0xFFu) != INFW_XDP_DROP) continue;
        if (k < cap)  // a single-buffer AF_XDP frame: linear = frame length = the descriptor's len
            infw_fill_sample(samples[k], infw_xdp_frame(umem, descs[i].addr), descs[i].len, descs[i].len, ifindex,
                             results[i]);
        k++;
    }
    *count = k;
    return 0;
}
