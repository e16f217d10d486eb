// abi.cpp — libinfw C ABI (include/infw.h): context, pending table map,
// epoch commit + upload, classify dispatch, statistics slots.
#include <errno.h>
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <memory>
#include <array>
#include <mutex>
#include <set>
#include <thread>
#include <algorithm>

#include "infw_internal.h"

extern "C" int infw_launch_classify_frames(const infw_dev_tables *T, const infw_frame_batch *fb, uint64_t n,
                                           uint32_t *results, uint8_t *verdicts, uint64_t *stats, uint32_t cus,
                                           hipStream_t stream, infw_event_rec *ev, uint64_t ev_cap, uint64_t *ev_count,
                                           uint64_t *dbg_fp, uint32_t *dbg_keys, uint32_t *dbg_count,
                                           uint32_t dbg_slots);
extern "C" int infw_launch_classify(const infw_dev_tables *T, const infw_batch_soa *in, uint64_t n,
                                    uint32_t *results, uint8_t *verdicts, uint64_t *stats, uint32_t cus,
                                    int block, int group, int blocks_per_cu, hipStream_t stream,
                                    infw_event_rec *ev, uint64_t ev_cap, uint64_t *ev_count,
                                    uint64_t *dbg_fp, uint32_t *dbg_keys, uint32_t *dbg_count, uint32_t dbg_slots,
                                    const infw_batch_soa_c *in_c);
extern "C" int infw_launch_soa_compact(const infw_batch_soa *in, uint64_t n, uint32_t *saddr4, uint8_t *v6tail,
                                       uint32_t cus, hipStream_t stream);

extern "C" int infw_launch_scatter(const uint32_t *staging, const void *descs, uint32_t n, uint32_t cus,
                                   hipStream_t stream);

struct infw_patch_desc {  // patch.hip
    uint64_t dst, src, nwords;
};

extern "C" int infw_launch_pack_frames(const infw_frame_batch *fb, uint64_t n, const infw_batch_soa_out *out,
                                       const infw_batch_soa_c_out *out_c, uint32_t cus, hipStream_t stream);

extern "C" int infw_launch_event_samples(const infw_frame_batch *fb, const infw_event_rec *ev, uint64_t cap,
                                         const uint64_t *count, uint64_t n_frames, infw_event_sample *samples,
                                         uint32_t cus, hipStream_t stream);

namespace infw {

static thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }

#define HIP_OK(expr)                                                             \
    do {                                                                         \
        hipError_t e_ = (expr);                                                  \
        if (e_ != hipSuccess) {                                                  \
            set_error(std::string(#expr) + ": " + hipGetErrorString(e_));       \
            return -EIO;                                                         \
        }                                                                        \
    } while (0)

// Restores the caller's current HIP device (callers such as torch keep their own).
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// One table image resident on one device.  Buffers are allocated with room to
// grow (appended rule lists and tbl8 groups), so an incremental commit can
// patch an image in place; `pending` holds the host ranges changed since the
// image was last brought up to date.
struct DeviceEpoch {
    int ordinal = -1;
    void *buf[TB_COUNT] = {};
    size_t cap[TB_COUNT] = {};
    infw_dev_tables view;
    uint64_t bytes = 0;
    std::vector<DirtyRange> pending;
    // The last classify launch on this image per stream.  An incremental commit orders its
    // upload into this image (while it is the spare) after exactly these launches — on the
    // device, through its patch stream — and records `ready` behind the upload; launches on
    // the image once it is live wait for `ready` in their own stream.  Neither the host nor
    // the batch running on the live image waits for the other.
    std::mutex use_mu;
    std::vector<std::pair<hipStream_t, hipEvent_t>> uses;
    bool use_overflow = false;  // more streams than tracked: the host waits for the device instead
    hipEvent_t ready = nullptr;
    bool ready_armed = false;
    void mark_use(hipStream_t s) {
        std::lock_guard<std::mutex> lk(use_mu);
        hipEvent_t ev = nullptr;
        for (auto &u : uses)
            if (u.first == s) ev = u.second;
        if (!ev) {
            if (uses.size() >= 32 || hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
                use_overflow = true;
                return;
            }
            uses.emplace_back(s, ev);
        }
        if (hipEventRecord(ev, s) != hipSuccess) use_overflow = true;
    }
    // make stream `ps` wait for every launch that read this image
    int order_after_uses(hipStream_t ps) {
        std::lock_guard<std::mutex> lk(use_mu);
        DeviceGuard g(ordinal);
        if (use_overflow) {
            use_overflow = false;
            return hipDeviceSynchronize() == hipSuccess ? 0 : -EIO;
        }
        for (auto &u : uses)
            if (hipStreamWaitEvent(ps, u.second, 0) != hipSuccess) return -EIO;
        return 0;
    }
    // a launch on this image, on stream s, starts after the image's last upload
    int wait_ready(hipStream_t s) {
        if (!ready_armed) return 0;
        return hipStreamWaitEvent(s, ready, 0) == hipSuccess ? 0 : -EIO;
    }
    ~DeviceEpoch() {
        if (ordinal < 0) return;
        DeviceGuard g(ordinal);
        (void)hipDeviceSynchronize();  // batches launched on this image have finished
        for (void *p : buf)
            if (p) (void)hipFree(p);
        for (auto &u : uses) (void)hipEventDestroy(u.second);
        if (ready) (void)hipEventDestroy(ready);
    }
};

// Incremental-commit upload path of one device: a non-blocking stream (never ordered
// behind classify launches on the null or any blocking stream) and pinned host + device
// staging buffers, grown on demand and kept.
struct PatchPipe {
    int ordinal = -1;
    hipStream_t stream = nullptr;
    uint8_t *host = nullptr, *dev = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;  // the last upload out of the staging buffers
    bool done_armed = false;
    int reserve(size_t bytes) {
        if (done_armed) {  // the previous commit's upload has left the staging buffers
            if (hipEventSynchronize(done) != hipSuccess) return -EIO;
            done_armed = false;
        }
        if (bytes <= cap) return 0;
        size_t c = cap ? cap : (1u << 20);
        while (c < bytes) c *= 2;
        if (host) (void)hipHostFree(host);
        if (dev) (void)hipFree(dev);
        host = dev = nullptr;
        cap = 0;
        if (hipHostMalloc(reinterpret_cast<void **>(&host), c, hipHostMallocDefault) != hipSuccess) return -ENOMEM;
        if (hipMalloc(reinterpret_cast<void **>(&dev), c) != hipSuccess) return -ENOMEM;
        cap = c;
        return 0;
    }
    ~PatchPipe() {
        if (ordinal < 0) return;
        DeviceGuard g(ordinal);
        if (stream) (void)hipStreamSynchronize(stream);
        if (done) (void)hipEventDestroy(done);
        if (host) (void)hipHostFree(host);
        if (dev) (void)hipFree(dev);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

// Two images per device: `epoch` is live (new batches read it), `spare` holds
// the previous epoch and is patched up to the next one while `epoch` serves.
struct Device {
    int ordinal = 0;
    uint32_t cus = 256;
    uint64_t *stats_own = nullptr;
    uint64_t *stats = nullptr;
    std::shared_ptr<DeviceEpoch> epoch, spare;
    // debug lookup capture set (allocated when debug_lookup is first set)
    uint64_t *dbg_fp = nullptr;
    uint32_t *dbg_keys = nullptr;
    uint32_t *dbg_count = nullptr;
    std::shared_ptr<struct HostPipe> pipe;  // infw_classify_host chunk buffers + streams
    std::shared_ptr<PatchPipe> patch;       // incremental-commit uploads
};

// Two chunk slots of device buffers and three streams for host-resident batches.
struct HostPipe {
    int ordinal = -1;
    uint64_t chunk = 0;
    hipStream_t h2d = nullptr, run = nullptr, d2h = nullptr;
    struct Slot {
        uint8_t *saddr = nullptr;
        uint32_t *ifindex = nullptr, *pkt_len = nullptr, *meta = nullptr, *l4word = nullptr, *res = nullptr;
        uint8_t *ver = nullptr;
        hipEvent_t in_done = nullptr, run_done = nullptr, out_done = nullptr;
    } slot[2];
    std::mutex mu;
    ~HostPipe() {
        if (ordinal < 0) return;
        DeviceGuard g(ordinal);
        (void)hipDeviceSynchronize();
        for (auto &s : slot) {
            for (void *p : {(void *)s.saddr, (void *)s.ifindex, (void *)s.pkt_len, (void *)s.meta, (void *)s.l4word,
                            (void *)s.res, (void *)s.ver})
                if (p) (void)hipFree(p);
            for (hipEvent_t e : {s.in_done, s.run_done, s.out_done})
                if (e) (void)hipEventDestroy(e);
        }
        for (hipStream_t st : {h2d, run, d2h})
            if (st) (void)hipStreamDestroy(st);
    }
};

constexpr uint32_t kDbgSlots = 2 * INFW_DBG_MAX_ENTRIES;

}  // namespace infw

using namespace infw;

struct infw_ctx {
    std::vector<Device> devs;
    uint32_t flags = 0;
    PendingMap map;
    std::unique_ptr<HostTables> host_image;  // the committed image (patched by incremental commits)
    IncState inc;
    std::mutex epoch_mu;  // guards devs[*].epoch swaps vs classify snapshots
    // launch shape of the classify kernel (infw_set_launch / INFW_BLOCK, INFW_SCAN_GROUP, INFW_BLOCKS_PER_CU)
    int block = 768, group = 0, blocks_per_cu = 2;
    uint32_t debug_lookup = 0;  // kernel.c:78
    uint64_t epoch_no = 0;
    uint64_t committed_gen = ~0ull;
    struct infw_table_info info{};
};

static bool growable(int b) { return b == TB_TBL8 || b == TB_DESC || b == TB_RULES || b == TB_DTE || b == TB_DTL; }

// Point the kernel's table view at an image's buffers.
static void bind_view(DeviceEpoch &e, const HostTables &h) {
    infw_dev_tables &t = e.view;
    memset(&t, 0, sizeof(t));
    t.if_keys = static_cast<const uint32_t *>(e.buf[TB_IFK]);
    t.if_slot = static_cast<const uint32_t *>(e.buf[TB_IFS]);
    t.l16 = static_cast<const uint32_t *>(e.buf[TB_L16]);
    t.nodes = static_cast<const infw_bnode *>(e.buf[TB_NODES]);
    t.vpool = static_cast<const uint32_t *>(e.buf[TB_VPOOL]);
    t.tbl24 = static_cast<const uint64_t *>(e.buf[TB_TBL24]);
    t.tbl8 = static_cast<const uint32_t *>(e.buf[TB_TBL8]);
    t.ltab = static_cast<const infw_long_entry *>(e.buf[TB_LTAB]);
    t.btab = static_cast<const infw_v6_bucket *>(e.buf[TB_BTAB]);
    t.desc = static_cast<const uint64_t *>(e.buf[TB_DESC]);
    t.rules = static_cast<const uint64_t *>(e.buf[TB_RULES]);
    t.dte = static_cast<const infw_dt_line *>(e.buf[TB_DTE]);
    t.dtl = static_cast<const infw_dt_line *>(e.buf[TB_DTL]);
    t.levels = static_cast<const uint8_t *>(e.buf[TB_LEVELS]);
    t.wild = static_cast<const uint32_t *>(e.buf[TB_WILD]);
    t.n_wild = h.n_wild;
    t.lean = (h.short_mode == INFW_SHORT_DIR24 || h.short_mode == INFW_SHORT_NONE ||
              h.short_mode == INFW_SHORT_DXR) && h.n_overflow_groups == 0 &&
             h.n_wild == 0;
    t.if_mask = (uint32_t)h.if_keys.size() - 1;
    t.if_mult = h.if_mult;
    t.if_shift = h.if_shift;
    t.n_slots = h.n_slots;
    t.lmask = h.ltab.size() - 1;
    t.bmask = h.btab.size() - 1;
    t.b2n = h.b2n;
    t.short_mode = h.short_mode;
    t.n_levels = (uint32_t)h.levels.size();
    t.dt_plog2 = h.dt_plog2;
    t.dt_pl = static_cast<const uint32_t *>(e.buf[TB_DTPL]);
    t.n_dt_pl = (uint32_t)h.dt_pl.size();
    t.dxr_idx = static_cast<const uint32_t *>(e.buf[TB_DXRI]);
    t.dxr_lines = static_cast<const infw_dt_line *>(e.buf[TB_DXRL]);
}

static int upload_epoch(const HostTables &h, int ordinal, std::shared_ptr<DeviceEpoch> &out) {
    DeviceGuard g(ordinal);
    if (!g.ok) {
        set_error("hipSetDevice failed");
        return -ENODEV;
    }
    auto ep = std::make_shared<DeviceEpoch>();
    ep->ordinal = ordinal;
    for (int b = 0; b < TB_COUNT; b++) {
        const void *p;
        size_t bytes;
        host_buffer(h, b, &p, &bytes);
        size_t cap = bytes < 64 ? 64 : bytes;
        if (growable(b)) cap += std::max<size_t>(bytes / 4, 256u << 10);
        HIP_OK(hipMalloc(&ep->buf[b], cap));
        ep->cap[b] = cap;
        ep->bytes += cap;
        if (bytes) HIP_OK(hipMemcpy(ep->buf[b], p, bytes, hipMemcpyHostToDevice));
    }
    bind_view(*ep, h);
    out = ep;
    return 0;
}

// A second image with the same capacities and contents (device-to-device copy):
// the spare an incremental commit patches.
static int clone_epoch(const DeviceEpoch &src, const HostTables &h, std::shared_ptr<DeviceEpoch> &out) {
    DeviceGuard g(src.ordinal);
    if (!g.ok) return -ENODEV;
    auto ep = std::make_shared<DeviceEpoch>();
    ep->ordinal = src.ordinal;
    for (int b = 0; b < TB_COUNT; b++) {
        const void *p;
        size_t bytes;
        host_buffer(h, b, &p, &bytes);
        HIP_OK(hipMalloc(&ep->buf[b], src.cap[b]));
        ep->cap[b] = src.cap[b];
        ep->bytes += src.cap[b];
        if (bytes) HIP_OK(hipMemcpy(ep->buf[b], src.buf[b], bytes, hipMemcpyDeviceToDevice));
    }
    bind_view(*ep, h);
    HIP_OK(hipDeviceSynchronize());
    out = ep;
    return 0;
}

static bool image_fits(const DeviceEpoch &ep, const HostTables &h) {
    for (int b = 0; b < TB_COUNT; b++) {
        const void *p;
        size_t bytes;
        host_buffer(h, b, &p, &bytes);
        if (bytes > ep.cap[b]) return false;
    }
    return true;
}

// Copy ep.pending (merged, widened to whole words) from the host image into the
// device image through the device's non-blocking patch stream, asynchronously: the
// caller has ordered the stream after the image's last readers; ep.ready marks the end.
static int flush_pending(DeviceEpoch &ep, const HostTables &h, uint32_t cus, PatchPipe &pp, uint64_t *bytes_out) {
    std::vector<DirtyRange> &r = ep.pending;
    for (DirtyRange &x : r) {  // whole 4-B words (every table buffer is an array of >= 4-B elements)
        const uint64_t end = (x.off + x.len + 3) & ~3ull;
        x.off &= ~3ull;
        x.len = end - x.off;
    }
    std::sort(r.begin(), r.end(), [](const DirtyRange &a, const DirtyRange &b) {
        return a.buf != b.buf ? a.buf < b.buf : a.off < b.off;
    });
    std::vector<DirtyRange> m;
    for (const DirtyRange &x : r) {
        if (!m.empty() && m.back().buf == x.buf && x.off <= m.back().off + m.back().len + 64) {
            m.back().len = std::max(m.back().off + m.back().len, x.off + x.len) - m.back().off;
        } else {
            m.push_back(x);
        }
    }
    r.clear();
    DeviceGuard g(ep.ordinal);
    struct Piece {
        const uint8_t *src;
        uint8_t *dst;
        uint64_t len;
    };
    std::vector<Piece> pieces;
    uint64_t total = 0;
    for (const DirtyRange &x : m) {
        const void *p;
        size_t bytes;
        host_buffer(h, (int)x.buf, &p, &bytes);
        const uint64_t len = std::min<uint64_t>(x.len, bytes > x.off ? (bytes - x.off) & ~3ull : 0);
        if (!len) continue;
        pieces.push_back({static_cast<const uint8_t *>(p) + x.off, static_cast<uint8_t *>(ep.buf[x.buf]) + x.off, len});
        total += len;
    }
    if (!pieces.empty()) {
        const size_t dbytes = (pieces.size() * sizeof(infw_patch_desc) + 255) & ~(size_t)255;
        int rc = pp.reserve(dbytes + total);
        if (rc) {
            set_error("table patch: staging allocation failed");
            return rc;
        }
        auto *descs = reinterpret_cast<infw_patch_desc *>(pp.host);
        uint8_t *words = pp.host + dbytes;
        uint64_t w = 0;
        for (size_t i = 0; i < pieces.size(); i++) {
            memcpy(words + 4 * w, pieces[i].src, pieces[i].len);
            descs[i] = infw_patch_desc{(uint64_t)(uintptr_t)pieces[i].dst, w, pieces[i].len / 4};
            w += pieces[i].len / 4;
        }
        // few ranges: DMA copies straight from the pinned staging (no compute unit needed, so they
        // proceed while a classify launch occupies every CU); many: one upload + one scatter launch
        bool ok = true;
        if (pieces.size() <= 64) {
            for (size_t i = 0; i < pieces.size() && ok; i++)
                ok = hipMemcpyAsync(pieces[i].dst, words + 4 * descs[i].src, pieces[i].len, hipMemcpyHostToDevice,
                                    pp.stream) == hipSuccess;
        } else {
            ok = hipMemcpyAsync(pp.dev, pp.host, dbytes + total, hipMemcpyHostToDevice, pp.stream) == hipSuccess &&
                 !infw_launch_scatter(reinterpret_cast<const uint32_t *>(pp.dev + dbytes), pp.dev,
                                      (uint32_t)pieces.size(), cus, pp.stream);
        }
        if (ok && !ep.ready) ok = hipEventCreateWithFlags(&ep.ready, hipEventDisableTiming) == hipSuccess;
        if (ok && !pp.done) ok = hipEventCreateWithFlags(&pp.done, hipEventDisableTiming) == hipSuccess;
        if (ok) ok = hipEventRecord(ep.ready, pp.stream) == hipSuccess && hipEventRecord(pp.done, pp.stream) == hipSuccess;
        if (!ok) {
            set_error(std::string("table patch upload failed: ") + hipGetErrorString(hipGetLastError()));
            (void)hipStreamSynchronize(pp.stream);
            return -EIO;
        }
        ep.ready_armed = true;
        pp.done_armed = true;
    }
    if (bytes_out) *bytes_out += total;
    return 0;
}

// The incremental-commit upload path of a device, warmed up: stream, pinned and device staging, and one
// DMA copy + one scatter launch (the first of each pays for queue and code-object setup — ~0.1 s — which
// would otherwise land on the first incremental commit).
static int make_patch_pipe(Device &d) {
    DeviceGuard g(d.ordinal);
    if (!g.ok) return -ENODEV;
    auto pp = std::make_shared<PatchPipe>();
    pp->ordinal = d.ordinal;
    HIP_OK(hipStreamCreateWithFlags(&pp->stream, hipStreamNonBlocking));
    if (pp->reserve(1u << 20)) {
        set_error("patch pipe: staging allocation failed");
        return -ENOMEM;
    }
    auto *desc = reinterpret_cast<infw_patch_desc *>(pp->host);
    *desc = infw_patch_desc{(uint64_t)(uintptr_t)(pp->dev + 512), 0, 16};  // 64 B within the staging buffer
    HIP_OK(hipMemcpyAsync(pp->dev, pp->host, 256, hipMemcpyHostToDevice, pp->stream));
    if (infw_launch_scatter(reinterpret_cast<const uint32_t *>(pp->dev + 256), pp->dev, 1, d.cus, pp->stream)) {
        set_error("patch pipe: warm-up launch failed");
        return -EIO;
    }
    HIP_OK(hipStreamSynchronize(pp->stream));
    d.patch = pp;
    return 0;
}

extern "C" {

const char *infw_last_error(void) { return g_err.c_str(); }
int infw_abi_version(void) { return INFW_ABI_VERSION; }

int infw_create(infw_ctx **out, const int *hip_devices, int n_dev, uint32_t max_entries,
                uint32_t flags) {
    if (!out) return -EINVAL;
    *out = nullptr;
    std::unique_ptr<infw_ctx> ctx(new infw_ctx());
    ctx->flags = flags;
    ctx->map.max_entries = max_entries ? max_entries : (1u << 22);
    if (flags & INFW_F_HOST_ONLY) {
        int rc = infw_table_commit(ctx.get());
        if (rc) return rc;
        ctx->epoch_no = 0;
        ctx->info.epoch = 0;
        *out = ctx.release();
        return 0;
    }
    // default shape: 2 x 768-thread workgroups per CU = 24 waves (6 per SIMD). Measured on MI355X at configs[2]:
    // 24 waves beat 32 (512 x 4) by 8 % and 16 (512 x 2) by 17 % — fewer lines in flight thrash the L2 less —
    // and 768 lets the LDS word cache hold 4096 entries (tools/tune.py, profiles/r01i/occupancy_sweep.log)
    ctx->block = 768;
    if (const char *e = getenv("INFW_BLOCK")) ctx->block = atoi(e) == 256 ? 256 : atoi(e) == 512 ? 512 : 768;
    if (const char *e = getenv("INFW_SCAN_GROUP")) {
        int g = atoi(e);
        ctx->group = (g == 1 || g == 4 || g == 8) ? g : 0;
    }
    ctx->blocks_per_cu = ctx->block == 768 ? 2 : ctx->block == 512 ? 3 : 6;  // 24 waves per CU
    if (const char *e = getenv("INFW_BLOCKS_PER_CU")) ctx->blocks_per_cu = atoi(e) > 0 ? atoi(e) : ctx->blocks_per_cu;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        set_error("no HIP device visible: the classifier has no CPU fallback");
        return -ENODEV;
    }
    std::vector<int> ords;
    if (!hip_devices || n_dev <= 0) {
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) cur = 0;
        ords.push_back(cur);
    } else {
        for (int i = 0; i < n_dev; i++) {
            if (hip_devices[i] < 0 || hip_devices[i] >= count) {
                set_error("device ordinal out of range");
                return -ENODEV;
            }
            ords.push_back(hip_devices[i]);
        }
    }
    for (int o : ords) {
        Device d;
        d.ordinal = o;
        DeviceGuard g(o);
        if (!g.ok) {
            set_error("hipSetDevice failed");
            return -ENODEV;
        }
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, o);
        d.cus = (uint32_t)cus;
        HIP_OK(hipMalloc(&d.stats_own, INFW_MAX_TARGETS * sizeof(ruleStatistics_st)));
        HIP_OK(hipMemset(d.stats_own, 0, INFW_MAX_TARGETS * sizeof(ruleStatistics_st)));
        d.stats = d.stats_own;
        ctx->devs.push_back(d);
    }
    // an empty epoch so classify works before the first commit (everything misses)
    int rc = infw_table_commit(ctx.get());
    if (rc) return rc;
    for (auto &d : ctx->devs)
        if ((rc = make_patch_pipe(d))) return rc;
    ctx->epoch_no = 0;
    ctx->info.epoch = 0;
    *out = ctx.release();
    return 0;
}

void infw_destroy(infw_ctx *ctx) {
    if (!ctx) return;
    for (auto &d : ctx->devs) {
        d.pipe.reset();
        d.patch.reset();
        d.epoch.reset();
        d.spare.reset();
        DeviceGuard g(d.ordinal);
        (void)hipDeviceSynchronize();
        if (d.stats_own) (void)hipFree(d.stats_own);
        if (d.dbg_fp) (void)hipFree(d.dbg_fp);
        if (d.dbg_keys) (void)hipFree(d.dbg_keys);
        if (d.dbg_count) (void)hipFree(d.dbg_count);
    }
    delete ctx;
}

int infw_num_devices(const infw_ctx *ctx) { return ctx ? (int)ctx->devs.size() : 0; }

int infw_table_update(infw_ctx *ctx, const lpm_ip_key_st *key, const rulesVal_st *val,
                      uint64_t flags) {
    if (!ctx || !key || !val) return -EINVAL;
    return ctx->map.update(key, reinterpret_cast<const uint8_t *>(val), flags);
}

int infw_table_update_batch(infw_ctx *ctx, const lpm_ip_key_st *keys, const rulesVal_st *vals,
                            const uint32_t *val_index, uint64_t n, uint64_t flags, uint64_t *done) {
    if (done) *done = 0;
    if (!ctx || (n && (!keys || !vals))) return -EINVAL;
    for (uint64_t i = 0; i < n; i++) {
        const rulesVal_st *v = val_index ? &vals[val_index[i]] : &vals[i];
        int rc = ctx->map.update(&keys[i], reinterpret_cast<const uint8_t *>(v), flags);
        if (rc) return rc;
        if (done) *done = i + 1;
    }
    return 0;
}

int infw_table_delete(infw_ctx *ctx, const lpm_ip_key_st *key) {
    if (!ctx || !key) return -EINVAL;
    return ctx->map.remove(key);
}

int infw_table_get_next_key(infw_ctx *ctx, const lpm_ip_key_st *key, lpm_ip_key_st *next) {
    if (!ctx || !next) return -EINVAL;
    return ctx->map.next_key(key, next);
}

int infw_table_lookup(infw_ctx *ctx, const lpm_ip_key_st *key, rulesVal_st *val) {
    if (!ctx || !key) return -EINVAL;
    return ctx->map.lookup(key, reinterpret_cast<uint8_t *>(val));
}

int infw_table_count(infw_ctx *ctx, uint64_t *n) {
    if (!ctx || !n) return -EINVAL;
    *n = ctx->map.nodes.size();
    return 0;
}

int infw_table_commit(infw_ctx *ctx) {
    if (!ctx) return -EINVAL;
    auto t0 = std::chrono::steady_clock::now();
    std::vector<DirtyRange> ranges;
    std::string why;
    int rc = 1;
    const char *fe = getenv("INFW_FULL_COMMIT");
    const bool force_full = (ctx->flags & INFW_F_FULL_COMMIT) || (fe && atoi(fe) != 0);
    if (ctx->host_image && !force_full) rc = patch_tables(ctx->map, *ctx->host_image, ctx->inc, ranges, &why);
    if (rc < 0) rc = 1;  // the patch gave up half-way (image marked invalid): recompile
    uint32_t mode = INFW_COMMIT_INCREMENTAL;
    uint64_t patched = 0;
    auto t1 = t0;
    if (rc == 1) {
        mode = INFW_COMMIT_FULL;
        std::unique_ptr<HostTables> h(new HostTables());
        int smode = -1;
        if (const char *e = getenv("INFW_SHORT_TABLE"))
            smode = strcmp(e, "compressed") == 0 ? 1 : strcmp(e, "dir24") == 0 ? 0 : strcmp(e, "dxr") == 0 ? 3 : -1;
        IncState inc;
        rc = compile_tables(ctx->map, *h, smode, 4ull << 30, &inc);
        if (rc) return rc;  // the previous epoch stays live
        t1 = std::chrono::steady_clock::now();
        std::vector<std::shared_ptr<DeviceEpoch>> eps(ctx->devs.size()), spares(ctx->devs.size());
        for (size_t i = 0; i < ctx->devs.size(); i++) {
            rc = upload_epoch(*h, ctx->devs[i].ordinal, eps[i]);
            if (!rc) rc = clone_epoch(*eps[i], *h, spares[i]);
            if (rc) return rc;  // nothing swapped: the previous epoch stays live
        }
        std::vector<std::shared_ptr<DeviceEpoch>> old;
        {
            std::lock_guard<std::mutex> lk(ctx->epoch_mu);
            for (size_t i = 0; i < ctx->devs.size(); i++) {
                old.push_back(ctx->devs[i].epoch);
                old.push_back(ctx->devs[i].spare);
                ctx->devs[i].epoch = eps[i];
                ctx->devs[i].spare = spares[i];
            }
        }
        old.clear();  // waits for batches still running on the old images, then frees them
        ctx->host_image = std::move(h);
        ctx->inc = std::move(inc);
        for (auto &e : eps) patched += e->bytes;
    } else {
        t1 = std::chrono::steady_clock::now();
        const HostTables &h = *ctx->host_image;
        for (auto &d : ctx->devs) {
            std::shared_ptr<DeviceEpoch> next, fresh_spare;
            if (d.spare && image_fits(*d.spare, h)) {
                // batches that took the spare while it was live have launched and finished
                while (d.spare.use_count() > 1) std::this_thread::sleep_for(std::chrono::microseconds(50));
                next = d.spare;
                if (!d.patch) {
                    rc = make_patch_pipe(d);
                    if (rc) return rc;
                }
                const auto w0 = std::chrono::steady_clock::now();
                rc = next->order_after_uses(d.patch->stream);  // after the batches that read this image
                const auto w1 = std::chrono::steady_clock::now();
                next->pending.insert(next->pending.end(), ranges.begin(), ranges.end());
                if (!rc) rc = flush_pending(*next, h, d.cus, *d.patch, &patched);
                if (getenv("INFW_COMMIT_TRACE"))
                    fprintf(stderr, "[commit] patch %.3f ms, order %.3f ms, stage %.3f ms, %zu ranges\n",
                            std::chrono::duration<double, std::milli>(w0 - t1).count() +
                                std::chrono::duration<double, std::milli>(t1 - t0).count(),
                            std::chrono::duration<double, std::milli>(w1 - w0).count(),
                            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w1).count(),
                            ranges.size());
                if (rc) {
                    std::lock_guard<std::mutex> lk(ctx->epoch_mu);
                    d.spare.reset();  // half-patched: never used again
                    return rc;
                }
            } else {
                // the patched host image outgrew the spare's buffers: a fresh pair from it
                rc = upload_epoch(h, d.ordinal, next);
                if (!rc) rc = clone_epoch(*next, h, fresh_spare);
                if (rc) return rc;
                mode = INFW_COMMIT_REUPLOAD;
                patched += next->bytes;
            }
            std::shared_ptr<DeviceEpoch> prev;
            {
                std::lock_guard<std::mutex> lk(ctx->epoch_mu);
                prev = d.epoch;
                d.epoch = next;
                d.spare = fresh_spare;
                if (!fresh_spare && prev && image_fits(*prev, h)) {
                    prev->pending.insert(prev->pending.end(), ranges.begin(), ranges.end());
                    d.spare = prev;
                }
            }
        }
    }
    auto t2 = std::chrono::steady_clock::now();
    ctx->map.dirty.clear();
    ctx->epoch_no++;
    const HostTables &h = *ctx->host_image;
    struct infw_table_info &in = ctx->info;
    in.epoch = ctx->epoch_no;
    in.n_entries = h.n_entries;
    in.n_if_slots = h.n_slots;
    in.n_lists = h.n_lists;
    in.n_rules = h.rules.size();
    in.n_tbl8_groups = h.n_tbl8_groups;
    in.n_long_levels = (uint32_t)h.levels.size();
    in.n_long_entries = h.n_long_entries;
    in.device_bytes = ctx->devs.empty() || !ctx->devs[0].epoch ? 0 : ctx->devs[0].epoch->bytes;
    in.compile_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    in.upload_ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
    in.n_v6_groups = h.n_buckets;
    in.n_v6_overflow = h.n_overflow_groups;
    in.v6_slot_buckets = h.b2n;
    in.short_mode = h.short_mode;
    in.dxr_lines = h.short_mode == INFW_SHORT_DXR ? (uint32_t)h.dxr_lines.size() : 0u;
    in.commit_mode = mode;
    in.dt_parts = 1u << h.dt_plog2;
    in.patch_bytes = patched;
    in.dead_lists = ctx->inc.dead_lists;
    memset(in.full_reason, 0, sizeof(in.full_reason));
    if (mode == INFW_COMMIT_FULL) strncpy(in.full_reason, force_full ? "forced" : why.c_str(), sizeof(in.full_reason) - 1);
    ctx->committed_gen = ctx->map.generation;
    return 0;
}

int infw_debug_walk(infw_ctx *ctx, const uint32_t *tuples, uint64_t n, uint32_t *out) {
    if (!ctx || (n && (!tuples || !out))) return -EINVAL;
    if (!ctx->host_image) {
        set_error("debug_walk: no committed table image");
        return -ENODATA;
    }
    const infw_dev_tables t = ctx->host_image->view();
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t *q = tuples + 8 * i;
        int cls = 0;
        uint32_t val = 0, result = 0;
        int pk = infw_parse(q[6], q[7], &cls, &val);
        if (pk >= INFW_PK_V4) {
            uint32_t l1 = infw_lpm(t, pk, q[4], q);
            if (l1) {
                const uint64_t row = (uint64_t)(l1 - 1) * INFW_DESC_STRIDE + cls;
                result = infw_dt_eval(t, l1 - 1, cls, val);
                const uint32_t scan = infw_scan_serial(t, t.desc[row], val);
                if (scan != result) {
                    set_error("debug_walk: decision table disagrees with the rule scan");
                    return -EIO;
                }
            }
        }
        out[i] = result;
    }
    return 0;
}

int infw_table_info(infw_ctx *ctx, struct infw_table_info *info) {
    if (!ctx || !info) return -EINVAL;
    *info = ctx->info;
    return 0;
}

int infw_classify(infw_ctx *ctx, int dev, const infw_batch_soa *in, uint64_t n,
                  uint32_t *result_words, uint8_t *xdp_verdicts, void *stream) {
    return infw_classify_ex(ctx, dev, in, n, result_words, xdp_verdicts, nullptr, stream);
}

static int classify_impl(infw_ctx *ctx, int dev, const infw_batch_soa *in, const infw_batch_soa_c *in_c, uint64_t n,
                         uint32_t *result_words, uint8_t *xdp_verdicts, const struct infw_classify_ex *ex, void *stream);

int infw_classify_ex(infw_ctx *ctx, int dev, const infw_batch_soa *in, uint64_t n, uint32_t *result_words,
                     uint8_t *xdp_verdicts, const struct infw_classify_ex *ex, void *stream) {
    return classify_impl(ctx, dev, in, nullptr, n, result_words, xdp_verdicts, ex, stream);
}

int infw_classify_c(infw_ctx *ctx, int dev, const infw_batch_soa_c *in, uint64_t n, uint32_t *result_words,
                    uint8_t *xdp_verdicts, void *stream) {
    if (!in) return -EINVAL;
    if (n && (!in->saddr4 || !in->v6tail || ((uintptr_t)in->v6tail & 3) != 0)) {
        set_error("classify_c: null or misaligned address stream");
        return -EINVAL;
    }
    return classify_impl(ctx, dev, nullptr, in, n, result_words, xdp_verdicts, nullptr, stream);
}

int infw_soa_compact(infw_ctx *ctx, int dev, const infw_batch_soa *in, uint64_t n, uint32_t *saddr4, uint8_t *v6tail,
                     void *stream) {
    if (!ctx || !in || (n && (!in->saddr || !in->meta || !saddr4 || !v6tail))) return -EINVAL;
    if (ctx->devs.empty()) return -ENODEV;
    if (dev < 0 || dev >= (int)ctx->devs.size()) return -EINVAL;
    if (((uintptr_t)in->saddr & 15) != 0 || ((uintptr_t)v6tail & 3) != 0) {
        set_error("soa_compact: saddr must be 16-byte and v6tail 4-byte aligned");
        return -EINVAL;
    }
    Device &d = ctx->devs[dev];
    DeviceGuard g(d.ordinal);
    if (!g.ok) return -ENODEV;
    if (infw_launch_soa_compact(in, n, saddr4, v6tail, d.cus, static_cast<hipStream_t>(stream))) {
        set_error(std::string("soa_compact launch failed: ") + hipGetErrorString(hipGetLastError()));
        return -EIO;
    }
    return 0;
}

static int classify_impl(infw_ctx *ctx, int dev, const infw_batch_soa *in, const infw_batch_soa_c *in_c, uint64_t n,
                         uint32_t *result_words, uint8_t *xdp_verdicts, const struct infw_classify_ex *ex, void *stream) {
    if (ex && (ex->size < sizeof(struct infw_classify_ex) || ex->flags != 0 || (ex->events_cap && !ex->events) ||
               (ex->events && !ex->events_count))) {
        set_error("classify_ex: bad options");
        return -EINVAL;
    }
    if (!ctx || (!in && !in_c)) return -EINVAL;
    if (ctx->devs.empty()) {
        set_error("classify: host-only context has no device tables");
        return -ENODEV;
    }
    if (dev < 0 || dev >= (int)ctx->devs.size()) return -EINVAL;
    const uint32_t *ifx = in ? in->ifindex : in_c->ifindex, *pl = in ? in->pkt_len : in_c->pkt_len;
    const uint32_t *mt = in ? in->meta : in_c->meta, *l4 = in ? in->l4word : in_c->l4word;
    if (n && ((in && !in->saddr) || !ifx || !pl || !mt || !l4)) {
        set_error("classify: null input stream");
        return -EINVAL;
    }
    if (in && ((uintptr_t)in->saddr & 15) != 0) {
        set_error("classify: saddr must be 16-byte aligned");
        return -EINVAL;
    }
    Device &d = ctx->devs[dev];
    std::shared_ptr<DeviceEpoch> ep;
    {
        std::lock_guard<std::mutex> lk(ctx->epoch_mu);
        ep = d.epoch;
    }
    DeviceGuard g(d.ordinal);
    if (!g.ok) {
        set_error("hipSetDevice failed");
        return -ENODEV;
    }
    const bool evs = ex && ex->events_count;
    if (ep->wait_ready(static_cast<hipStream_t>(stream))) {
        set_error("classify: stream wait on the epoch's upload failed");
        return -EIO;
    }
    int rc = infw_launch_classify(&ep->view, in, n, result_words, xdp_verdicts, d.stats, d.cus, ctx->block,
                                  ctx->group, ctx->blocks_per_cu, static_cast<hipStream_t>(stream),
                                  evs ? ex->events : nullptr, evs ? ex->events_cap : 0, evs ? ex->events_count : nullptr,
                                  ctx->debug_lookup ? d.dbg_fp : nullptr, d.dbg_keys, d.dbg_count, kDbgSlots, in_c);
    if (rc) {
        set_error(std::string("classify launch failed: ") + hipGetErrorString(hipGetLastError()));
        return -EIO;
    }
    ep->mark_use(static_cast<hipStream_t>(stream));
    return 0;
}

static int make_pipe(int ordinal, uint64_t chunk, std::shared_ptr<HostPipe> &out) {
    DeviceGuard g(ordinal);
    if (!g.ok) return -ENODEV;
    auto p = std::make_shared<HostPipe>();
    p->ordinal = ordinal;
    p->chunk = chunk;
    HIP_OK(hipStreamCreateWithFlags(&p->h2d, hipStreamNonBlocking));
    HIP_OK(hipStreamCreateWithFlags(&p->run, hipStreamNonBlocking));
    HIP_OK(hipStreamCreateWithFlags(&p->d2h, hipStreamNonBlocking));
    for (auto &s : p->slot) {
        HIP_OK(hipMalloc(&s.saddr, chunk * 16));
        HIP_OK(hipMalloc(&s.ifindex, chunk * 4));
        HIP_OK(hipMalloc(&s.pkt_len, chunk * 4));
        HIP_OK(hipMalloc(&s.meta, chunk * 4));
        HIP_OK(hipMalloc(&s.l4word, chunk * 4));
        HIP_OK(hipMalloc(&s.res, chunk * 4));
        HIP_OK(hipMalloc(&s.ver, chunk));
        HIP_OK(hipEventCreateWithFlags(&s.in_done, hipEventDisableTiming));
        HIP_OK(hipEventCreateWithFlags(&s.run_done, hipEventDisableTiming));
        HIP_OK(hipEventCreateWithFlags(&s.out_done, hipEventDisableTiming));
    }
    out = p;
    return 0;
}

static int classify_host_chunks(infw_ctx *ctx, Device &d, const std::shared_ptr<DeviceEpoch> &ep, HostPipe &p,
                                const infw_batch_soa *in, uint64_t n, uint32_t *results, uint8_t *verdicts);

int infw_classify_host(infw_ctx *ctx, int dev, const infw_batch_soa *in, uint64_t n, uint32_t *results,
                       uint8_t *verdicts, uint64_t chunk) {
    if (!ctx || !in) return -EINVAL;
    if (ctx->devs.empty()) {
        set_error("classify_host: host-only context has no device tables");
        return -ENODEV;
    }
    if (dev < 0 || dev >= (int)ctx->devs.size()) return -EINVAL;
    if (n && (!in->saddr || !in->ifindex || !in->pkt_len || !in->meta || !in->l4word)) {
        set_error("classify_host: null input stream");
        return -EINVAL;
    }
    if (n == 0) return 0;
    chunk = chunk ? chunk : (4u << 20);
    chunk = (chunk + 511) & ~511ull;  // whole tiles
    Device &d = ctx->devs[dev];
    std::shared_ptr<HostPipe> pipe;
    {
        std::lock_guard<std::mutex> lk(ctx->epoch_mu);
        pipe = d.pipe;
    }
    if (!pipe || pipe->chunk != chunk) {
        int rc = make_pipe(d.ordinal, chunk, pipe);
        if (rc) return rc;
        std::lock_guard<std::mutex> lk(ctx->epoch_mu);
        d.pipe = pipe;
    }
    std::lock_guard<std::mutex> plk(pipe->mu);  // one host batch at a time per device
    std::shared_ptr<DeviceEpoch> ep;             // the whole batch reads one epoch
    {
        std::lock_guard<std::mutex> lk(ctx->epoch_mu);
        ep = d.epoch;
    }
    DeviceGuard g(d.ordinal);
    if (!g.ok) return -ENODEV;
    HIP_OK(ep->wait_ready(pipe->run) ? hipErrorUnknown : hipSuccess);
    int rc = classify_host_chunks(ctx, d, ep, *pipe, in, n, results, verdicts);
    // also on an error exit: the launches already queued read this epoch, and the copies already queued read from
    // and write into the caller's host buffers — none may be in flight once this returns
    ep->mark_use(pipe->run);
    hipError_t e1 = hipStreamSynchronize(pipe->h2d), e2 = hipStreamSynchronize(pipe->run),
               e3 = hipStreamSynchronize(pipe->d2h);
    if (rc) return rc;
    for (hipError_t e : {e1, e2, e3})
        if (e != hipSuccess) {
            set_error(std::string("classify_host: stream synchronize: ") + hipGetErrorString(e));
            return -EIO;
        }
    return 0;
}

static int classify_host_chunks(infw_ctx *ctx, Device &d, const std::shared_ptr<DeviceEpoch> &ep, HostPipe &p,
                                const infw_batch_soa *in, uint64_t n, uint32_t *results, uint8_t *verdicts) {
    HostPipe *pipe = &p;
    const uint64_t chunk = p.chunk;
    const uint64_t nchunks = (n + chunk - 1) / chunk;
    for (uint64_t k = 0; k < nchunks; k++) {
        HostPipe::Slot &s = pipe->slot[k & 1];
        const uint64_t a = k * chunk, c = std::min(chunk, n - a);
        // the slot's buffers are free once chunk k-2's results left the device
        HIP_OK(hipStreamWaitEvent(pipe->h2d, s.out_done, 0));
        HIP_OK(hipMemcpyAsync(s.saddr, in->saddr + 16 * a, c * 16, hipMemcpyHostToDevice, pipe->h2d));
        HIP_OK(hipMemcpyAsync(s.ifindex, in->ifindex + a, c * 4, hipMemcpyHostToDevice, pipe->h2d));
        HIP_OK(hipMemcpyAsync(s.pkt_len, in->pkt_len + a, c * 4, hipMemcpyHostToDevice, pipe->h2d));
        HIP_OK(hipMemcpyAsync(s.meta, in->meta + a, c * 4, hipMemcpyHostToDevice, pipe->h2d));
        HIP_OK(hipMemcpyAsync(s.l4word, in->l4word + a, c * 4, hipMemcpyHostToDevice, pipe->h2d));
        HIP_OK(hipEventRecord(s.in_done, pipe->h2d));
        HIP_OK(hipStreamWaitEvent(pipe->run, s.in_done, 0));
        const infw_batch_soa db{s.saddr, s.ifindex, s.pkt_len, s.meta, s.l4word};
        if (infw_launch_classify(&ep->view, &db, c, results ? s.res : nullptr, verdicts ? s.ver : nullptr, d.stats,
                                 d.cus, ctx->block, ctx->group, ctx->blocks_per_cu, pipe->run, nullptr, 0, nullptr,
                                 ctx->debug_lookup ? d.dbg_fp : nullptr, d.dbg_keys, d.dbg_count, kDbgSlots, nullptr)) {
            set_error(std::string("classify_host launch failed: ") + hipGetErrorString(hipGetLastError()));
            return -EIO;
        }
        HIP_OK(hipEventRecord(s.run_done, pipe->run));
        HIP_OK(hipStreamWaitEvent(pipe->d2h, s.run_done, 0));
        if (results) HIP_OK(hipMemcpyAsync(results + a, s.res, c * 4, hipMemcpyDeviceToHost, pipe->d2h));
        if (verdicts) HIP_OK(hipMemcpyAsync(verdicts + a, s.ver, c, hipMemcpyDeviceToHost, pipe->d2h));
        HIP_OK(hipEventRecord(s.out_done, pipe->d2h));
    }
    return 0;
}

int infw_host_register(infw_ctx *ctx, void *ptr, uint64_t bytes) {
    if (!ctx || !ptr || !bytes) return -EINVAL;
    HIP_OK(hipHostRegister(ptr, bytes, hipHostRegisterDefault));
    return 0;
}

int infw_host_unregister(infw_ctx *ctx, void *ptr) {
    if (!ctx || !ptr) return -EINVAL;
    HIP_OK(hipHostUnregister(ptr));
    return 0;
}

int infw_debug_lookup_set(infw_ctx *ctx, uint32_t debug_lookup) {
    if (!ctx) return -EINVAL;
    if (debug_lookup)
        for (auto &d : ctx->devs) {
            if (d.dbg_fp) continue;
            DeviceGuard g(d.ordinal);
            if (!g.ok) return -ENODEV;
            HIP_OK(hipMalloc(&d.dbg_fp, kDbgSlots * sizeof(uint64_t)));
            HIP_OK(hipMalloc(&d.dbg_keys, kDbgSlots * 24));
            HIP_OK(hipMalloc(&d.dbg_count, sizeof(uint32_t)));
            HIP_OK(hipMemset(d.dbg_fp, 0, kDbgSlots * sizeof(uint64_t)));
            HIP_OK(hipMemset(d.dbg_count, 0, sizeof(uint32_t)));
        }
    ctx->debug_lookup = debug_lookup;
    return 0;
}

int infw_debug_keys_read(infw_ctx *ctx, lpm_ip_key_st *keys, uint32_t cap, uint32_t *n) {
    if (!ctx || !n || (cap && !keys)) return -EINVAL;
    std::set<std::array<uint8_t, 24>> all;
    std::vector<uint64_t> fp(kDbgSlots);
    std::vector<uint8_t> kb((size_t)kDbgSlots * 24);
    for (auto &d : ctx->devs) {
        if (!d.dbg_fp) continue;
        DeviceGuard g(d.ordinal);
        HIP_OK(hipDeviceSynchronize());
        HIP_OK(hipMemcpy(fp.data(), d.dbg_fp, fp.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(kb.data(), d.dbg_keys, kb.size(), hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < kDbgSlots && all.size() < INFW_DBG_MAX_ENTRIES; i++)
            if (fp[i] & 1) {  // a key's fingerprint (0 = free, 2 = tombstone)
                std::array<uint8_t, 24> k;
                memcpy(k.data(), &kb[(size_t)i * 24], 24);
                all.insert(k);
            }
    }
    uint32_t i = 0;
    for (const auto &k : all) {
        if (i < cap) memcpy(&keys[i], k.data(), 24);
        i++;
    }
    *n = i;
    return 0;
}

int infw_debug_keys_clear(infw_ctx *ctx) {
    if (!ctx) return -EINVAL;
    for (auto &d : ctx->devs) {
        if (!d.dbg_fp) continue;
        DeviceGuard g(d.ordinal);
        HIP_OK(hipDeviceSynchronize());
        HIP_OK(hipMemset(d.dbg_fp, 0, kDbgSlots * sizeof(uint64_t)));
        HIP_OK(hipMemset(d.dbg_count, 0, sizeof(uint32_t)));
    }
    return 0;
}

int infw_pack_frames(infw_ctx *ctx, int dev, const infw_frame_batch *fb, uint64_t n, const infw_batch_soa_out *out,
                     void *stream) {
    if (!ctx || !fb || !out) return -EINVAL;
    if (ctx->devs.empty()) {
        set_error("pack_frames: host-only context");
        return -ENODEV;
    }
    if (dev < 0 || dev >= (int)ctx->devs.size()) return -EINVAL;
    if (n && (!fb->frames || !fb->linear_len || !fb->ifindex || (!fb->offsets && !fb->stride) || !out->saddr ||
              !out->ifindex || !out->pkt_len || !out->meta || !out->l4word || ((uintptr_t)out->saddr & 15))) {
        set_error("pack_frames: bad arguments");
        return -EINVAL;
    }
    DeviceGuard g(ctx->devs[dev].ordinal);
    if (!g.ok) return -ENODEV;
    if (infw_launch_pack_frames(fb, n, out, nullptr, ctx->devs[dev].cus, static_cast<hipStream_t>(stream))) {
        set_error(std::string("pack launch failed: ") + hipGetErrorString(hipGetLastError()));
        return -EIO;
    }
    return 0;
}

int infw_classify_frames(infw_ctx *ctx, int dev, const infw_frame_batch *fb, uint64_t n, uint32_t *result_words,
                         uint8_t *xdp_verdicts, void *stream) {
    return infw_classify_frames_ex(ctx, dev, fb, n, result_words, xdp_verdicts, nullptr, stream);
}

int infw_classify_frames_ex(infw_ctx *ctx, int dev, const infw_frame_batch *fb, uint64_t n, uint32_t *result_words,
                            uint8_t *xdp_verdicts, const struct infw_classify_ex *ex, void *stream) {
    if (ex && (ex->size < sizeof(struct infw_classify_ex) || ex->flags != 0 || (ex->events_cap && !ex->events) ||
               (ex->events && !ex->events_count))) {
        set_error("classify_frames_ex: bad options");
        return -EINVAL;
    }
    if (!ctx || !fb) return -EINVAL;
    if (ctx->devs.empty()) {
        set_error("classify_frames: host-only context has no device tables");
        return -ENODEV;
    }
    if (dev < 0 || dev >= (int)ctx->devs.size()) return -EINVAL;
    if (n && (!fb->frames || !fb->linear_len || !fb->ifindex || (!fb->offsets && !fb->stride))) {
        set_error("classify_frames: bad arguments");
        return -EINVAL;
    }
    Device &d = ctx->devs[dev];
    std::shared_ptr<DeviceEpoch> ep;
    {
        std::lock_guard<std::mutex> lk(ctx->epoch_mu);
        ep = d.epoch;
    }
    DeviceGuard g(d.ordinal);
    if (!g.ok) {
        set_error("hipSetDevice failed");
        return -ENODEV;
    }
    if (ep->wait_ready(static_cast<hipStream_t>(stream))) {
        set_error("classify_frames: stream wait on the epoch's upload failed");
        return -EIO;
    }
    const bool evs = ex && ex->events_count;
    if (infw_launch_classify_frames(&ep->view, fb, n, result_words, xdp_verdicts, d.stats, d.cus,
                                    static_cast<hipStream_t>(stream), evs ? ex->events : nullptr,
                                    evs ? ex->events_cap : 0, evs ? ex->events_count : nullptr,
                                    ctx->debug_lookup ? d.dbg_fp : nullptr, d.dbg_keys, d.dbg_count, kDbgSlots)) {
        set_error(std::string("classify_frames launch failed: ") + hipGetErrorString(hipGetLastError()));
        return -EIO;
    }
    ep->mark_use(static_cast<hipStream_t>(stream));
    return 0;
}

int infw_pack_frames_c(infw_ctx *ctx, int dev, const infw_frame_batch *fb, uint64_t n, const infw_batch_soa_c_out *out,
                       void *stream) {
    if (!ctx || !fb || !out) return -EINVAL;
    if (ctx->devs.empty()) {
        set_error("pack_frames_c: host-only context");
        return -ENODEV;
    }
    if (dev < 0 || dev >= (int)ctx->devs.size()) return -EINVAL;
    if (n && (!fb->frames || !fb->linear_len || !fb->ifindex || (!fb->offsets && !fb->stride) || !out->saddr4 ||
              !out->v6tail || !out->ifindex || !out->pkt_len || !out->meta || !out->l4word ||
              ((uintptr_t)out->v6tail & 3))) {
        set_error("pack_frames_c: bad arguments");
        return -EINVAL;
    }
    DeviceGuard g(ctx->devs[dev].ordinal);
    if (!g.ok) return -ENODEV;
    if (infw_launch_pack_frames(fb, n, nullptr, out, ctx->devs[dev].cus, static_cast<hipStream_t>(stream))) {
        set_error(std::string("pack launch failed: ") + hipGetErrorString(hipGetLastError()));
        return -EIO;
    }
    return 0;
}

int infw_events_capture(infw_ctx *ctx, int dev, const infw_frame_batch *fb, uint64_t n_frames,
                        const infw_event_rec *events, uint64_t events_cap, const uint64_t *events_count,
                        infw_event_sample *samples, void *stream) {
    if (!ctx || !fb) return -EINVAL;
    if (ctx->devs.empty()) {
        set_error("events_capture: host-only context");
        return -ENODEV;
    }
    if (dev < 0 || dev >= (int)ctx->devs.size()) return -EINVAL;
    if (events_cap && (!events || !events_count || !samples || ((uintptr_t)samples & 7) ||
                       (n_frames && (!fb->frames || !fb->linear_len || (!fb->offsets && !fb->stride))))) {
        set_error("events_capture: bad arguments");
        return -EINVAL;
    }
    DeviceGuard g(ctx->devs[dev].ordinal);
    if (!g.ok) return -ENODEV;
    if (infw_launch_event_samples(fb, events, events_cap, events_count, n_frames, samples, ctx->devs[dev].cus,
                                  static_cast<hipStream_t>(stream))) {
        set_error(std::string("events_capture launch failed: ") + hipGetErrorString(hipGetLastError()));
        return -EIO;
    }
    return 0;
}

int infw_set_launch(infw_ctx *ctx, int block, int scan_group, int blocks_per_cu) {
    if (!ctx || block < 64 || block > 1024 || block % 64 || (scan_group != 0 && scan_group != 1 && scan_group != 4 && scan_group != 8) ||
        blocks_per_cu < 1 || blocks_per_cu > 32)
        return -EINVAL;
    ctx->block = block;
    ctx->group = scan_group;
    ctx->blocks_per_cu = blocks_per_cu;
    return 0;
}

int infw_get_launch(infw_ctx *ctx, int *block, int *scan_group, int *blocks_per_cu) {
    if (!ctx || !block || !scan_group || !blocks_per_cu) return -EINVAL;
    *block = ctx->block;
    *scan_group = ctx->group;
    *blocks_per_cu = ctx->blocks_per_cu;
    return 0;
}

int infw_stats_read(infw_ctx *ctx, uint32_t rule_id, ruleStatistics_st *per_slot, int *n_slots) {
    if (!ctx || !per_slot) return -EINVAL;
    if (rule_id >= INFW_MAX_TARGETS) return -ENOENT;
    for (size_t i = 0; i < ctx->devs.size(); i++) {
        DeviceGuard g(ctx->devs[i].ordinal);
        HIP_OK(hipDeviceSynchronize());
        HIP_OK(hipMemcpy(&per_slot[i], ctx->devs[i].stats + 4 * rule_id, sizeof(ruleStatistics_st),
                         hipMemcpyDeviceToHost));
    }
    if (n_slots) *n_slots = (int)ctx->devs.size();
    return 0;
}

int infw_stats_read_all(infw_ctx *ctx, ruleStatistics_st out[INFW_MAX_TARGETS]) {
    if (!ctx || !out) return -EINVAL;
    memset(out, 0, sizeof(ruleStatistics_st) * INFW_MAX_TARGETS);
    std::vector<ruleStatistics_st> tmp(INFW_MAX_TARGETS);
    for (auto &d : ctx->devs) {
        DeviceGuard g(d.ordinal);
        HIP_OK(hipDeviceSynchronize());
        HIP_OK(hipMemcpy(tmp.data(), d.stats, sizeof(ruleStatistics_st) * INFW_MAX_TARGETS,
                         hipMemcpyDeviceToHost));
        for (int k = 0; k < INFW_MAX_TARGETS; k++) {
            out[k].allow_stats.packets += tmp[k].allow_stats.packets;
            out[k].allow_stats.bytes += tmp[k].allow_stats.bytes;
            out[k].deny_stats.packets += tmp[k].deny_stats.packets;
            out[k].deny_stats.bytes += tmp[k].deny_stats.bytes;
        }
    }
    return 0;
}

int infw_stats_reset(infw_ctx *ctx) {
    if (!ctx) return -EINVAL;
    for (auto &d : ctx->devs) {
        DeviceGuard g(d.ordinal);
        HIP_OK(hipDeviceSynchronize());
        HIP_OK(hipMemset(d.stats, 0, sizeof(ruleStatistics_st) * INFW_MAX_TARGETS));
    }
    return 0;
}

int infw_stats_bind(infw_ctx *ctx, int dev, uint64_t *device_stats) {
    if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return -EINVAL;
    if (((uintptr_t)device_stats & 7) != 0) return -EINVAL;
    ctx->devs[dev].stats = device_stats ? device_stats : ctx->devs[dev].stats_own;
    return 0;
}

int infw_stats_device_ptr(infw_ctx *ctx, int dev, uint64_t **device_stats) {
    if (!ctx || !device_stats || dev < 0 || dev >= (int)ctx->devs.size()) return -EINVAL;
    *device_stats = ctx->devs[dev].stats;
    return 0;
}

}  // extern "C"
