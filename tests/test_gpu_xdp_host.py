"""The host-fed AF_XDP path (infw_classify_xdp_host): RX rings over a umem in ordinary (pageable) host memory, read by
the context's packer threads, the packed tuples pipelined through the device in chunks.

One ring per interface (a socket is bound to one interface queue), rings of ragged sizes (empty, one frame, a partial
group, several chunks plus a partial one) so that chunks run from one ring into the next and the host slots are
reused many times; aligned and unaligned descriptor modes.  Result words, verdicts and per-rule counters must equal
the oracle's on the same frames (oracle/infw_oracle.c from the frame bytes), and equal infw_classify_xdp's — the
kernel reading the same rings in place — when the memory is registered."""
import mmap

import numpy as np
import pytest
import torch

import infw
from infw import workloads as W

from parity import oracle_for
from test_hostpack_cpu import ring

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.fixture(scope="module")
def setup():
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=50000, n_templates=256)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    return wl, clf, oracle_for(wl)


def rings_of(wl, start, sizes, mode, seed):
    """Frames of packets [start, ...) split by interface into rings of the given sizes (one ifindex per ring)."""
    rng = np.random.default_rng(seed)
    hdr, cap, pl, ifx = wl.frames(start, 4 * sum(sizes) + 4096)
    out, used = [], np.zeros(hdr.shape[0], bool)
    for r, size in enumerate(sizes):
        v = np.unique(ifx)[r % len(np.unique(ifx))]
        idx = np.nonzero((ifx == v) & ~used)[0][:size]
        assert idx.size == size
        used[idx] = True
        umem, desc = ring(hdr[idx], pl[idx], mode, rng)
        out.append(dict(ifindex=int(v), hdr=hdr[idx], pl=pl[idx], umem=umem, desc=desc))
    return out


def oracle_of(m, rings):
    """Per-ring expected result words and verdicts, and the counters of all rings together."""
    hdr = np.concatenate([r["hdr"] for r in rings])
    pl = np.concatenate([r["pl"] for r in rings])
    ifx = np.concatenate([np.full(r["pl"].size, r["ifindex"], np.uint32) for r in rings])
    want, wver, wst, _ = m.classify_frames(hdr, pl, pl, ifx, nthreads=8)
    cut = np.cumsum([0] + [r["pl"].size for r in rings])
    return [want[a:b] for a, b in zip(cut, cut[1:])], [wver[a:b] for a, b in zip(cut, cut[1:])], wst


def run_host(clf, rings, chunk, pinned_out=False):
    res, ver, args = [], [], []
    for r in rings:
        n = r["pl"].size
        if pinned_out:
            rr = torch.full((max(n, 1),), -1, dtype=torch.int32).pin_memory()
            vv = torch.full((max(n, 1),), 7, dtype=torch.uint8).pin_memory()
        else:  # ordinary pageable host memory
            rr, vv = torch.full((max(n, 1),), -1, dtype=torch.int32), torch.full((max(n, 1),), 7, dtype=torch.uint8)
        res.append(rr)
        ver.append(vv)
        args.append((r["umem"], r["desc"], n, r["ifindex"], rr, vv))
    clf.stats_reset()
    clf.classify_xdp_host(args, chunk=chunk)
    return [x[:r["pl"].size].numpy().view(np.uint32) for x, r in zip(res, rings)], \
        [x[:r["pl"].size].numpy() for x, r in zip(ver, rings)], clf.stats_read_all()


@pytest.mark.parametrize("mode", ["aligned", "unaligned"])
@pytest.mark.parametrize("chunk", [512, 0])
def test_xdp_host_matches_oracle(setup, mode, chunk):
    wl, clf, m = setup
    sizes = [0, 1, 29, 3 * 512 + 64 + 17, 40000 + 3, 1200]
    rings = rings_of(wl, 1000 + chunk, sizes, mode, seed=7 + chunk)
    want, wver, wst = oracle_of(m, rings)
    got, gver, gst = run_host(clf, rings, chunk, pinned_out=(chunk == 0))
    for i, (g, w) in enumerate(zip(got, want)):
        bad = np.nonzero(g != w)[0]
        assert bad.size == 0, (mode, chunk, i, bad[:5], g[bad[:5]], w[bad[:5]])
        assert np.array_equal(gver[i], wver[i]), (mode, chunk, i)
    assert np.array_equal(gst, wst)
    both = np.concatenate(want)
    assert (both & 0xFF).astype(bool).mean() > 0.3 and len({r["ifindex"] for r in rings}) > 1


def test_xdp_host_threads_and_chunks_agree(setup):
    """Any packer thread count and chunk size gives the same words and counters (the split of a chunk among the
    threads and the slot reuse are invisible)."""
    wl, clf, m = setup
    rings = rings_of(wl, 50000, [70001, 333], "aligned", seed=9)
    want, _, wst = oracle_of(m, rings)
    try:
        for threads, chunk in ((1, 4096), (3, 1024), (16, 512), (0, 0)):
            clf.set_option("host_threads", threads)
            got, _, gst = run_host(clf, rings, chunk)
            assert all(np.array_equal(g, w) for g, w in zip(got, want)), (threads, chunk)
            assert np.array_equal(gst, wst), (threads, chunk)
    finally:
        clf.set_option("host_threads", 0)


def test_xdp_host_equals_device_read(setup):
    """The same rings in registered memory: infw_classify_xdp (the kernel reading umem and ring over PCIe) and
    infw_classify_xdp_host give identical result words and counters."""
    wl, clf, m = setup
    rings = rings_of(wl, 90000, [5000, 7777], "unaligned", seed=11)
    got, _, gst = run_host(clf, rings, 0)
    clf.stats_reset()
    dres = []
    for r in rings:
        u = torch.from_numpy(r["umem"]).pin_memory()
        d = torch.from_numpy(r["desc"].view(np.int32)).pin_memory()
        out = torch.empty(r["pl"].size, dtype=torch.int32, device="cuda:0")
        clf.classify_xdp(u, d, r["pl"].size, r["ifindex"], results=out)
        torch.cuda.synchronize()
        dres.append(out.cpu().numpy().view(np.uint32))
    assert all(np.array_equal(g, d) for g, d in zip(got, dres))
    assert np.array_equal(clf.stats_read_all(), gst)


def test_xdp_device_read_rejects_pageable(setup):
    """infw_classify_xdp on pageable memory (a socket's mmapped ring as it is) returns -EFAULT instead of faulting
    the GPU; registered with infw_host_register, the same memory classifies."""
    wl, clf, _ = setup
    r = rings_of(wl, 123, [300], "aligned", seed=13)[0]
    maps, arrs = [], []
    for a in (r["umem"], r["desc"]):  # the process's own anonymous mappings (page-aligned), as a daemon's
        mm = mmap.mmap(-1, max(a.nbytes, 4096))
        b = np.frombuffer(mm, dtype=a.dtype, count=a.size).reshape(a.shape)
        b[...] = a
        maps.append(mm)
        arrs.append(b)
    u, d = torch.from_numpy(arrs[0]), torch.from_numpy(arrs[1].view(np.int32))  # pageable CPU tensors
    out = torch.empty(300, dtype=torch.int32, device="cuda:0")
    with pytest.raises(infw.InfwError) as e:
        clf.classify_xdp(u, d, 300, r["ifindex"], results=out)
    assert e.value.errno == 14
    for b in arrs:
        clf.host_register(b)
    try:
        clf.classify_xdp(u, d, 300, r["ifindex"], results=out)
        torch.cuda.synchronize()
        ref, _, _ = run_host(clf, [r], 0)
        assert np.array_equal(out.cpu().numpy().view(np.uint32), ref[0])
    finally:
        for b in arrs:
            clf.host_unregister(b)
        del u, d, b, arrs


def test_xdp_host_rejects_bad_rings(setup):
    _, clf, _ = setup
    from infw import _native as N
    arr = (N.XdpRing * 1)()
    arr[0] = N.XdpRing(None, None, 5, 1, 0, None, None)  # frames but no umem
    assert N.lib.infw_classify_xdp_host(clf._ctx, 0, arr, 1, 0) == -22
    u = np.zeros(4096, np.uint8)
    d = np.zeros((1, 4), np.uint32)
    arr[0] = N.XdpRing(u.ctypes.data, d.ctypes.data, 1, 1, 1, None, None)  # flags != 0
    assert N.lib.infw_classify_xdp_host(clf._ctx, 0, arr, 1, 0) == -22
    assert N.lib.infw_classify_xdp_host(clf._ctx, 0, arr, 0, 0) == 0  # no rings: nothing to do
    assert N.lib.infw_classify_xdp_host(clf._ctx, 5, arr, 1, 0) == -22  # no such device slot


def test_xdp_host_small_calls_back_to_back(setup):
    """A daemon's polling shape: many small calls in a row, each taking a few descriptors from every ring (chunks of
    several interfaces; calls of one unit wake no packer thread), between large ones (packers still waking up from
    the last job).  Every call's words equal the oracle's; the median per-call latency is printed."""
    import time
    wl, clf, m = setup
    rings = rings_of(wl, 7000, [3000, 2500, 6000], "aligned", seed=17)
    want, _, _ = oracle_of(m, rings)
    rng = np.random.default_rng(5)
    res = [np.full(r["pl"].size, 0xFFFFFFFF, np.uint32) for r in rings]
    at = [0] * len(rings)
    lat = []
    while any(a < r["pl"].size for a, r in zip(at, rings)):
        args = []
        for i, r in enumerate(rings):
            q = int(rng.integers(1, 300))
            a, b = at[i], min(r["pl"].size, at[i] + q)
            if a < b:
                args.append((r["umem"], r["desc"][a:b], b - a, r["ifindex"], res[i][a:b], None))
            at[i] = b
        t0 = time.perf_counter()
        clf.classify_xdp_host(args)
        lat.append(time.perf_counter() - t0)
        if len(lat) % 10 == 0:  # a large call in between
            big = rings_of(wl, 90000 + len(lat), [20000], "unaligned", seed=len(lat))
            run_host(clf, big, 0)
    for g, w in zip(res, want):
        bad = np.nonzero(g != w)[0]
        assert bad.size == 0, (bad[:5], g[bad[:5]], w[bad[:5]])
    print(f"[xdp_host small calls] {len(lat)} calls of up to 3 x 300 descriptors: median "
          f"{np.median(lat) * 1e6:.0f} us, p90 {np.percentile(lat, 90) * 1e6:.0f} us per call")


def test_xdp_host_optional_outputs(setup):
    """Rings that want only verdicts, only result words, or neither (statistics only) in one call, sharing chunks:
    each ring gets exactly what it asked for and the counters still cover every ring."""
    wl, clf, m = setup
    rings = rings_of(wl, 31000, [700, 900, 1100], "aligned", seed=23)
    want, wver, wst = oracle_of(m, rings)
    res = np.full(900, 0xFFFFFFFF, np.uint32)
    ver = np.full(700, 7, np.uint8)
    args = [(rings[0]["umem"], rings[0]["desc"], 700, rings[0]["ifindex"], None, ver),
            (rings[1]["umem"], rings[1]["desc"], 900, rings[1]["ifindex"], res, None),
            (rings[2]["umem"], rings[2]["desc"], 1100, rings[2]["ifindex"], None, None)]
    clf.stats_reset()
    clf.classify_xdp_host(args, chunk=512)  # chunks of 512: every chunk boundary inside or between rings
    assert np.array_equal(ver, wver[0]) and np.array_equal(res, want[1])
    assert np.array_equal(clf.stats_read_all(), wst)


def test_xdp_host_deny_events_from_device_results(setup):
    """The host-fed path's deny events (include/infw_host.h infw_xdp_host_events) from the result words the device
    returned: every ring's perf samples equal the oracle's (kernel.c:392-399) for the same frames, and their number
    equals the deny counters' packet total."""
    wl, clf, m = setup
    rings = rings_of(wl, 60000, [3000, 4000], "unaligned", seed=29)
    got, _, gst = run_host(clf, rings, 0)
    total = 0
    for r, res in zip(rings, got):
        addr = r["desc"][:, 0].astype(np.uint64) | r["desc"][:, 1].astype(np.uint64) << np.uint64(32)
        offs = (addr & np.uint64((1 << 48) - 1)) + (addr >> np.uint64(48))
        _, want = m.collect_event_samples(r["umem"], offs, r["pl"], r["pl"],
                                          np.full(len(offs), r["ifindex"], np.uint32))
        samples, k = infw.xdp_host_events(r["umem"], r["desc"], r["ifindex"], res, len(want) + 1)
        assert k == len(want) and np.array_equal(samples[:k], want)
        total += k
    assert total == int(gst[:, 2].sum()) and total > 0  # deny packets counted = events emitted


def test_xdp_host_two_slots_concurrently(setup):
    """A daemon with two device slots (both on device 0 here) calls infw_classify_xdp_host from two threads at once,
    each slot with its own packer pool and pinned slots: every call's words equal the oracle's, and each slot's
    counters are its own rings' (the per-slot statistics a reader sums like per-CPU slots)."""
    import threading
    wl, _, m = setup
    clf = infw.Classifier(devices=[0, 0], max_entries=wl.n_entries + 16, options={"host_threads": 4})
    wl.load_into(clf)
    clf.commit()
    work = [rings_of(wl, 200000 + 50000 * s, [9000, 7000], "aligned", seed=31 + s) for s in range(2)]
    want = [oracle_of(m, rs) for rs in work]
    outs = [[np.full(r["pl"].size, 0xFFFFFFFF, np.uint32) for r in rs] for rs in work]
    errors = []

    def run(slot):
        try:
            for _ in range(5):
                clf.classify_xdp_host([(r["umem"], r["desc"], r["pl"].size, r["ifindex"], o, None)
                                       for r, o in zip(work[slot], outs[slot])], chunk=4096, dev=slot)
        except BaseException as e:  # surfaced below
            errors.append(e)
    clf.stats_reset()
    th = [threading.Thread(target=run, args=(s,)) for s in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    for s in range(2):
        assert all(np.array_equal(g, w) for g, w in zip(outs[s], want[s][0])), s
    per_rule = [clf.stats_read(rule) for rule in range(1, 100)]
    for s in range(2):  # slot s counted its own rings five times
        got = np.array([[p[s].allow_packets, p[s].allow_bytes, p[s].deny_packets, p[s].deny_bytes] for p in per_rule],
                       np.uint64)
        assert np.array_equal(got, want[s][2][1:100] * np.uint64(5)), s
    clf.close()


@pytest.mark.parametrize("chunk", [512, 0])
def test_bursts_host_match_oracle(setup, chunk):
    """infw_classify_bursts_host (include/infw_host.h): DPDK-style bursts — one pointer per frame, first segments
    shorter than the frame for most, one port per burst, ragged sizes — give the oracle's result words, verdicts and
    counters for the same frames (linear length = the first segment's, frame length = the whole frame's)."""
    from test_hostpack_cpu import _burst_of
    wl, clf, m = setup
    hdr, cap, pl, ifx = wl.frames(300000 + chunk, 30000)
    rng = np.random.default_rng(41 + chunk)
    cap = np.minimum(cap, rng.choice(np.array([60, 64, 128, 30, 9000], np.uint32), cap.size,
                                     p=[.3, .3, .2, .05, .15])).astype(np.uint32)
    bursts, keep, want_r, want_v = [], [], [], []
    for port, size in zip(np.unique(ifx)[:3], [1, 4097, 9000]):
        idx = np.nonzero(ifx == port)[0][:size]
        buf, b, _ = _burst_of(hdr[idx], cap[idx], pl[idx], int(port))
        b.results = np.full(idx.size, 0xFFFFFFFF, np.uint32)
        b.verdicts = np.full(idx.size, 7, np.uint8)
        bursts.append(b)
        keep.append(buf)
        r, v, _, _ = m.classify_frames(hdr[idx], cap[idx], pl[idx], ifx[idx], nthreads=8)
        want_r.append(r)
        want_v.append(v)
    allidx = np.concatenate([np.nonzero(ifx == port)[0][:size] for port, size in zip(np.unique(ifx)[:3], [1, 4097, 9000])])
    _, _, wst, _ = m.classify_frames(hdr[allidx], cap[allidx], pl[allidx], ifx[allidx], nthreads=8)
    clf.stats_reset()
    clf.classify_bursts_host(bursts, chunk=chunk)
    for b, r, v in zip(bursts, want_r, want_v):
        assert np.array_equal(b.results, r) and np.array_equal(b.verdicts, v)
    assert np.array_equal(clf.stats_read_all(), wst)


@pytest.mark.parametrize("arrays", ["own", "slices"])
def test_small_bursts_host_match_oracle(setup, arrays):
    """rx_burst-sized bursts (1..40 frames, ports interleaved) through infw_classify_bursts_host: thousands of segments
    per chunk.  "own": every burst its own result / verdict arrays — a chunk's words come back in one copy and are
    scattered on the host (abi.cpp xdp_scatter); "slices": the bursts' arrays are consecutive slices of one array per
    call — adjacent destinations merge into one copy (xdp_copies).  Both: the oracle's words, verdicts and counters."""
    from test_hostpack_cpu import _burst_of
    wl, clf, m = setup
    n = 30000
    hdr, cap, pl, ifx = wl.frames(900000 + (arrays == "own") * n, n)
    rng = np.random.default_rng(5)
    cap = np.minimum(cap, rng.choice(np.array([60, 64, 128, 9000], np.uint32), n, p=[.3, .3, .2, .2])).astype(np.uint32)
    buf, whole, _ = _burst_of(hdr, cap, pl, 0)
    want_r, want_v, wst, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
    res = np.full(n, 0xFFFFFFFF, np.uint32)
    ver = np.full(n, 7, np.uint8)
    bursts, at = [], 0
    while at < n:  # a burst holds frames of one port: cut where the port changes or at its size
        size = int(rng.integers(1, 41))
        hi = at + 1
        while hi < min(n, at + size) and ifx[hi] == ifx[at]:
            hi += 1
        r = res[at:hi] if arrays == "slices" else np.full(hi - at, 0xFFFFFFFF, np.uint32)
        v = ver[at:hi] if arrays == "slices" else np.full(hi - at, 7, np.uint8)
        bursts.append((at, hi, infw.Burst(whole.frames[at:hi], cap[at:hi], pl[at:hi], int(ifx[at]), results=r,
                                          verdicts=v)))
        at = hi
    assert len(bursts) > 2000
    arr = infw.BurstArray([b for _, _, b in bursts])
    for chunk in (4096, 0):
        clf.stats_reset()
        clf.classify_bursts_host(arr, chunk=chunk)
        for lo, hi, b in bursts:
            assert np.array_equal(b.results, want_r[lo:hi]) and np.array_equal(b.verdicts, want_v[lo:hi]), (chunk, lo)
        assert np.array_equal(clf.stats_read_all(), wst)
        for _, _, b in bursts:
            b.results[:] = 0xFFFFFFFF
            b.verdicts[:] = 7
    del buf


def test_many_bursts_threaded_cut_match_oracle(setup):
    """A call of more than 65536 bursts (1..2 frames each, ports interleaved, result arrays slices of one array with a
    gap now and then): the cut runs in two passes split over several threads (hostfeed.cpp cut_chunks), and the call
    still gives the oracle's words, verdicts and counters."""
    from test_hostpack_cpu import _burst_of
    wl, clf, m = setup
    n = 110000
    hdr, cap, pl, ifx = wl.frames(2000000, n)
    buf, whole, _ = _burst_of(hdr, cap, pl, 0, stride=128)
    want_r, want_v, wst, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
    rng = np.random.default_rng(77)
    res = np.full(n + n // 8, 0xFFFFFFFF, np.uint32)
    bursts, at, gap = [], 0, 0
    while at < n:
        hi = at + 1 if rng.random() < 0.5 or at + 1 == n or ifx[at + 1] != ifx[at] else at + 2
        gap += rng.random() < 0.05  # a burst whose words do not continue the previous one's
        bursts.append((at, hi, gap, infw.Burst(whole.frames[at:hi], cap[at:hi], pl[at:hi], int(ifx[at]),
                                               results=res[at + gap:hi + gap])))
        at = hi
    assert len(bursts) > 65536
    clf.stats_reset()
    clf.classify_bursts_host(infw.BurstArray([b for _, _, _, b in bursts]))
    for lo, hi, _, b in bursts:
        assert np.array_equal(b.results, want_r[lo:hi]), lo
    assert np.array_equal(clf.stats_read_all(), wst)
    del buf
