"""The two-phase classify form (classify.hip: classify_kernel<..., kSplit> writes each packet's decision-line
address, decide_kernel reads those words and the decision lines as independent gathers) against the oracle: result
words, verdicts and per-rule counters.  It is chosen per launch for epochs with many distinct rule lists (abi.cpp
split_of, option split_min_mb); the option split=1 forces it onto every table shape here so each phase-1 instantiation
(lean epochs: per-list part counts, /16 words) runs -- non-lean epochs and the family-compact layout keep their fused
kernel, which must give the same results -- and the distinct-lists workload takes it by default.  Its per-packet
scratch comes from a pool the context owns: the device default pool is left as it was."""
import numpy as np
import pytest
import torch

import infw
from infw import workloads as W
from infw.batch import SoaBatch
from parity import assert_parity, check_cfg, gpu_run, stats_from_results

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


CASES = [  # (cfg, n packets, prefixes, templates, layout)
    (W.CFG2_MIXED_1M, 1 << 20, 100000, 4096, "standard"),   # lean, per-list part counts
    (W.CFG2_MIXED_1M, 1 << 20, 100000, 4096, "compact"),
    (W.CFG1_V4_10K, 1 << 20, 0, 0, "standard"),              # /16 words
    (W.CFG4_ADVERSARIAL, 1 << 20, 0, 0, "standard"),         # IPv6-heavy, leaf lines
    (W.CFG4_ADVERSARIAL, 1 << 19, 0, 0, "compact"),
    (W.CFG0_DEMO, 1 << 18, 0, 0, "standard"),
]


@pytest.mark.parametrize("cfg,n,npfx,ntmpl,layout", CASES)
def test_split_parity(monkeypatch, cfg, n, npfx, ntmpl, layout):
    monkeypatch.setitem(infw.DEFAULT_OPTIONS, "split", int("1"))
    r = check_cfg(cfg, n, n_prefixes=npfx, n_templates=ntmpl, layout=layout)
    assert r["clf"].info()["split"] == 1
    assert_parity(r, f"split cfg{cfg} {layout}")


def test_split_distinct_lists_default(monkeypatch):
    """One rule list per key at 100k keys with a 64-MiB threshold: the epoch picks the split form by itself."""
    monkeypatch.setitem(infw.DEFAULT_OPTIONS, "split_min_mb", int("64"))
    r = check_cfg(W.CFG2_MIXED_1M, 1 << 20, n_prefixes=100000, n_templates=100000)
    assert r["clf"].info()["split"] == 1 and r["clf"].info()["n_lists"] > 50000
    assert_parity(r, "split distinct lists")


@pytest.mark.parametrize("n", [1, 63, 65, 511, 513, 4097, 100003])
def test_split_ragged(monkeypatch, n):
    monkeypatch.setitem(infw.DEFAULT_OPTIONS, "split", int("1"))
    r = check_cfg(W.CFG2_MIXED_1M, n, n_prefixes=20000, n_templates=128, start=77)
    assert_parity(r, f"split n={n}")


@pytest.mark.parametrize("flush_tiles", ["1", None])
def test_split_counter_paths(monkeypatch, flush_tiles):
    """Frame lengths that do not fit the phase-1 word (>= 0xFFFF B: phase 2 reads pkt_len) and >= 2^20 B (device
    counters directly), with workgroups flushing after every tile or at the default interval."""
    monkeypatch.setitem(infw.DEFAULT_OPTIONS, "split", int("1"))
    if flush_tiles:
        monkeypatch.setitem(infw.DEFAULT_OPTIONS, "stat_flush_tiles", int(flush_tiles))
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=50000, n_templates=256)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    assert clf.info()["split"] == 1
    dev = torch.device("cuda", 0)
    n = 1 << 18
    b = SoaBatch.empty(n, dev)
    wl.gen_device(b, 999, 0)
    torch.cuda.synchronize()
    ref_res, ref_ver = gpu_run(clf, b, n)  # lengths only change counters, not result words
    g = torch.Generator(device="cpu").manual_seed(11)
    sel = torch.rand(n, generator=g)
    pl = b.pkt_len.cpu().to(torch.int64)
    mid = sel < 0.02
    big = sel > 0.99
    pl[mid] = torch.randint(0xFFFF, 1 << 20, (n,), generator=g, dtype=torch.int64)[mid]
    pl[big] = torch.randint(1 << 20, (1 << 32) - 1, (n,), generator=g, dtype=torch.int64)[big]
    b.pkt_len.copy_(pl.to(torch.int32).to(dev))
    clf.stats_reset()
    gres, gver = gpu_run(clf, b, n)
    assert np.array_equal(gres, ref_res) and np.array_equal(gver, ref_ver)
    plen = b.pkt_len.cpu().numpy().view(np.uint32)
    assert np.array_equal(clf.stats_read_all(), stats_from_results(gres, plen))


def test_split_concurrent_streams(monkeypatch):
    """Two batches on two streams at once: each call's phase-1 words live in its own stream-ordered scratch."""
    monkeypatch.setitem(infw.DEFAULT_OPTIONS, "split", int("1"))
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=50000, n_templates=256)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    dev = torch.device("cuda", 0)
    n = 1 << 20
    bs = [SoaBatch.empty(n, dev) for _ in range(2)]
    for k, b in enumerate(bs):
        wl.gen_device(b, k * n, 0)
    torch.cuda.synchronize()
    want = [gpu_run(clf, b, n)[0] for b in bs]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(2)]
    for _ in range(3):
        for b, s, o in zip(bs, streams, outs):
            clf.classify(b, results=o, stream=s)
        torch.cuda.synchronize()
        for o, w in zip(outs, want):
            assert np.array_equal(o.cpu().numpy().view(np.uint32), w)


def _hip():
    """The HIP runtime this process already runs (torch's), through ctypes."""
    import ctypes as C
    path = next(l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64.so" in l)
    hip = C.CDLL(path)
    hip.hipDeviceGetDefaultMemPool.argtypes = [C.POINTER(C.c_void_p), C.c_int]
    hip.hipMemPoolGetAttribute.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    return hip


def test_split_leaves_the_default_pool_alone(monkeypatch):
    """The two-phase scratch is allocated from the context's own pool: the device default pool's release threshold
    (which every hipMallocAsync user of the process shares) is the same before and after split launches."""
    import ctypes as C
    monkeypatch.setitem(infw.DEFAULT_OPTIONS, "split", 1)
    torch.zeros(1, device="cuda:0")
    hip = _hip()

    def threshold():
        pool, v = C.c_void_p(), C.c_uint64(0)
        assert hip.hipDeviceGetDefaultMemPool(C.byref(pool), 0) == 0
        assert hip.hipMemPoolGetAttribute(pool, 4, C.byref(v)) == 0  # hipMemPoolAttrReleaseThreshold
        return v.value

    before = threshold()
    r = check_cfg(W.CFG2_MIXED_1M, 1 << 20, n_prefixes=50000, n_templates=256)
    assert r["clf"].variant().endswith("+decide.512")
    assert_parity(r, "split, own pool")
    r["clf"].classify(r["batch"])
    torch.cuda.synchronize()
    assert threshold() == before
