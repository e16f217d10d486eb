"""GPU parity: the HIP classifier (through the C ABI) against the oracle.

Bit-exact on result words ((ruleId & 0xFFFFFF) << 8 | action), XDP verdicts and
the per-rule allow/deny packet/byte counters, for every BASELINE config at
sizes the oracle finishes in seconds, plus size-independent properties at the
bench sizes.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import infw  # noqa: E402
from infw import workloads as W  # noqa: E402
from infw.batch import SoaBatch  # noqa: E402

from parity import assert_parity, check_cfg, gpu_run, oracle_for, stats_from_results  # noqa: E402

_SHORT = {"dir24": 0, "compressed": 1}  # option short_table (include/infw.h)


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.mark.parametrize("cfg,n,npfx,ntmpl", [
    (W.CFG0_DEMO, 1 << 20, 0, 0),            # configs[0]: demo-1 sample on 1M packets
    (W.CFG1_V4_10K, 1 << 20, 0, 0),          # configs[1] table at full size
    (W.CFG2_MIXED_1M, 1 << 19, 100000, 512),  # configs[2] shape, reduced table
    (W.CFG2_MIXED_1M, 1 << 19, 100000, 100000),  # configs[2] distinct-lists variant: one list per key
    (W.CFG4_ADVERSARIAL, 1 << 19, 20000, 64),
    (W.CFG4_ADVERSARIAL, 1 << 19, 100000, 0),  # configs[4] at 100k prefixes (its bench default table)
])
def test_parity_configs(cfg, n, npfx, ntmpl):
    r = check_cfg(cfg, n, npfx, ntmpl)
    assert_parity(r, f"cfg{cfg}")
    # the workload must exercise the path: matches of both actions
    acts = np.bincount(r["ores"] & 0xFF, minlength=3)
    assert acts[1] + acts[2] > 0


@pytest.mark.parametrize("half", ["0", "1"])
def test_parity_dt_half_reads(monkeypatch, half):
    """Decision lines read half-first (INFW_DT_HALF=1: the first 32 B, the second half only for roots, u32 leaves and
    compact leaves of > 9 segments past their key 8; the compiler's choice for configs[1]-like epochs, run by the
    /16-word kernel shape) or whole (0): bit-exact either way on configs[1]; on configs[2] (100k) and [4] (20k) rule
    lists in that shape (/16 words forced, no per-list part counts: leaves of up to 20 segments, root entries); and on
    an IPv4 table of rule values with ids past 127 and actions outside {1, 2} (u32-form leaves)."""
    import random
    import struct
    import orc
    from test_compiler_cpu import _val
    from test_incremental_cpu import _packets_for
    monkeypatch.setitem(infw.DEFAULT_OPTIONS, "dt_half", int(half))
    r = check_cfg(W.CFG1_V4_10K, 1 << 18)
    assert r["clf"].info()["dt_half_reads"] == int(half) and r["clf"].info()["d16"] == 1
    assert_parity(r, f"cfg1-dt-half{half}")
    monkeypatch.setitem(infw.DEFAULT_OPTIONS, "d16", int("1"))
    monkeypatch.setitem(infw.DEFAULT_OPTIONS, "dt_adapt", int("0"))
    for cfg, npfx, ntmpl in ((W.CFG2_MIXED_1M, 100000, 512), (W.CFG4_ADVERSARIAL, 20000, 64)):
        r = check_cfg(cfg, 1 << 18, npfx, ntmpl)
        assert r["clf"].info()["dt_half_reads"] == int(half) and r["clf"].info()["d16"] == 1
        assert_parity(r, f"cfg{cfg}-dt-half{half}")
    rng = random.Random(21)
    ents = []
    for i in range(3000):
        L = rng.choice([16, 18, 20, 24, 28, 32])
        a = rng.getrandbits(32) & (~((1 << (32 - L)) - 1) & 0xFFFFFFFF)
        ents.append((struct.pack("<II", L + 32, rng.choice([3, 4])) + a.to_bytes(4, "big") + bytes(12), _val(rng, i)))
    clf = infw.Classifier(devices=[0])
    m = orc.OracleMap()
    for k, v in ents:
        assert clf.update_rc(infw.LpmIpKeySt.from_buffer_copy(k), infw.RulesValSt.from_buffer_copy(v)) == m.update(k, v)
    clf.commit()
    assert clf.info()["dt_half_reads"] == int(half) and clf.info()["d16"] == 1
    hdr, cap, pl, ifx = _packets_for([k for k, _ in ents], rng, 8)
    want, _, _, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
    got, _ = gpu_run(clf, SoaBatch.from_tuples(W.pack_frames(hdr, cap, pl, ifx), torch.device("cuda", 0)), len(ifx))
    assert np.array_equal(got, want)
    assert (want != 0).mean() > 0.3


def test_parity_cfg2_full_table_subsample():
    """configs[2] at its full 1M-prefix table, 256k packets from the middle of a shard."""
    r = check_cfg(W.CFG2_MIXED_1M, 1 << 18, start=(1 << 27) + 12345)
    assert_parity(r, "cfg2-full")


def test_ragged_and_empty_batches():
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=20000, n_templates=128)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    m = oracle_for(wl)
    dev = torch.device("cuda", 0)
    for n in (0, 1, 63, 64, 65, 255, 257, 1000, 4097):
        batch = SoaBatch.empty(max(n, 1), dev).slice(0, n)
        if n:
            wl.gen_device(batch, 777, 0)
        clf.stats_reset()
        gres, gver = gpu_run(clf, batch, n)
        hdr, cap, pl, ifx = wl.frames(777, n)
        ores, over, ostats, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=2)
        assert np.array_equal(gres, ores), n
        assert np.array_equal(gver, over), n
        assert np.array_equal(clf.stats_read_all(), ostats), n


def test_ipv4_ignores_saddr_tail_and_stats_accumulate():
    """IPv4 keys use only ip_data[0..3] (kernel.c:207-212): garbage in bytes 4..15 changes nothing;
    counters accumulate across batches like the per-CPU map (no reset between runs)."""
    r = check_cfg(W.CFG1_V4_10K, 1 << 16)
    batch, clf = r["batch"], r["clf"]
    b2 = SoaBatch(batch.saddr.clone(), batch.ifindex, batch.pkt_len, batch.meta, batch.l4word)
    b2.saddr[:, 4:] = torch.randint(0, 256, (batch.n, 12), dtype=torch.uint8, device=batch.device)
    v4 = (batch.meta & 0xFFFF) == 0x0800
    b2.saddr[~v4] = batch.saddr[~v4]
    gres2, _ = gpu_run(clf, b2, batch.n)
    assert np.array_equal(gres2, r["ores"])
    assert np.array_equal(clf.stats_read_all(), 2 * r["ostats"])


def test_epoch_swap_between_batches():
    """configs[4]: live table swap mid-stream — batch A on epoch 1, commit, batch B on epoch 2;
    the oracle applies the identical key updates between the same two batches."""
    wl = W.Workload(W.CFG4_ADVERSARIAL, n_prefixes=20000, n_templates=64)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 64)
    wl.load_into(clf)
    clf.commit()
    m = oracle_for(wl)
    dev = torch.device("cuda", 0)
    n = 1 << 18
    clf.stats_reset()
    a = SoaBatch.empty(n, dev)
    wl.gen_device(a, 0, 0)
    gres_a, _ = gpu_run(clf, a, n)
    hdr, cap, pl, ifx = wl.frames(0, n)
    ores_a, _, ost_a, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
    assert np.array_equal(gres_a, ores_a)
    # swap: delete every 3rd key, rewrite every 5th with another template, add /128 overrides
    keys = wl.keys_bytes().reshape(-1, 24)
    tmpl = wl.templates_bytes().reshape(-1, 1200)
    for i in range(0, keys.shape[0], 3):
        kb = keys[i].tobytes()
        rc1 = clf.delete_rc(infw.LpmIpKeySt.from_buffer_copy(kb))
        rc2 = m.delete(kb)
        assert rc1 == rc2
    for i in range(1, keys.shape[0], 5):
        kb, vb = keys[i].tobytes(), tmpl[(i * 7) % tmpl.shape[0]].tobytes()
        assert clf.update_rc(infw.LpmIpKeySt.from_buffer_copy(kb), infw.RulesValSt.from_buffer_copy(vb)) == \
            m.update(kb, vb)
    clf.commit()
    b = SoaBatch.empty(n, dev)
    wl.gen_device(b, n, 0)
    gres_b, _ = gpu_run(clf, b, n)
    hdr, cap, pl, ifx = wl.frames(n, n)
    ores_b, _, ost_b, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
    assert np.array_equal(gres_b, ores_b)
    assert np.array_equal(clf.stats_read_all(), ost_a + ost_b)  # stats persist across swaps


@pytest.mark.parametrize("ntmpl", [0, 1000000])
def test_full_size_properties(ntmpl):
    """configs[2] at the bench size (128M packets, full table; ntmpl 1M: the distinct-lists variant, one
    1200-B value per key): size-independent properties — per-rule counters == counters implied by the
    result words; two runs identical; the first and last 64k packets bit-exact against the oracle."""
    n = 1 << 27
    wl = W.Workload(W.CFG2_MIXED_1M, n_templates=ntmpl)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    dev = torch.device("cuda", 0)
    batch = SoaBatch.empty(n, dev)
    wl.gen_device(batch, 0, 0)
    res = torch.empty(n, dtype=torch.int32, device=dev)
    stats = torch.zeros((1024, 4), dtype=torch.int64, device=dev)
    clf.stats_bind(0, stats.data_ptr())
    clf.classify(batch, results=res)
    torch.cuda.synchronize()
    res1 = res.clone()
    # counters implied by result words, computed with torch on the device
    r = res.to(torch.int64) & 0xFFFFFFFF
    act, key = r & 0xFF, (r >> 8) & 0xFFFF
    plen = batch.pkt_len.to(torch.int64)
    want = torch.zeros((1024, 4), dtype=torch.int64, device=dev)
    for a, col in ((2, 0), (1, 2)):
        sel = (act == a) & (key < 1024)
        want[:, col] = torch.bincount(key[sel], minlength=1024)
        want[:, col + 1] = torch.zeros(1024, dtype=torch.int64, device=dev).index_add_(0, key[sel], plen[sel])
    assert torch.equal(stats, want)
    clf.classify(batch, results=res)
    torch.cuda.synchronize()
    assert torch.equal(res, res1)
    assert torch.equal(stats, 2 * want)
    clf.stats_bind(0, None)
    m = oracle_for(wl)
    for start in (0, n - (1 << 16)):
        hdr, cap, pl, ifx = wl.frames(start, 1 << 16)
        ores, _, _, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
        got = res1[start:start + (1 << 16)].cpu().numpy().view(np.uint32)
        assert np.array_equal(got, ores), start


def _implied_stats(res, batch, dev):
    """Per-rule counters implied by result words (kernel.c:441-456, :376-387), with torch on the device."""
    r = res.to(torch.int64) & 0xFFFFFFFF
    act, key = r & 0xFF, (r >> 8) & 0xFFFF
    plen = batch.pkt_len.to(torch.int64)
    want = torch.zeros((1024, 4), dtype=torch.int64, device=dev)
    for a, col in ((2, 0), (1, 2)):
        sel = (act == a) & (key < 1024)
        want[:, col] = torch.bincount(key[sel], minlength=1024)
        want[:, col + 1] = torch.zeros(1024, dtype=torch.int64, device=dev).index_add_(0, key[sel], plen[sel])
    return want


def test_cfg4_headline_scale_live_swap():
    """configs[4] (adversarial: /128 deepest-prefix hits, last-slot ICMPv6 type/code, aliasing keys) at the
    headline table size — 1M generated prefixes, 1.27M entries, ~800k IPv6 /32 groups — with a live swap: batch A
    (32M packets) on epoch 1, 2000 key edits committed incrementally, batch B on epoch 2.  Size-independent
    properties on both batches (device counters == counters implied by the result words), and the first and last
    64k packets of each batch bit-exact against the oracle with the identical edits applied between them."""
    import random
    wl = W.Workload(W.CFG4_ADVERSARIAL, n_prefixes=1000000)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 64)
    wl.load_into(clf)
    clf.commit()
    m = oracle_for(wl)
    dev = torch.device("cuda", 0)
    n = 1 << 25
    batch = SoaBatch.empty(n, dev)
    res = torch.empty(n, dtype=torch.int32, device=dev)
    stats = torch.zeros((1024, 4), dtype=torch.int64, device=dev)
    keys = wl.keys_bytes().reshape(-1, 24)
    tmpl = wl.templates_bytes().reshape(-1, 1200)
    rng = random.Random(4)
    for epoch, start in ((1, 0), (2, n)):
        if epoch == 2:
            for i in rng.sample(range(keys.shape[0]), 2000):
                kb = keys[i].tobytes()
                if rng.random() < 0.33:
                    assert clf.delete_rc(infw.LpmIpKeySt.from_buffer_copy(kb)) == m.delete(kb)
                else:
                    vb = tmpl[rng.randrange(tmpl.shape[0])].tobytes()
                    assert clf.update_rc(infw.LpmIpKeySt.from_buffer_copy(kb),
                                         infw.RulesValSt.from_buffer_copy(vb)) == m.update(kb, vb)
            clf.commit()
            assert clf.info()["commit_mode"] == infw.COMMIT_INCREMENTAL, clf.info()["full_reason"]
        wl.gen_device(batch, start, 0)
        stats.zero_()
        clf.stats_bind(0, stats.data_ptr())
        clf.classify(batch, results=res)
        torch.cuda.synchronize()
        clf.stats_bind(0, None)
        assert torch.equal(stats, _implied_stats(res, batch, dev)), epoch
        acts = torch.bincount((res & 0xFF).to(torch.int64), minlength=3).cpu().numpy()
        assert acts[1] > 0 and acts[2] > 0
        for off in (0, n - (1 << 16)):
            hdr, cap, pl, ifx = wl.frames(start + off, 1 << 16)
            ores, _, _, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
            assert np.array_equal(res[off:off + (1 << 16)].cpu().numpy().view(np.uint32), ores), (epoch, off)


def _gpu_events(clf, batch, cap):
    import ctypes as C
    from infw import _native as N
    ev = torch.zeros(cap * C.sizeof(N.EventRec), dtype=torch.uint8, device=batch.device)
    cnt = torch.zeros(1, dtype=torch.int64, device=batch.device)
    res = torch.empty(batch.n, dtype=torch.int32, device=batch.device)
    clf.classify_events(batch, ev, cnt, results=res)
    torch.cuda.synchronize()
    raw = ev.cpu().numpy().view(np.uint64).reshape(-1, 3)
    k = min(int(cnt.item()), cap)
    h = raw[:k, 0]
    rec = np.stack([raw[:k, 2], h & 0xFFFF, (h >> 16) & 0xFFFF, (h >> 32) & 0xFF, h >> 48, raw[:k, 1]], axis=1)
    return rec, int(cnt.item()), res.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("cfg,npfx,ntmpl", [(W.CFG2_MIXED_1M, 50000, 256), (W.CFG4_ADVERSARIAL, 20000, 64)])
def test_deny_events_match_oracle(cfg, npfx, ntmpl):
    """Deny-event stream (kernel.c:392-399): one record per rule DROP, identical to the oracle's perf records
    (event_hdr_st fields, captured length, packet index); overflow counts lost records like perf."""
    wl = W.Workload(cfg, n_prefixes=npfx, n_templates=ntmpl)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    m = oracle_for(wl)
    n = 1 << 18
    dev = torch.device("cuda", 0)
    batch = SoaBatch.empty(n, dev)
    wl.gen_device(batch, 4242, 0)
    hdr, cap, pl, ifx = wl.frames(4242, n)
    want = m.collect_events(hdr, cap, pl, ifx)
    assert want.shape[0] > 1000
    got, count, res = _gpu_events(clf, batch, n)
    assert count == want.shape[0]
    got = got[np.argsort(got[:, 0], kind="stable")]
    assert np.array_equal(got, want)
    ores, _, _, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
    assert np.array_equal(res, ores)
    # a ring smaller than the event count: every record written is a real event, the count is exact
    small, count2, _ = _gpu_events(clf, batch, 1000)
    assert count2 == want.shape[0] and small.shape[0] == 1000
    wset = {tuple(r) for r in want.tolist()}
    assert all(tuple(r) in wset for r in small.tolist())


def event_frames(wl, n_real=20000, seed=11):
    """Frames for the deny-event payload tests: (a) the generator's 80-B header snapshots of 64k packets at a fixed
    stride (pkt_len beyond the linear 80 B stands for frags), (b) n_real variable-length real frames back to back
    (40..300 B) whose IPv4 sources are taken from the generator's IPv4 packets, so most hit a prefix.
    Each: (buf u8, offsets u64, linear u32, pkt_len u32, ifindex u32, stride or 0)."""
    from frames import frame
    rng = np.random.default_rng(seed)
    hdr, cap, pl, ifx = wl.frames(31337, 1 << 16)
    v4 = np.nonzero((hdr[:, 12] == 8) & (hdr[:, 13] == 0))[0]
    fr, fifx = [], []
    for k in range(n_real):
        j = int(v4[rng.integers(0, v4.size)])
        src = "%d.%d.%d.%d" % tuple(int(x) for x in hdr[j, 26:30])
        fr.append(frame(src, proto=["tcp", "udp", "icmp", "sctp"][k % 4], dport=int(rng.integers(0, 1024)),
                        icmp_type=int(rng.integers(0, 20)), length=int(rng.integers(40, 300))))
        fifx.append(int(ifx[j]))
    offs = np.cumsum([0] + [len(f) for f in fr[:-1]]).astype(np.uint64)
    lens = np.array([len(f) for f in fr], np.uint32)
    return [(np.ascontiguousarray(hdr).reshape(-1), np.arange(hdr.shape[0], dtype=np.uint64) * 80,
             np.minimum(cap, 80).astype(np.uint32), pl, ifx, 80),
            (np.frombuffer(b"".join(fr), np.uint8), offs, lens, lens.copy(), np.array(fifx, np.uint32), 0)]


def test_event_samples():
    """§8f-1 deny-event payload: frames in HBM -> packer -> classify_events -> infw_events_capture; every perf
    sample (raw size, event_hdr_st, min(len, 256) frame bytes, pad) bit-exact vs the oracle's, and the consumer's
    syslog lines (infw/events.py, events.go:77-166) identical for both.  Frames: event_frames() — header snapshots
    at a fixed stride and variable-length real frames back to back, up to 300 B (256-B captures, and lengths past
    260 that the consumer rejects)."""
    import ctypes as C
    from infw import events as E
    from infw import _native as N
    dev = torch.device("cuda", 0)
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=50000, n_templates=256)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    m = oracle_for(wl)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
    names = lambda i: "if%d" % i
    for buf, offs, lens, plen, fifx, stride in event_frames(wl):
        n = len(offs)
        dbuf = torch.from_numpy(np.ascontiguousarray(buf).copy()).to(dev)
        fkw = dict(stride=stride) if stride else dict(offsets=torch.from_numpy(offs.view(np.int64)).to(dev))
        batch = SoaBatch.empty(n, dev)
        clf.pack_frames(dbuf, t(lens), t(fifx), batch, pkt_len=t(plen), **fkw)
        want_rec, want = m.collect_event_samples(buf, offs, lens, plen, fifx)
        k = want_rec.shape[0]
        assert k > 200
        for cap_ev in (n, 16):  # a ring for every event, and one smaller than the event count
            ev = torch.zeros(cap_ev * C.sizeof(N.EventRec), dtype=torch.uint8, device=dev)
            cnt = torch.zeros(1, dtype=torch.int64, device=dev)
            clf.classify_events(batch, ev, cnt)
            smp = torch.full((cap_ev * N.EVENT_SAMPLE_BYTES,), 0xEE, dtype=torch.uint8, device=dev)
            clf.events_capture(dbuf, t(lens), t(fifx), n, ev, cnt, smp, pkt_len=t(plen), **fkw)
            torch.cuda.synchronize()
            assert int(cnt.item()) == k
            w = min(k, cap_ev)
            idx = ev.cpu().numpy().view(np.uint64).reshape(-1, 3)[:w, 2]
            got = smp.cpu().numpy().reshape(-1, N.EVENT_SAMPLE_BYTES)[:w][np.argsort(idx, kind="stable")]
            if cap_ev == n:
                assert np.array_equal(got, want)
                assert E.drain(got, k, names) == E.drain(want, k, names)
                lines, log = E.drain(want, k, names)
                assert len(lines) >= 2 * (k - len(log))
            else:
                rows = {bytes(r) for r in want}
                assert all(bytes(r) in rows for r in got)
                assert E.drain(got, k, names)[1][0] == f"Perf event ring buffer full, dropped {k - 16} samples"


def test_partial_ifindex_prefixes_on_device():
    """Keys shorter than the ifindex (prefixLen < 32) through the kernel: slot defaults baked into the short table
    (both forms) and the partial-prefix list for interfaces without entries, vs the oracle."""
    import os
    import orc
    from test_golden import partial_ifindex_case
    entries, vals, hdr, cap, pl, fifx, tup = partial_ifindex_case()
    dev = torch.device("cuda", 0)
    for mode in ("dir24", "compressed"):
        c = infw.Classifier(devices=[0], options={"short_table": _SHORT[mode]})
        m = orc.OracleMap()
        for kb, rid in entries:
            c.update(infw.LpmIpKeySt.from_buffer_copy(kb), infw.RulesValSt.from_buffer_copy(vals[rid]))
            m.update(kb, vals[rid])
        c.commit()
        gres, gver = gpu_run(c, SoaBatch.from_tuples(tup, dev), tup.shape[0])
        want, over, ost, _ = m.classify_frames(hdr, cap, pl, fifx, nthreads=2)
        assert np.array_equal(gres, want), mode
        assert np.array_equal(gver, over) and np.array_equal(c.stats_read_all(), ost), mode


def test_device_frame_generator():
    """The bench's frames-in-HBM input (bench.py --from-frames): the device frame generator writes the host frame
    builder's header snapshots at the stride, and pack -> classify of them equals the oracle on those frames."""
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=20000, n_templates=128)
    dev = torch.device("cuda", 0)
    n, stride = 5000, 128
    frames = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
    lin, plen, ifx = (torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(3))
    wl.gen_frames_device(frames, stride, lin, plen, ifx, start=999, dev_ordinal=0)
    torch.cuda.synchronize()
    hdr, cap, pl, fx = wl.frames(999, n)
    f = frames.cpu().numpy().reshape(n, stride)
    assert np.array_equal(f[:, :80], hdr) and not f[:, 80:].any()
    assert np.array_equal(lin.cpu().numpy().view(np.uint32), np.minimum(cap, 80))
    assert np.array_equal(plen.cpu().numpy().view(np.uint32), pl)
    assert np.array_equal(ifx.cpu().numpy().view(np.uint32), fx)


@pytest.mark.parametrize("d16", ["0", "1"])
def test_parity_d16_words(monkeypatch, d16):
    """/16 words in front of DIR-24-8 (infw_tables.h; INFW_D16 forces them on or off, the compiler chooses them
    for sparse short tables such as configs[1] and [4]): bit-identical either way, on configs[1], [2] (100k
    prefixes, and the full 1M table, where the compiler would not choose them) and [4]."""
    monkeypatch.setitem(infw.DEFAULT_OPTIONS, "d16", int(d16))
    for cfg, n, npfx, ntmpl, start in [(W.CFG1_V4_10K, 1 << 18, 0, 0, 0), (W.CFG2_MIXED_1M, 1 << 18, 100000, 512, 0),
                                       (W.CFG4_ADVERSARIAL, 1 << 18, 20000, 64, 0),
                                       (W.CFG2_MIXED_1M, 1 << 17, 0, 0, (1 << 26) + 777)]:
        r = check_cfg(cfg, n, npfx, ntmpl, start=start)
        assert_parity(r, f"cfg{cfg}-{npfx}-d16={d16}")


def test_parity_compressed_short_table(monkeypatch):
    """The compressed 16-8-8 short-table form (chosen automatically when DIR-24-8 would exceed its memory
    budget, e.g. many ifindexes) classifies bit-identically."""
    monkeypatch.setitem(infw.DEFAULT_OPTIONS, "short_table", _SHORT["compressed"])
    r = check_cfg(W.CFG2_MIXED_1M, 1 << 18, 100000, 512)
    assert_parity(r, "cfg2-compressed")
    r = check_cfg(W.CFG4_ADVERSARIAL, 1 << 18, 20000, 64)
    assert_parity(r, "cfg4-compressed")


def test_pack_frames_on_device():
    """§8f-3 raw-frame ingestion: frames in HBM (fixed-stride chunks, and back-to-back variable-length frames
    with an offset array) packed on the GPU equal the host packer's tuples; classifying them matches the oracle."""
    from frames import frame, snapshots
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=50000, n_templates=256)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    m = oracle_for(wl)
    dev = torch.device("cuda", 0)
    n = 1 << 18
    hdr, cap, pl, ifx = wl.frames(99, n)
    t = lambda a, dt=torch.int32: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
    out = SoaBatch.empty(n, dev)
    clf.pack_frames(torch.from_numpy(hdr).to(dev), t(np.minimum(cap, 80)), t(ifx), out, pkt_len=t(pl), stride=80)
    torch.cuda.synchronize()
    want = W.pack_frames(hdr, np.minimum(cap, 80), pl, ifx)
    assert np.array_equal(out.to_tuples(), want)
    gres, gver = gpu_run(clf, out, n)
    ores, over, _, _ = m.classify_frames(hdr, np.minimum(cap, 80), pl, ifx, nthreads=8)
    assert np.array_equal(gres, ores) and np.array_equal(gver, over)
    # variable-length real frames, back to back, the shortest at the very end of the buffer
    rng = np.random.default_rng(5)
    fr = []
    for k in range(3000):
        src = "1.1.%d.%d" % (k & 255, (k >> 8) & 255) if k % 2 else "100:1::%x" % k
        f = frame(src, proto=["tcp", "udp", "icmp", "icmpv6", "sctp", "gre"][k % 6], dport=int(rng.integers(0, 65536)),
                  icmp_type=8, length=int(rng.integers(40, 300)))
        fr.append(f[: int(rng.integers(0, len(f) + 1))] if k % 7 == 0 else f)
    fr.append(frame("1.1.1.1", proto="tcp", dport=150)[:15])
    offs = np.cumsum([0] + [len(f) for f in fr[:-1]]).astype(np.uint64)
    buf = torch.from_numpy(np.frombuffer(b"".join(fr), np.uint8).copy()).to(dev)
    lens = np.array([len(f) for f in fr], np.uint32)
    ifs = np.ones(len(fr), np.uint32)
    out2 = SoaBatch.empty(len(fr), dev)
    clf.pack_frames(buf, t(lens), t(ifs), out2, offsets=torch.from_numpy(offs.view(np.int64)).to(dev))
    torch.cuda.synchronize()
    h2, c2, p2 = snapshots(fr)
    assert np.array_equal(out2.to_tuples(), W.pack_frames(h2, c2, p2, ifs))
    # the family-compact output: the same bytes as infw_soa_compact of the standard output, and the oracle's results
    from infw.batch import SoaBatchC
    for std, (fbuf, flen, fifx, fkw) in ((out, (torch.from_numpy(hdr).to(dev), t(np.minimum(cap, 80)), t(ifx),
                                                 dict(pkt_len=t(pl), stride=80))),
                                         (out2, (buf, t(lens), t(ifs),
                                                 dict(offsets=torch.from_numpy(offs.view(np.int64)).to(dev))))):
        oc = SoaBatchC.empty(std.n, dev)
        clf.pack_frames_c(fbuf, flen, fifx, oc, **fkw)
        ref = clf.compact(std)
        torch.cuda.synchronize()
        assert torch.equal(oc.saddr4, ref.saddr4) and torch.equal(oc.v6tail, ref.v6tail)
        for a, b in ((oc.ifindex, std.ifindex), (oc.pkt_len, std.pkt_len), (oc.meta, std.meta), (oc.l4word, std.l4word)):
            assert torch.equal(a, b)
        res = torch.empty(std.n, dtype=torch.int32, device=dev)
        clf.classify_c(oc, results=res)
        g_std, _ = gpu_run(clf, std, std.n)
        assert np.array_equal(res.cpu().numpy().view(np.uint32), g_std)


def _frames_run(clf, dbuf, lens, fifx, n, dev, plen=None, offs=None, stride=0):
    """infw_classify_frames over frames already on the device: (result words, verdicts, counters)."""
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
    res = torch.full((max(n, 1),), -1, dtype=torch.int32, device=dev)
    ver = torch.full((max(n, 1),), 0xEE, dtype=torch.uint8, device=dev)
    kw = dict(stride=stride) if stride else dict(offsets=torch.from_numpy(offs.view(np.int64)).to(dev))
    clf.stats_reset()
    clf.classify_frames(dbuf, t(lens), t(fifx), n, results=res, verdicts=ver,
                        pkt_len=t(plen) if plen is not None else None, **kw)
    torch.cuda.synchronize()
    return res.cpu().numpy().view(np.uint32)[:n], ver.cpu().numpy()[:n], clf.stats_read_all()


@pytest.mark.parametrize("short_table,d16", [("dir24", "1"), ("dir24", "0"), ("compressed", "")])
def test_classify_frames_on_device(monkeypatch, short_table, d16):
    """§8f-3 classification straight from raw frames (infw_classify_frames: the tuple is built in the kernel from
    the staged header window): result words, verdicts and counters equal the oracle's on the same frames —
    header snapshots at a fixed stride (a ragged count), and variable-length real frames back to back with an
    offset array (truncated ones, the shortest at the very end of the buffer).  The compressed short table runs
    the kernel's full (non-lean) instantiation."""
    from frames import frame, snapshots
    monkeypatch.setitem(infw.DEFAULT_OPTIONS, "short_table", _SHORT[short_table])
    if d16:  # /16 words in front of DIR-24-8 forced on / off
        monkeypatch.setitem(infw.DEFAULT_OPTIONS, "d16", int(d16))
    dev = torch.device("cuda", 0)
    for cfg, npre, ntpl in ((W.CFG2_MIXED_1M, 50000, 256), (W.CFG4_ADVERSARIAL, 20000, 64)):
        wl = W.Workload(cfg, n_prefixes=npre, n_templates=ntpl)
        clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
        wl.load_into(clf)
        clf.commit()
        m = oracle_for(wl)
        n = (1 << 18) + 77
        hdr, cap, pl, ifx = wl.frames(7, n)
        cap = np.minimum(cap, 80).astype(np.uint32)
        gres, gver, gst = _frames_run(clf, torch.from_numpy(np.ascontiguousarray(hdr)).to(dev), cap, ifx, n, dev,
                                      plen=pl, stride=80)
        ores, over, ost, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
        assert np.array_equal(gres, ores) and np.array_equal(gver, over), cfg
        assert np.array_equal(gst, ost), cfg
    # variable-length real frames, back to back (frame bytes past each one's length belong to the next frame)
    rng = np.random.default_rng(17)
    fr = []
    for k in range(5000):
        src = "1.1.%d.%d" % (k & 255, (k >> 8) & 255) if k % 2 else "100:1::%x" % k
        f = frame(src, proto=["tcp", "udp", "icmp", "icmpv6", "sctp", "gre"][k % 6], dport=int(rng.integers(0, 65536)),
                  icmp_type=8, length=int(rng.integers(40, 300)))
        fr.append(f[: int(rng.integers(0, len(f) + 1))] if k % 5 == 0 else f)
    fr.append(frame("1.1.1.1", proto="tcp", dport=150)[:15])
    offs = np.cumsum([0] + [len(f) for f in fr[:-1]]).astype(np.uint64)
    buf = torch.from_numpy(np.frombuffer(b"".join(fr), np.uint8).copy()).to(dev)
    lens = np.array([len(f) for f in fr], np.uint32)
    ifs = np.where(np.arange(len(fr)) % 3 == 0, 2, 1).astype(np.uint32)
    h2, c2, p2 = snapshots(fr)
    gres, gver, gst = _frames_run(clf, buf, lens, ifs, len(fr), dev, offs=offs)
    ores, over, ost, _ = m.classify_frames(h2, c2, p2, ifs, nthreads=2)
    assert np.array_equal(gres, ores) and np.array_equal(gver, over) and np.array_equal(gst, ost)
    # an empty batch launches nothing
    gres, gver, gst = _frames_run(clf, buf, lens[:0], ifs[:0], 0, dev, offs=offs[:0])
    assert not gst.any()


def test_frames_event_samples():
    """Deny events from infw_classify_frames_ex (the frames kernel with the event sideband): the records equal the
    packer path's (classify_events over the packed batch) after ordering by packet index, and
    infw_events_capture over the same frames writes the oracle's perf samples (kernel.c:392-399)."""
    import ctypes as C
    from infw import _native as N
    dev = torch.device("cuda", 0)
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=50000, n_templates=256)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    m = oracle_for(wl)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
    for buf, offs, lens, plen, fifx, stride in event_frames(wl):
        n = len(offs)
        dbuf = torch.from_numpy(np.ascontiguousarray(buf).copy()).to(dev)
        fkw = dict(stride=stride) if stride else dict(offsets=torch.from_numpy(offs.view(np.int64)).to(dev))
        batch = SoaBatch.empty(n, dev)
        clf.pack_frames(dbuf, t(lens), t(fifx), batch, pkt_len=t(plen), **fkw)
        want_rec, want = m.collect_event_samples(buf, offs, lens, plen, fifx)
        recs = []
        for fused in (False, True):
            ev = torch.zeros(n * C.sizeof(N.EventRec), dtype=torch.uint8, device=dev)
            cnt = torch.zeros(1, dtype=torch.int64, device=dev)
            res = torch.empty(n, dtype=torch.int32, device=dev)
            if fused:
                clf.classify_frames(dbuf, t(lens), t(fifx), n, results=res, pkt_len=t(plen), events=ev,
                                    events_count=cnt, **fkw)
            else:
                clf.classify_events(batch, ev, cnt, results=res)
            smp = torch.zeros((n * N.EVENT_SAMPLE_BYTES,), dtype=torch.uint8, device=dev)
            clf.events_capture(dbuf, t(lens), t(fifx), n, ev, cnt, smp, pkt_len=t(plen), **fkw)
            torch.cuda.synchronize()
            k = int(cnt.item())
            r = ev.cpu().numpy().view(np.uint64).reshape(-1, 3)[:k]
            order = np.argsort(r[:, 2], kind="stable")
            recs.append((k, r[order], smp.cpu().numpy().reshape(-1, N.EVENT_SAMPLE_BYTES)[:k][order],
                         res.cpu().numpy()))
        assert recs[0][0] == recs[1][0] == want_rec.shape[0] > 200
        assert np.array_equal(recs[0][1], recs[1][1]) and np.array_equal(recs[0][3], recs[1][3])
        assert np.array_equal(recs[1][2], want)


def test_survey_probes_from_frames_on_device():
    """Every survey probe (truncation at each header boundary, family gating, unified key space ...) as real frames
    back to back through infw_classify_frames: verdicts, result words and counters as recorded."""
    import goenc
    from test_golden import expected_stats, load, probe_frames
    dev = torch.device("cuda", 0)
    for case in load("survey_probes.json")["cases"]:
        c = infw.Classifier(devices=[0])
        for e in case["table"]:
            c.update(infw.build_ebpf_key(e["key"]["ifindex"], e["key"]["cidr"]),
                     infw.RulesValSt.from_buffer_copy(goenc.raw_value(e["rules"])))
        c.commit()
        frames, ifx = probe_frames(case)
        offs = np.cumsum([0] + [len(f) for f in frames[:-1]]).astype(np.uint64)
        buf = torch.from_numpy(np.frombuffer(b"".join(frames) + b"\0" * 16, np.uint8).copy()).to(dev)
        lens = np.array([len(f) for f in frames], np.uint32)
        res, ver, st = _frames_run(c, buf, lens, np.array(ifx, np.uint32), len(frames), dev, offs=offs)
        for p, v, r in zip(case["packets"], ver, res):
            assert v == p["expect"]["retval"], (case["name"], p, v, hex(r))
            if "result" in p["expect"]:
                assert r == p["expect"]["result"], (case["name"], p, hex(r))
        assert np.array_equal(st, expected_stats(case, frames)), case["name"]


@pytest.mark.parametrize("short_table", ["dir24", "compressed"])
def test_survey_probes_on_device(monkeypatch, short_table):
    """Every probe of tests/golden/survey_probes.json (the reference's edge semantics:
    truncation, family gating, unified key space, IPv4-mapped keys, tables with no
    <= /32 entry ...) through the HIP kernel: verdicts, result words and counters."""
    import goenc
    from frames import snapshots
    from test_golden import expected_stats, load, probe_frames
    monkeypatch.setitem(infw.DEFAULT_OPTIONS, "short_table", _SHORT[short_table])
    dev = torch.device("cuda", 0)
    for case in load("survey_probes.json")["cases"]:
        c = infw.Classifier(devices=[0])
        for e in case["table"]:
            c.update(infw.build_ebpf_key(e["key"]["ifindex"], e["key"]["cidr"]),
                     infw.RulesValSt.from_buffer_copy(goenc.raw_value(e["rules"])))
        c.commit()
        frames, ifx = probe_frames(case)
        hdr, cap, pl = snapshots(frames)
        tuples = W.pack_frames(hdr, cap, pl, np.array(ifx, np.uint32))
        n = tuples.shape[0]
        res, ver = gpu_run(c, SoaBatch.from_tuples(tuples, dev), n)
        for p, v, r in zip(case["packets"], ver, res):
            assert v == p["expect"]["retval"], (case["name"], p, v, hex(r))
            if "result" in p["expect"]:
                assert r == p["expect"]["result"], (case["name"], p, hex(r))
        assert np.array_equal(c.stats_read_all(), expected_stats(case, frames)), case["name"]


def test_debug_lookup_capture_compact_layout():
    """The debug lookup sideband in the family-compact kernels (classify_c: the IPv6 key words come from the
    v6tail loads): the captured set equals the oracle's dbg map, and results equal the oracle's."""
    import orc
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=50000, n_templates=256)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    m = oracle_for(wl)
    dev = torch.device("cuda", 0)
    n = 8000
    batch = SoaBatch.empty(n, dev)
    wl.gen_device(batch, 4321, 0)
    hdr, cap, pl, ifx = wl.frames(4321, n)
    want, n_distinct = orc.debug_map_after(hdr, cap, pl, ifx)
    assert 1000 < n_distinct < orc.DBG_MAX_ENTRIES
    bc = clf.compact(batch)
    clf.debug_lookup(1)
    res = torch.empty(n, dtype=torch.int32, device=dev)
    clf.classify_c(bc, results=res)
    torch.cuda.synchronize()
    got = clf.debug_keys()
    assert len(got) == len(want) and set(got) == set(want)
    ores, _, _, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=4)
    assert np.array_equal(res.cpu().numpy().view(np.uint32), ores)


def test_multi_device_context():
    """One context over two device slots (devices=[0, 0]: the path a cgo caller with several GPUs takes, on one
    card): tables replicated per slot through full and incremental commits, one statistics slot per device
    summed like per-CPU slots (statistics.go:126-157), debug keys the union of the per-device sets."""
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=20000, n_templates=128)
    clf = infw.Classifier(devices=[0, 0], max_entries=wl.n_entries + 64)
    assert clf.num_devices == 2
    wl.load_into(clf)
    clf.commit()
    m = oracle_for(wl)
    dev = torch.device("cuda", 0)
    n = 1 << 16
    halves = []
    for d, start in ((0, 0), (1, n)):
        b = SoaBatch.empty(n, dev)
        wl.gen_device(b, start, 0)
        halves.append((d, start, b))
    clf.debug_lookup(1)
    for epoch in range(2):
        clf.stats_reset()
        want_stats = np.zeros((1024, 4), np.uint64)
        for d, start, b in halves:
            gres, _ = gpu_run(clf, b, n, dev_index=d)
            hdr, cap, pl, ifx = wl.frames(start, n)
            ores, _, ost, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
            assert np.array_equal(gres, ores), (epoch, d)
            want_stats += ost
            slots = clf.stats_read(1)
            assert len(slots) == 2
        assert np.array_equal(clf.stats_read_all(), want_stats)
        per_slot = [clf.stats_read(r) for r in range(1, 100)]
        assert all(s[0].allow_packets + s[1].allow_packets == want_stats[r + 1, 0] for r, s in enumerate(per_slot))
        if epoch == 0:  # an incremental commit: delete every 4th key, rewrite every 7th
            keys = wl.keys_bytes().reshape(-1, 24)
            tmpl = wl.templates_bytes().reshape(-1, 1200)
            for i in range(0, keys.shape[0], 4):
                kb = keys[i].tobytes()
                assert clf.delete_rc(infw.LpmIpKeySt.from_buffer_copy(kb)) == m.delete(kb)
            for i in range(1, keys.shape[0], 7):
                kb, vb = keys[i].tobytes(), tmpl[(i * 3) % tmpl.shape[0]].tobytes()
                assert clf.update_rc(infw.LpmIpKeySt.from_buffer_copy(kb),
                                     infw.RulesValSt.from_buffer_copy(vb)) == m.update(kb, vb)
            clf.commit()
            assert clf.info()["commit_mode"] == 1  # INFW_COMMIT_INCREMENTAL, applied to both device slots
    import orc
    allk = set()
    for d, start, b in halves:
        hdr, cap, pl, ifx = wl.frames(start, n)
        allk |= set(orc.debug_map_after(hdr, cap, pl, ifx, max_entries=2 * n)[0])
    got = clf.debug_keys()
    assert len(got) == len(set(got)) == min(len(allk), orc.DBG_MAX_ENTRIES) and set(got) <= allk


def test_debug_lookup_capture():
    """§8f-4 debug lookup capture (kernel.c:59-64, :214-216, :297-299): with debug_lookup set, the set of
    lookup keys equals the oracle's dbg map (first-seen NOEXIST inserts, <= 16384 keys); repeats leave it
    unchanged; classification is unaffected; once full, exactly 16384 keys, all of them real lookup keys."""
    import orc
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=50000, n_templates=256)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    m = oracle_for(wl)
    dev = torch.device("cuda", 0)
    n = 8000
    batch = SoaBatch.empty(n, dev)
    wl.gen_device(batch, 555, 0)
    hdr, cap, pl, ifx = wl.frames(555, n)
    want, n_distinct = orc.debug_map_after(hdr, cap, pl, ifx)
    assert 1000 < n_distinct < orc.DBG_MAX_ENTRIES
    assert clf.debug_keys() == []
    clf.debug_lookup(1)
    clf.stats_reset()
    gres, gver = gpu_run(clf, batch, n)
    got = clf.debug_keys()
    assert len(got) == len(want) and set(got) == set(want)
    ores, over, ostats, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=4)
    assert np.array_equal(gres, ores) and np.array_equal(gver, over)
    assert np.array_equal(clf.stats_read_all(), ostats)
    gpu_run(clf, batch, n)                       # NOEXIST: the same keys again change nothing
    assert sorted(clf.debug_keys()) == sorted(want)
    # heavy duplication inside waves and across workgroups: 64 distinct packets, 1024 copies each
    clf.debug_keys_clear()
    assert clf.debug_keys() == []
    tup = np.tile(W.pack_frames(hdr[:64], cap[:64], pl[:64], ifx[:64]), (1024, 1))
    gpu_run(clf, SoaBatch.from_tuples(tup, dev), tup.shape[0])
    want64, _ = orc.debug_map_after(hdr[:64], cap[:64], pl[:64], ifx[:64])
    assert sorted(clf.debug_keys()) == sorted(want64)
    # debug_lookup 0: nothing captured
    clf.debug_keys_clear()
    clf.debug_lookup(0)
    gpu_run(clf, batch, n)
    assert clf.debug_keys() == []
    # more distinct keys than the map holds: exactly 16384 keys, each a real lookup key of the batch
    clf.debug_lookup(1)
    nb = 1 << 17
    big = SoaBatch.empty(nb, dev)
    wl.gen_device(big, 1 << 20, 0)
    hb, cb, pb, ib = wl.frames(1 << 20, nb)
    allk, nd = orc.debug_map_after(hb, cb, pb, ib, max_entries=nb)
    assert nd > orc.DBG_MAX_ENTRIES
    gres_b, _ = gpu_run(clf, big, nb)
    got = clf.debug_keys()
    assert len(got) == orc.DBG_MAX_ENTRIES == len(set(got))
    assert set(got) <= set(allk)
    gpu_run(clf, batch, n)                       # full: new keys are dropped, the set is unchanged
    assert set(clf.debug_keys()) == set(got)
    assert np.array_equal(gres_b, m.classify_frames(hb, cb, pb, ib, nthreads=8)[0])


@pytest.mark.parametrize("d16,split", [("", ""), ("1", ""), ("", "1")])
def test_incremental_commits_on_device(monkeypatch, d16, split):
    """§8f-2: a run of incremental commits (both device images ping-pong, one commit re-uploads
    after its new rule lists outgrow the spare's buffers); after every commit the device results
    equal the oracle's on the workload and on packets aimed at the edited prefixes — also with /16 words in
    front of DIR-24-8 forced on, whose re-derived words the patch uploads with the rest, and in the two-phase
    classify form (its decision lines patched and appended like the fused kernel's)."""
    import random
    import orc
    from test_incremental_cpu import _apply, _packets_for, _val
    if d16:
        monkeypatch.setitem(infw.DEFAULT_OPTIONS, "d16", int(d16))
    if split:
        monkeypatch.setitem(infw.DEFAULT_OPTIONS, "split", int(split))
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=100000, n_templates=512)
    ents = list(wl.entries())
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 4096)
    m = orc.OracleMap(max_entries=wl.n_entries + 4096)
    for k, v in ents:
        _apply((clf,), m, k, v)
    clf.commit()
    assert clf.info()["d16"] == (1 if d16 else 0)
    dev = torch.device("cuda", 0)
    n = 1 << 17
    batch = SoaBatch.empty(n, dev)
    wl.gen_device(batch, 0, 0)
    hdr, cap, pl, ifx = wl.frames(0, n)
    rng = random.Random(17)
    vals = [v for _, v in ents[:4000]]
    modes = []
    for step in range(7):
        touched = []
        n_new_vals = 1500 if step == 4 else 20
        for k, _ in rng.sample(ents, 400 + n_new_vals):
            if n_new_vals:
                v = _val(rng, step)
                n_new_vals -= 1
            else:
                v = None if rng.random() < 0.3 else rng.choice(vals)
            _apply((clf,), m, k, v)
            touched.append(k)
        clf.commit()
        info = clf.info()
        modes.append(info["commit_mode"])
        ores, _, _, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
        gres, _ = gpu_run(clf, batch, n)
        assert np.array_equal(gres, ores), (step, info["commit_mode"])
        th, tc, tp, ti = _packets_for(touched, rng, 2)
        want, _, _, _ = m.classify_frames(th, tc, tp, ti, nthreads=8)
        tb = SoaBatch.from_tuples(W.pack_frames(th, tc, tp, ti), dev)
        got, _ = gpu_run(clf, tb, len(ti))
        assert np.array_equal(got, want), (step, info["commit_mode"])
        if info["commit_mode"] == infw.COMMIT_INCREMENTAL:
            assert info["patch_bytes"] < (8 << 20), info["patch_bytes"]
    assert modes.count(infw.COMMIT_INCREMENTAL) >= 4 and infw.COMMIT_REUPLOAD in modes, modes


def test_commits_while_batches_in_flight():
    """configs[4] live swap with the device busy: batch A is queued on a side stream (repeated, so it is
    still running), then two incremental commits are made before A finishes and batch B is classified on
    the second new epoch.  Incremental commits patch only the spare image and wait only for the launches
    that read it, so A (on epoch 1) must equal the oracle's epoch 1 and B the oracle's epoch 3."""
    import random
    import orc
    from test_incremental_cpu import _apply
    wl = W.Workload(W.CFG4_ADVERSARIAL, n_prefixes=20000, n_templates=64)
    ents = list(wl.entries())
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 4096)
    m1 = orc.OracleMap(max_entries=wl.n_entries + 4096)
    for k, v in ents:
        _apply((clf,), m1, k, v)
    clf.commit()
    dev = torch.device("cuda", 0)
    n = 1 << 20
    a, b = SoaBatch.empty(n, dev), SoaBatch.empty(n, dev)
    wl.gen_device(a, 0, 0)
    wl.gen_device(b, n, 0)
    torch.cuda.synchronize()
    rng = random.Random(5)
    vals = [v for _, v in ents]
    edits = [[(k, None if rng.random() < 0.25 else rng.choice(vals)) for k, _ in rng.sample(ents, 300)]
             for _ in range(2)]
    m3 = orc.OracleMap(max_entries=wl.n_entries + 4096)
    for k, v in ents:
        m3.update(k, v)
    for k, v in edits[0]:  # staged: classify keeps reading epoch 1 until the commit
        _apply((clf,), m3, k, v)
    side = torch.cuda.Stream(dev)
    res_a = torch.empty(n, dtype=torch.int32, device=dev)
    with torch.cuda.stream(side):
        for _ in range(400):  # >10 ms of work queued on epoch 1
            clf.classify(a, results=res_a, stream=side)
    clf.commit()  # patches the spare; A keeps running on epoch 1
    assert clf.info()["commit_mode"] == infw.COMMIT_INCREMENTAL
    for k, v in edits[1]:
        _apply((clf,), m3, k, v)
    clf.commit()  # the spare is now epoch 1's image: this one waits for A's launches
    assert clf.info()["commit_mode"] == infw.COMMIT_INCREMENTAL
    gres_b, _ = gpu_run(clf, b, n)
    side.synchronize()
    hdr, cap, pl, ifx = wl.frames(0, n)
    want_a, _, _, _ = m1.classify_frames(hdr, cap, pl, ifx, nthreads=8)
    assert np.array_equal(res_a.cpu().numpy().view(np.uint32), want_a)
    hdr, cap, pl, ifx = wl.frames(n, n)
    want_b, _, _, _ = m3.classify_frames(hdr, cap, pl, ifx, nthreads=8)
    assert np.array_equal(gres_b, want_b)
    assert not np.array_equal(want_a, m3.classify_frames(*wl.frames(0, n), nthreads=8)[0])  # the edits matter


@pytest.mark.parametrize("n_if", [100, 129, 400])
def test_many_ifindexes(n_if):
    """The ifindex map outside LDS (> 128 ifindexes: the map no longer fits the kernel's 256-entry LDS copy) and
    the short-table form chosen by size (> 32 ifindexes: DIR-24-8 would exceed 4 GiB -> compressed 16-8-8):
    random v4/v6 prefixes on n_if ifindexes, packets aimed at them and at unknown ifindexes, vs the oracle."""
    import random
    import struct
    import orc
    from test_compiler_cpu import _val
    from test_incremental_cpu import _packets_for
    rng = random.Random(n_if)
    ifs = rng.sample(range(1, 1 << 20), n_if)
    ents = {}
    for i in range(6000):
        ifx = ifs[i % n_if]
        if rng.random() < 0.6:
            L = rng.choice([0, 8, 16, 20, 24, 25, 28, 32])
            ip = rng.getrandbits(32).to_bytes(4, "big") + bytes(12)
        else:
            L = rng.choice([16, 32, 40, 48, 56, 64, 96, 128])
            ip = rng.getrandbits(128).to_bytes(16, "big")
        ents[struct.pack("<II", L + 32, ifx) + ip] = _val(rng, i)
    clf = infw.Classifier(devices=[0], max_entries=len(ents) + 16)
    m = orc.OracleMap(max_entries=len(ents) + 16)
    for k, v in ents.items():
        assert clf.update_rc(infw.LpmIpKeySt.from_buffer_copy(k), infw.RulesValSt.from_buffer_copy(v)) == m.update(k, v)
    clf.commit()
    keys = list(ents)
    hdr, cap, pl, ifx = _packets_for(rng.sample(keys, 3000), rng, 3)
    ifx[::7] = np.array([rng.randrange(1 << 20, 1 << 21) for _ in range(ifx[::7].size)], np.uint32)  # unknown
    want, _, wst, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
    dev = torch.device("cuda", 0)
    clf.stats_reset()
    got, _ = gpu_run(clf, SoaBatch.from_tuples(W.pack_frames(hdr, cap, pl, ifx), dev), len(ifx))
    assert np.array_equal(got, want)
    assert np.array_equal(clf.stats_read_all(), wst)
    assert (want != 0).mean() > 0.3


@pytest.mark.parametrize("cfg,npfx,ntmpl", [(W.CFG2_MIXED_1M, 50000, 256), (W.CFG4_ADVERSARIAL, 20000, 64),
                                            (W.CFG1_V4_10K, 0, 0)])
def test_compact_layout(cfg, npfx, ntmpl):
    """infw_soa_compact + infw_classify_c: the family-compact address layout gives the oracle's result words,
    verdicts and counters (ragged batch: the last 64-packet group is partial; cfg1 has no IPv6 packets)."""
    wl = W.Workload(cfg, n_prefixes=npfx, n_templates=ntmpl)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    m = oracle_for(wl)
    dev = torch.device("cuda", 0)
    n = (1 << 18) + 37
    b = SoaBatch.empty(n, dev)
    wl.gen_device(b, 7, 0)
    bc = clf.compact(b)
    res = torch.empty(n, dtype=torch.int32, device=dev)
    ver = torch.empty(n, dtype=torch.uint8, device=dev)
    clf.stats_reset()
    clf.classify_c(bc, results=res, verdicts=ver)
    torch.cuda.synchronize()
    hdr, cap, pl, ifx = wl.frames(7, n)
    want, wver, wst, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
    assert np.array_equal(res.cpu().numpy().view(np.uint32), want)
    assert np.array_equal(ver.cpu().numpy(), wver)
    assert np.array_equal(clf.stats_read_all(), wst)


@pytest.mark.parametrize("block,group,bpc", [(768, 0, 2), (512, 0, 3), (512, 0, 4), (512, 0, 2), (256, 0, 6),
                                             (512, 8, 3), (256, 4, 6), (512, 1, 3)])
def test_launch_shapes(block, group, bpc):
    """Every launch shape infw_set_launch accepts (decision tables at 16-32 waves per CU, the one-lane-per-rule
    ballot scan with 1/4/8 packets in flight) gives the oracle's result words and counters."""
    r = check_cfg(W.CFG2_MIXED_1M, (1 << 17) + 333, 50000, 256, launch=(block, group, bpc))
    assert_parity(r, f"shape {block}x{bpc} g{group}")


def _bucket_hash(slot: int, top: int) -> int:
    """infw_bucket_hash (csrc/infw_tables.h), for aiming keys at one LDS cache entry."""
    M = (1 << 64) - 1
    h = (((slot << 32) | top) * 0x9E3779B97F4A7C15) & M
    h ^= h >> 31
    h = (h * 0xBF58476D1CE4E5B9) & M
    return h ^ (h >> 30)


def _b6_key(slot: int, top: int) -> int:
    """infw_b6_key (csrc/infw_tables.h): the IPv6 group cache's 40-bit bijective key (index = its top bits)."""
    M = (1 << 40) - 1
    k = ((slot << 32) | top) & M
    k = (k * 0x9E3779B97F) & M
    k ^= k >> 20
    k = (k * 0xC2B2AE3D27) & M
    return k ^ (k >> 23)


def test_lds_cache_collisions():
    """The kernel's LDS caches under maximal contention: 64 IPv6 single-record groups that all map to 2 entries of
    the IPv6 group cache and 64 IPv4 /24s that all map to 2 entries of the word cache, each with its own rule list;
    packets spread over them, so lanes of one wave keep overwriting the same entries with different groups.  Every
    result word must still be the oracle's (a torn or mixed entry would answer with another group's list)."""
    import random
    import struct
    import orc
    from test_incremental_cpu import _packets_for
    rng = random.Random(11)
    b6_log, c24_log = 8, 12  # the default shape's cache sizes with per-list part counts (768 x 2, <= 4096 lists)
    want6 = {}
    while len(want6) < 64:
        top = rng.getrandbits(32)
        idx = _b6_key(0, top) >> (40 - b6_log)
        if idx in (3, 77):
            want6[top] = idx
    want4 = {}
    while len(want4) < 64:
        a24 = rng.getrandbits(24)
        idx = ((a24 * 0x9E3779B1) & 0xFFFFFFFF) >> (32 - c24_log)  # key = slot << 24 | a24, slot 0
        if idx in (5, 901):
            want4[a24] = idx
    import goenc
    ents = {}
    for j, top in enumerate(want6):
        val = goenc.make_value([{"order": 1 + j % 90, "protocol": "TCP", "ports": "1-60000", "action": "Allow"}])
        ents[struct.pack("<II", 48 + 32, 1) + top.to_bytes(4, "big") + rng.getrandbits(96).to_bytes(12, "big")] = val
    for j, a24 in enumerate(want4):
        val = goenc.make_value([{"order": 1 + (j + 37) % 90, "protocol": "TCP", "ports": "1-60000", "action": "Deny"}])
        ents[struct.pack("<II", 24 + 32, 1) + (a24 << 8).to_bytes(4, "big") + bytes(12)] = val
    clf = infw.Classifier(devices=[0], max_entries=len(ents) + 16)
    m = orc.OracleMap(max_entries=len(ents) + 16)
    for k, v in ents.items():
        assert clf.update_rc(infw.LpmIpKeySt.from_buffer_copy(k), infw.RulesValSt.from_buffer_copy(v)) == m.update(k, v)
    clf.commit()
    hdr, cap, pl, ifx = _packets_for(list(ents), rng, 1500)
    perm = np.random.default_rng(3).permutation(len(ifx))
    hdr, cap, pl, ifx = hdr[perm], cap[perm], pl[perm], ifx[perm]
    want, _, wst, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
    dev = torch.device("cuda", 0)
    clf.stats_reset()
    got, _ = gpu_run(clf, SoaBatch.from_tuples(W.pack_frames(hdr, cap, pl, ifx), dev), len(ifx))
    assert np.array_equal(got, want)
    assert np.array_equal(clf.stats_read_all(), wst)
    assert len(np.unique(want[want != 0])) > 100  # the groups really answer with different lists


def test_lds_d16_cache_collisions(monkeypatch):
    """The LDS cache of /16 words (the kD16 kernels, INFW_D16=1) under maximal contention: 48 /16s answered by
    their /16 word (a /20 inside each) and 16 /16s that are not (five /24s of different lists each), all mapped to 2
    entries of the cache, each prefix with its own rule list; lanes of one wave keep overwriting the same entries
    with different /16s' words, so a torn pair or a mixed-up word would answer with another /16's list."""
    import random
    import struct
    import orc
    import goenc
    from test_incremental_cpu import _packets_for
    monkeypatch.setitem(infw.DEFAULT_OPTIONS, "d16", int("1"))
    rng = random.Random(12)
    idx_bits = 10  # the per-list-part-count shape: 2048 LDS words = 1024 /16-word entries
    his = []
    while len(his) < 64:
        hi = rng.getrandbits(16)
        if hi not in his and (((hi * 0x9E3779B1) & 0xFFFFFFFF) >> (32 - idx_bits)) in (7, 600):  # slot 0: key = hi
            his.append(hi)
    ents, order = {}, 1
    for j, hi in enumerate(his):
        subs = [(20, rng.getrandbits(4) << 12)] if j < 48 else [(24, rng.getrandbits(8) << 8) for _ in range(5)]
        for L, lo in subs:
            val = goenc.make_value([{"order": order % 99 + 1, "protocol": "TCP", "ports": "1-60000", "action": "Allow"}])
            order += 1
            ents[struct.pack("<II", L + 32, 1) + ((hi << 16) | lo).to_bytes(4, "big") + bytes(12)] = val
    clf = infw.Classifier(devices=[0], max_entries=len(ents) + 16)
    m = orc.OracleMap(max_entries=len(ents) + 16)
    for k, v in ents.items():
        assert clf.update_rc(infw.LpmIpKeySt.from_buffer_copy(k), infw.RulesValSt.from_buffer_copy(v)) == m.update(k, v)
    clf.commit()
    assert clf.info()["d16"] == 1
    hdr, cap, pl, ifx = _packets_for(list(ents), rng, 1200)
    perm = np.random.default_rng(5).permutation(len(ifx))
    hdr, cap, pl, ifx = hdr[perm], cap[perm], pl[perm], ifx[perm]
    want, _, wst, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
    dev = torch.device("cuda", 0)
    clf.stats_reset()
    got, _ = gpu_run(clf, SoaBatch.from_tuples(W.pack_frames(hdr, cap, pl, ifx), dev), len(ifx))
    assert np.array_equal(got, want)
    assert np.array_equal(clf.stats_read_all(), wst)
    assert len(np.unique(want[want != 0])) > 60


@pytest.mark.parametrize("split", ["", "1"])
def test_classify_host_batches(monkeypatch, split):
    """infw_classify_host: a host-resident batch pipelined through the device in chunks (ragged last chunk,
    pageable and page-locked memory) gives the same result words, verdicts and counters as the oracle — also in
    the two-phase form, whose per-chunk scratch is allocated on the pipeline's kernel stream."""
    if split:
        monkeypatch.setitem(infw.DEFAULT_OPTIONS, "split", int(split))
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=50000, n_templates=256)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    m = oracle_for(wl)
    n = 300001
    hdr, cap, pl, ifx = wl.frames(0, n)
    ores, over, ost, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
    soa = infw.HostSoa.from_tuples(wl.tuples(0, n))
    for chunk, pin in ((65536, False), (1 << 22, True)):
        if pin:
            for a in soa.arrays():
                clf.host_register(a)
        res = np.zeros(n, np.uint32)
        ver = np.zeros(n, np.uint8)
        clf.stats_reset()
        clf.classify_host(soa, res, ver, chunk=chunk)
        assert np.array_equal(res, ores), chunk
        assert np.array_equal(ver, over), chunk
        assert np.array_equal(clf.stats_read_all(), ost), chunk
        if pin:
            for a in soa.arrays():
                clf.host_unregister(a)


def test_lists_past_part_count_table_on_device():
    """New rule lists committed incrementally past the per-list part-count table (> 4096 lists): the kernel's LDS
    copy of the table covers the first 4096 lists, later ones take uniform parts — results equal the oracle."""
    import random
    from test_incremental_cpu import _apply, _packets_for
    from tools_commit import new_value
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=30000, n_templates=4096)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 4096)
    wl.load_into(clf)
    clf.commit()
    m = oracle_for(wl)
    rng = random.Random(9)
    keys = [k for k, _ in wl.entries()]
    dev = torch.device("cuda", 0)
    for rnd in range(2):
        touched = rng.sample(keys, 400)
        for k in touched:
            _apply([clf], m, k, new_value(rng))
        clf.commit()
        assert clf.info()["commit_mode"] == infw.COMMIT_INCREMENTAL, clf.info()["full_reason"]
        hdr, cap, pl, ifx = _packets_for(touched, rng)
        tup = W.pack_frames(hdr, cap, pl, ifx)
        b = SoaBatch.from_tuples(tup, dev)
        gres, _ = gpu_run(clf, b, b.n)
        ores, _, _, _ = m.classify_frames(hdr, cap, pl, ifx)
        assert np.array_equal(gres, ores), rnd
    assert clf.info()["n_lists"] > 4096


@pytest.mark.parametrize("flush_tiles", ["1", "3", None])
def test_counter_paths(monkeypatch, flush_tiles):
    """The packed per-workgroup LDS counters (packets << 40 | bytes) against the counters implied by the result
    words: workgroups flushing after every tile / every 3 tiles / at the default interval, and 1 % of the frames
    with lengths of 2^20 B or more (up to 2^32 - 1), which bypass the packed counters."""
    if flush_tiles:
        monkeypatch.setitem(infw.DEFAULT_OPTIONS, "stat_flush_tiles", int(flush_tiles))
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=50000, n_templates=256)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    dev = torch.device("cuda", 0)
    n = 1 << 18
    b = SoaBatch.empty(n, dev)
    wl.gen_device(b, 4321, 0)
    g = torch.Generator(device="cpu").manual_seed(7)
    big = torch.rand(n, generator=g) < 0.01
    lens = torch.randint(1 << 20, (1 << 32) - 1, (n,), generator=g, dtype=torch.int64)
    pl = b.pkt_len.cpu().to(torch.int64)
    pl[big] = lens[big]
    b.pkt_len.copy_(pl.to(torch.int32).to(dev))  # u32 bit pattern
    clf.stats_reset()
    gres, _ = gpu_run(clf, b, n)
    plen = b.pkt_len.cpu().numpy().view(np.uint32)
    want = stats_from_results(gres, plen)
    assert np.array_equal(clf.stats_read_all(), want)
    assert int(want[:, 1].max()) > (1 << 32) or int(want[:, 3].max()) > (1 << 32)  # byte sums past 32 bits


@pytest.mark.parametrize("short_table", ["dir24", "compressed"])
def test_clustered_adversarial_tables_on_device(monkeypatch, short_table):
    """Every LPM corner on the device (tests/test_compiler_cpu.py `_clustered_table`): IPv6 prefixes clustered
    under few /32s (groups past 3 records: the Waldvogel overflow table, the non-lean kernel), nested lengths
    /0../128 on three ifindexes (one above 2^16), IPv4 nesting, cross-family aliases; rule values with rule ids 0,
    1024 and > 65535, actions outside {1, 2}, empty and reversed ranges, every protocol.  Result words, verdicts and
    per-rule counters from the SoA kernel and the frames kernel, against the oracle."""
    import random
    import orc
    from test_compiler_cpu import _clustered_table, clustered_packets
    monkeypatch.setitem(infw.DEFAULT_OPTIONS, "short_table", _SHORT[short_table])
    entries, anchors = _clustered_table(random.Random(7))
    clf = infw.Classifier(devices=[0])
    m = orc.OracleMap()
    for k, v in entries:
        assert clf.update_rc(infw.LpmIpKeySt.from_buffer_copy(k), infw.RulesValSt.from_buffer_copy(v)) == m.update(k, v)
    clf.commit()
    info = clf.info()
    assert info["n_v6_overflow"] > 0 and info["short_mode"] == (1 if short_table == "compressed" else 0)
    hdr, cap, pl, ifx = clustered_packets(anchors, 20000, 3)
    ores, over, ost, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=4)
    dev = torch.device("cuda", 0)
    b = SoaBatch.from_tuples(W.pack_frames(hdr, cap, pl, ifx), dev)
    clf.stats_reset()
    gres, gver = gpu_run(clf, b, b.n)
    assert np.array_equal(gres, ores) and np.array_equal(gver, over)
    assert np.array_equal(clf.stats_read_all(), ost)
    assert (ores != 0).mean() > 0.3
    n = hdr.shape[0]
    stride = 128
    buf = np.zeros(n * stride, np.uint8)
    buf.reshape(n, stride)[:, :hdr.shape[1]] = hdr
    lin = np.minimum(cap, hdr.shape[1]).astype(np.uint32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).to(dev)
    res = torch.empty(n, dtype=torch.int32, device=dev)
    clf.stats_reset()
    clf.classify_frames(torch.from_numpy(buf).to(dev), t(lin), t(ifx), n, results=res, pkt_len=t(pl), stride=stride)
    torch.cuda.synchronize()
    assert np.array_equal(res.cpu().numpy().view(np.uint32), ores)
    assert np.array_equal(clf.stats_read_all(), ost)
