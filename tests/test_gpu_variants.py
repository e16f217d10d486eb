"""Every kernel instantiation the library can launch, on the device, against the oracle.

The registry (infw_kernel_variant_name) lists each classify_kernel instantiation and the decide kernel; for each one
this test builds the table kind and launch that the selector maps onto it (tests/variants.py; the CPU test
tests/test_variants_cpu.py proves every entry is reachable and nothing else is), asks infw_classify_variant which
instantiation the launch runs, runs it on a ragged batch and compares result words, XDP verdicts and per-rule
counters with the oracle bit for bit — the sideband launches also their event count and captured keys."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import infw  # noqa: E402
from infw import workloads as W  # noqa: E402
from infw.batch import SoaBatch  # noqa: E402

import variants as V  # noqa: E402
from parity import oracle_for  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def test_every_registered_variant_matches_the_oracle():
    dev = torch.device("cuda", 0)
    wl = W.Workload(W.CFG2_MIXED_1M, **V.TABLE)
    m = oracle_for(wl)
    n, start, stride = (1 << 18) + 37, 4242, 128
    hdr, cap, pl, ifx = wl.frames(start, n)
    ores, over, ostats, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
    # the same frames as an AF_XDP ring (infw_classify_xdp): one ifindex for the ring, the descriptor's length as
    # both the linear and the frame length, the 80-B snapshots back to back in a umem in HBM
    ring_if = int(np.bincount(ifx).argmax())
    xres, xver, xstats, _ = m.classify_frames(hdr, pl.astype(cap.dtype), pl, np.full(n, ring_if, np.uint32), nthreads=8)
    addr = np.arange(n, dtype=np.uint64) * np.uint64(hdr.shape[1])
    desc = np.zeros((n, 4), np.uint32)
    desc[:, 0], desc[:, 1], desc[:, 2] = addr & np.uint64(0xFFFFFFFF), addr >> np.uint64(32), pl
    umem = torch.from_numpy(np.concatenate([hdr.reshape(-1), np.zeros(64, np.uint8)])).to(dev)
    xdesc = torch.from_numpy(desc.view(np.int32)).to(dev)
    deny = int(((ores & 0xFF) == infw.XDP_DROP).sum())
    batch = SoaBatch.empty(n, dev)
    wl.gen_device(batch, start, 0)
    frames = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
    lin, plen, fifx = (torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(3))
    wl.gen_frames_device(frames, stride, lin, plen, fifx, start=start, dev_ordinal=0)
    res = torch.empty(n, dtype=torch.int32, device=dev)
    ver = torch.empty(n, dtype=torch.uint8, device=dev)
    events = torch.zeros(n * 24, dtype=torch.uint8, device=dev)
    events_count = torch.zeros(1, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()

    reg = V.registry()
    done = {}
    for kind in V.KINDS:
        clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16, options=V.KINDS[kind])
        wl.load_into(clf)
        clf.commit()
        bc = clf.compact(batch)
        for kind_, split, shape, inp, ev, dbg in V.scenarios():
            if kind_ != kind:
                continue
            clf.set_option("split", split)
            clf.set_launch(*shape)
            clf.debug_lookup(1 if dbg else 0)
            name = clf.variant(V.INPUTS[inp], events=ev)
            if all(x in done for x in V.names_of(name)):
                continue
            clf.stats_reset()
            res.fill_(-1)
            ver.fill_(7)
            events_count.zero_()
            evs = dict(events=events, events_count=events_count) if ev else {}
            split_before = clf.launch_counts()
            if inp == "soa":
                if ev:
                    clf.classify_events(batch, events, events_count, results=res, verdicts=ver)
                else:
                    clf.classify(batch, results=res, verdicts=ver)
            elif inp == "compact":
                clf.classify_c(bc, results=res, verdicts=ver)
            elif inp == "xdp":
                clf.classify_xdp(umem, xdesc, n, ring_if, results=res, verdicts=ver)
            else:
                clf.classify_frames(frames, lin, fifx, n, results=res, verdicts=ver, pkt_len=plen, stride=stride,
                                    **evs)
            torch.cuda.synchronize()
            label = f"{name} ({kind}, split={split}, shape={shape}, {inp}, ev={ev}, dbg={dbg})"
            # the launch really took the form the name says (a two-phase launch without scratch would run fused)
            taken, fell_back = (a - b for a, b in zip(clf.launch_counts(), split_before))
            assert (taken, fell_back) == ((1, 0) if "+decide" in name else (0, 0)), (label, taken, fell_back)
            wres, wver, wstats = (xres, xver, xstats) if inp == "xdp" else (ores, over, ostats)
            gres = res.cpu().numpy().view(np.uint32)
            bad = np.nonzero(gres != wres)[0]
            assert bad.size == 0, f"{label}: {bad.size} result words differ, first {bad[:4]}"
            assert np.array_equal(ver.cpu().numpy(), wver), f"{label}: verdicts"
            assert np.array_equal(clf.stats_read_all(), wstats), f"{label}: counters"
            if ev:
                assert int(events_count.item()) == deny, label
            if dbg:
                assert len(clf.debug_keys()) > 0, label
                clf.debug_keys_clear()
            for x in V.names_of(name):
                done[x] = label
        clf.close()
    missing = set(reg) - set(done)
    assert not missing, sorted(missing)
