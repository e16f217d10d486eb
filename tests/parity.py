"""Shared parity helpers for tests/ and __graft_entry__.smoke().

Builds the same table in the GPU classifier (through the C ABI) and in the
oracle, classifies the same packets both ways and compares result words,
XDP verdicts and per-rule counters bit for bit.
"""
from __future__ import annotations

import numpy as np

import infw
import orc
from infw import workloads as W


def oracle_for(wl: W.Workload) -> "orc.OracleMap":
    m = orc.OracleMap(max_entries=wl.n_entries + 16)
    for k, v in wl.entries():
        rc = m.update(k, v)
        assert rc == 0, rc
    return m


def oracle_run(m, wl: W.Workload, start: int, n: int, threads: int = 8):
    hdr, cap, pl, ifx = wl.frames(start, n)
    res, ver, stats, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=threads)
    return res, ver, stats, (hdr, cap, pl, ifx)


def gpu_run(clf, batch, n: int, dev_index: int = 0):
    """Classify a device SoA batch; returns (results u32, verdicts u8) on the host."""
    import torch
    res = torch.empty(n, dtype=torch.int32, device=batch.device)
    ver = torch.empty(n, dtype=torch.uint8, device=batch.device)
    clf.classify(batch, results=res, verdicts=ver, dev=dev_index)
    torch.cuda.synchronize(batch.device)
    return res.cpu().numpy().view(np.uint32), ver.cpu().numpy()


def stats_from_results(results: np.ndarray, pkt_len: np.ndarray) -> np.ndarray:
    """Per-rule counters implied by result words (kernel.c:441-456, :376-387)."""
    out = np.zeros((1024, 4), np.uint64)
    act = results & 0xFF
    key = (results >> 8) & 0xFFFF
    for a, col in ((infw.XDP_PASS, 0), (infw.XDP_DROP, 2)):
        sel = (act == a) & (key < 1024)
        out[:, col] += np.bincount(key[sel], minlength=1024).astype(np.uint64)
        out[:, col + 1] += np.bincount(key[sel], weights=pkt_len[sel].astype(np.float64),
                                       minlength=1024).astype(np.uint64)
    return out


def check_cfg(cfg: int, n: int, n_prefixes: int = 0, n_templates: int = 0, start: int = 0, device=None,
              layout: str = "standard", launch=None):
    """End-to-end parity on one config: device-generated SoA vs host frames + oracle.
    layout "compact": the batch is re-laid out by infw_soa_compact and classified by infw_classify_c."""
    import torch
    from infw.batch import SoaBatch
    device = device or torch.device("cuda", 0)
    wl = W.Workload(cfg, n_prefixes=n_prefixes, n_templates=n_templates)
    clf = infw.Classifier(devices=[device.index or 0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    if launch is not None:
        clf.set_launch(*launch)
    m = oracle_for(wl)
    ores, over, ostats, (hdr, cap, pl, ifx) = oracle_run(m, wl, start, n)
    batch = SoaBatch.empty(n, device)
    wl.gen_device(batch, start, device.index or 0)
    torch.cuda.synchronize(device)
    host_tuples = W.pack_frames(hdr, cap, pl, ifx)
    dev_tuples = batch.to_tuples()
    assert np.array_equal(dev_tuples, host_tuples), "device generator != host frames packed"
    clf.stats_reset()
    if layout == "compact":
        bc = clf.compact(batch)
        res = torch.empty(n, dtype=torch.int32, device=device)
        ver = torch.empty(n, dtype=torch.uint8, device=device)
        clf.classify_c(bc, results=res, verdicts=ver)
        torch.cuda.synchronize(device)
        gres, gver = res.cpu().numpy().view(np.uint32), ver.cpu().numpy()
    else:
        gres, gver = gpu_run(clf, batch, n)
    gstats = clf.stats_read_all()
    return dict(wl=wl, clf=clf, oracle=m, ores=ores, over=over, ostats=ostats, gres=gres, gver=gver,
                gstats=gstats, pkt_len=pl, batch=batch)


def assert_parity(r, label=""):
    bad = np.nonzero(r["gres"] != r["ores"])[0]
    assert bad.size == 0, f"{label}: {bad.size} result words differ, first {bad[:8]}: " \
                          f"gpu={r['gres'][bad[:8]]} oracle={r['ores'][bad[:8]]}"
    assert np.array_equal(r["gver"], r["over"]), f"{label}: verdicts differ"
    assert np.array_equal(r["gstats"], r["ostats"]), f"{label}: per-rule counters differ"
