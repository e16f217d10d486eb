#!/usr/bin/env python3
"""Diagnostic: what wave divergence between IPv4 and IPv6 lanes costs the classify kernel.  The same batch is
classified as generated and with each window of W packets stably sorted by address family (so all but one wave of
a window runs one family's path); alternated timings of the same kernel on the same packets.  The per-rule
counters must agree (a permutation).  Usage (GPU box): tools/ab_family_sort.py [--cfg C] [--windows 768,6144]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ingress-node-firewall_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import infw  # noqa: E402
from infw import workloads as W  # noqa: E402
from infw.batch import SoaBatch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=2)
    ap.add_argument("--n", type=int, default=(1 << 27) - (1 << 27) % 6144)  # whole windows
    ap.add_argument("--windows", default="768,6144")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    wl = W.Workload(a.cfg)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf, order=wl.shuffled_order())
    clf.commit()
    base = SoaBatch.empty(a.n, dev)
    wl.gen_device(base, start=0, dev_ordinal=0)
    torch.cuda.synchronize()
    fam = ((base.meta & 0xFFFF) == 0x86DD).to(torch.int64)
    variants = {"generated": base}
    chunk = 1 << 22  # permutations built and applied per chunk of whole windows (one huge index launch fails)
    for w in [int(x) for x in a.windows.split(",") if x]:
        b = SoaBatch.empty(a.n, dev)
        for c0 in range(0, a.n, chunk - chunk % w):
            c1 = min(a.n, c0 + chunk - chunk % w)
            f = fam[c0:c1].reshape(-1, w)  # (windows, w): IPv4 lanes first, IPv6 after, each in order
            c6 = torch.cumsum(f, dim=1)
            c4 = torch.cumsum(1 - f, dim=1)
            n4 = c4[:, -1:]
            dst = torch.where(f == 1, n4 + c6 - 1, c4 - 1) + torch.arange(f.shape[0], device=dev).unsqueeze(1) * w
            dst = dst.reshape(-1) + c0
            b.saddr.view(torch.int64).reshape(a.n, 2).index_copy_(0, dst, base.saddr[c0:c1].view(torch.int64).reshape(-1, 2))
            for name in ("ifindex", "pkt_len", "meta", "l4word"):
                getattr(b, name).index_copy_(0, dst, getattr(base, name)[c0:c1])
        variants[f"sorted_w{w}"] = b
    res = torch.empty(a.n, dtype=torch.int32, device=dev)
    ver = torch.empty(a.n, dtype=torch.uint8, device=dev)
    stats = {}
    times = {k: [] for k in variants}
    for k, b in variants.items():  # warm-up and counter check
        clf.stats_reset()
        clf.classify(b, results=res, verdicts=ver)
        torch.cuda.synchronize()
        stats[k] = clf.stats_read_all()
    ok = all(np.array_equal(stats["generated"], s) for s in stats.values())
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rep in range(a.reps):
        for k, b in variants.items():
            torch.cuda.synchronize()
            s0.record()
            for _ in range(a.iters):
                clf.classify(b, results=res, verdicts=ver)
            s1.record()
            torch.cuda.synchronize()
            times[k].append(s0.elapsed_time(s1) / a.iters)
    six = float(fam.float().mean().item())
    out = {"cfg": a.cfg, "n": a.n, "ipv6_share": six, "counters_equal": ok, "build_id": infw.build_id(),
           "ms_per_batch": {k: [round(t, 4) for t in v] for k, v in times.items()},
           "gpps_best": {k: round(a.n / min(v) / 1e6, 2) for k, v in times.items()}}
    print(json.dumps(out))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
