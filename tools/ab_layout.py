#!/usr/bin/env python3
"""In-process A/B of the two batch layouts on one resident batch (cfg2 by default):
infw_classify on the standard 16-B address layout vs infw_classify_c on the family-compact
layout (infw_soa_compact of the same batch).  Checks the result words are identical, then
interleaves timed launches (HIP events on the launch stream) and prints median/min per layout.
  python tools/ab_layout.py [--cfg 2] [--batch 134217728] [--rounds 5] [--iters 5]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ingress-node-firewall_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1 << 27)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    import torch
    import infw
    from infw import workloads as W
    from infw.batch import SoaBatch
    dev = torch.device("cuda", 0)
    wl = W.Workload(args.cfg)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    n = args.batch
    batch = SoaBatch.empty(n, dev)
    wl.gen_device(batch, 0, 0)
    bc = clf.compact(batch)
    r0 = torch.empty(n, dtype=torch.int32, device=dev)
    r1 = torch.empty(n, dtype=torch.int32, device=dev)
    clf.classify(batch, results=r0)
    clf.classify_c(bc, results=r1)
    torch.cuda.synchronize()
    assert torch.equal(r0, r1), "compact layout results differ"
    runs = {"standard": lambda: clf.classify(batch, results=r0), "compact": lambda: clf.classify_c(bc, results=r1)}
    times = {k: [] for k in runs}
    s = torch.cuda.current_stream()
    for _ in range(args.rounds):
        for k, f in runs.items():
            f()
            for _ in range(args.iters):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                f()
                b.record(s)
                b.synchronize()
                times[k].append(a.elapsed_time(b))
    v6 = float(((batch.meta & 0xFFFF) == 0x86DD).float().mean())
    for k, t in times.items():
        med = statistics.median(t)
        print(json.dumps({"layout": k, "cfg": args.cfg, "median_ms": round(med, 4), "min_ms": round(min(t), 4),
                          "gpps": round(n / med / 1e6, 2), "ipv6_share": round(v6, 4)}), flush=True)


if __name__ == "__main__":
    main()
