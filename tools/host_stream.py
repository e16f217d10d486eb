#!/usr/bin/env python3
"""PCIe-inclusive throughput: configs[2] batches resident in HOST memory, classified
through infw_classify_host (chunked H2D / kernel / D2H on three HIP streams).

Reports Mpps for page-locked (registered) host memory and for pageable memory,
plus the H2D bytes rate the pinned run implies (32 B in + 4 B out per packet).
  python tools/host_stream.py [--n 67108864] [--chunk 4194304] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ingress-node-firewall_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 26)
    ap.add_argument("--chunk", type=int, default=1 << 22)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--per-call", default="",
                    help="comma-separated packets per call: the per-call cost of infw_classify_host on the pinned "
                         "batch cut into calls of that size")
    args = ap.parse_args()
    import numpy as np
    import infw
    from infw import workloads as W
    wl = W.Workload(W.CFG2_MIXED_1M)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    n = args.n
    soa = infw.HostSoa.from_tuples(wl.tuples(0, n))
    res = np.zeros(n, np.uint32)
    out = {"workload": "cfg2 (1M prefixes, 4096 lists)", "packets": n, "chunk": args.chunk}
    for mode in ("pageable", "pinned"):
        if mode == "pinned":
            for a in soa.arrays() + (res,):
                clf.host_register(a)
        clf.classify_host(soa, res, chunk=args.chunk)  # warm (pipeline buffers, page faults)
        ts = []
        for _ in range(args.reps):
            t = time.perf_counter()
            clf.classify_host(soa, res, chunk=args.chunk)
            ts.append(time.perf_counter() - t)
        best = min(ts)
        out[mode] = {"mpps": round(n / best / 1e6, 1), "s": round(best, 4),
                     "h2d_GB_per_s": round(32 * n / best / 1e9, 1), "d2h_GB_per_s": round(4 * n / best / 1e9, 1)}
    print(json.dumps(out), flush=True)
    for per in [int(x) for x in args.per_call.split(",") if x]:  # (the pinned batch, still registered)
        parts = [(soa.slice(a, min(n, a + per)), res[a:min(n, a + per)]) for a in range(0, n, per)]
        for s, r in parts[:4]:
            clf.classify_host(s, r)
        best = 1e30
        for _ in range(args.reps):
            t = time.perf_counter()
            for s, r in parts:
                clf.classify_host(s, r)
            best = min(best, time.perf_counter() - t)
        print(json.dumps({"per_call": per, "calls": len(parts), "us_per_call": round(best / len(parts) * 1e6, 1),
                          "mpps": round(n / best / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
