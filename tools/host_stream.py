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
    # the device-resident rate of the same packets, for reference
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
