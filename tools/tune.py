#!/usr/bin/env python3
"""In-process A/B of classify launch shapes on one resident batch (cfg2 by default).

Interleaves variants over several rounds (one process, one device), checks that
every variant's result words are identical to the first one's, and prints the
median/min kernel time (HIP events on the launch stream) and Gpps per variant.
  python tools/tune.py [--cfg 2] [--batch 134217728] [--rounds 5] [--iters 5]
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
    ap.add_argument("--variants", default="768:0:2,512:0:3,512:0:4,256:0:6,512:8:3")
    ap.add_argument("--prefixes", type=int, default=0, help="table size (0 = config default)")
    ap.add_argument("--templates", type=int, default=0, help="distinct rule lists (0 = config default)")
    ap.add_argument("--key-order", choices=("workload", "shuffled"), default="workload",
                    help="table update order (bench.py's default is shuffled)")
    ap.add_argument("--ablate", default="", help="comma list of INFW_ABLATE codes to time (0 = full kernel)")
    args = ap.parse_args()
    import torch
    import infw
    from infw import workloads as W
    from infw.batch import SoaBatch
    dev = torch.device("cuda", 0)
    wl = W.Workload(args.cfg, n_prefixes=args.prefixes, n_templates=args.templates)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf, order=wl.shuffled_order() if args.key_order == "shuffled" else None)
    clf.commit()
    n = args.batch
    batch = SoaBatch.empty(n, dev)
    wl.gen_device(batch, 0, 0)
    res = torch.empty(n, dtype=torch.int32, device=dev)
    ref = None
    # variant "block:group:blocks_per_cu[:c24log]"; --ablate "a,b" times diagnostic builds instead
    variants = [tuple(int(x) for x in v.split(":")) for v in args.variants.split(",")]
    if args.ablate:
        variants = [(512, 0, 3, int(a)) for a in args.ablate.split(",")]
    times = {v: [] for v in variants}
    s = torch.cuda.current_stream()
    for r in range(args.rounds):
        for v in variants:
            clf.set_launch(*v[:3])
            if args.ablate:
                os.environ["INFW_ABLATE"] = str(v[3])
            elif len(v) > 3:
                os.environ["INFW_C24LOG"] = str(v[3])
            else:
                os.environ.pop("INFW_C24LOG", None)
            clf.classify(batch, results=res)  # warm
            torch.cuda.synchronize()
            if ref is None:
                ref = res.clone()
            elif r == 0 and not args.ablate:
                assert torch.equal(res, ref), f"variant {v} differs"
            for _ in range(args.iters):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                clf.classify(batch, results=res)
                b.record(s)
                b.synchronize()
                times[v].append(a.elapsed_time(b))
    out = []
    for v in variants:
        med, mn = statistics.median(times[v]), min(times[v])
        out.append({"block": v[0], "scan_group": v[1], "blocks_per_cu": v[2],
                    "ablate": v[3] if args.ablate else None, "c24log": v[3] if len(v) > 3 and not args.ablate else None,
                    "median_ms": round(med, 3),
                    "min_ms": round(mn, 3), "gpps_median": round(n / med / 1e6, 3)})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
