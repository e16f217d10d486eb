#!/usr/bin/env python3
"""Same-process sweep of the launch shapes infw_set_launch accepts (include/infw.h) on one bench workload: the
resident batch classified K times per shape, shapes alternated R times, kernel time by HIP events on the launch
stream.  The registry name of each shape's instantiation is printed beside it.
  python tools/shape_sweep.py [--cfg 2] [--layout standard|compact] [--reps 2] [--launches 10]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ingress-node-firewall_amd")]

SHAPES = [(768, 0, 2), (512, 0, 2), (512, 0, 3), (512, 0, 4), (256, 0, 6)]  # decision tables (group 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=2)
    ap.add_argument("--layout", default="standard", choices=("standard", "compact"))
    ap.add_argument("--batch", type=int, default=1 << 27)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--launches", type=int, default=10)
    args = ap.parse_args()
    import torch
    import infw
    from infw import workloads as W
    from infw.batch import SoaBatch

    cfg = {1: W.CFG1_V4_10K, 2: W.CFG2_MIXED_1M, 4: W.CFG4_ADVERSARIAL}[args.cfg]
    wl = W.Workload(cfg)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    dev = torch.device("cuda", 0)
    n = args.batch
    batch = SoaBatch.empty(n, dev)
    wl.gen_device(batch, start=0, dev_ordinal=0)
    bc = clf.compact(batch) if args.layout == "compact" else None
    res = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    ref = None
    out = {}
    for rep in range(args.reps):
        for shape in SHAPES:
            clf.set_launch(*shape)
            name = clf.variant(infw.INPUT_COMPACT if bc is not None else infw.INPUT_SOA)
            run = (lambda: clf.classify_c(bc, results=res)) if bc is not None else (lambda: clf.classify(batch, results=res))
            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = res.clone()
            assert torch.equal(res, ref), shape  # every shape gives the same words
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.launches):
                run()
            e1.record(stream)
            e1.synchronize()
            ms = e0.elapsed_time(e1) / args.launches
            out.setdefault(str(shape), []).append(round(ms, 4))
            print(json.dumps({"rep": rep, "shape": shape, "kernel": name, "ms": round(ms, 4),
                              "Gpps": round(n / ms / 1e6, 1)}), flush=True)
    print(json.dumps({"summary_ms": out, "cfg": args.cfg, "layout": args.layout, "packets": n}), flush=True)


if __name__ == "__main__":
    main()
