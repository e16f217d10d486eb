#!/usr/bin/env python3
"""In-process A/B of table-layout variants on one resident batch (cfg2 by default).

Each variant is a set of environment settings read by the table compiler at
commit time (e.g. INFW_DT_FORM=wide, INFW_SHORT_TABLE=compressed); every
variant gets its own Classifier (own device tables) over the same packets.
Variants are interleaved over several rounds; result words and per-rule
counters must be identical across variants.  Prints one JSON line per variant.
  python tools/ab_tables.py --variants "base;INFW_DT_FORM=wide" [--cfg 2] [--rounds 5]
With --launch the settings are launch-time ones (e.g. INFW_NT=4, read by
infw_launch_classify): one Classifier, the variant's environment applied
around each of its launches.
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
    ap.add_argument("--variants", default="base;INFW_DT_FORM=wide")
    ap.add_argument("--prefixes", type=int, default=0, help="table size (0 = config default)")
    ap.add_argument("--templates", type=int, default=0,
                    help="distinct rule lists (0 = config default; >= prefixes: one list per key)")
    ap.add_argument("--key-order", choices=("workload", "shuffled"), default="workload",
                    help="table update order (bench.py's default is shuffled)")
    ap.add_argument("--uniform", action="store_true", help="sources uniform over the prefixes (bench.py --uniform)")
    ap.add_argument("--launch", action="store_true", help="variants are launch-time settings (one table image)")
    args = ap.parse_args()
    import torch
    import infw
    from infw import workloads as W
    from infw.batch import SoaBatch
    dev = torch.device("cuda", 0)
    wl = W.Workload(args.cfg, n_prefixes=args.prefixes, n_templates=args.templates)
    if args.uniform:
        wl.uniform_sources()
    n = args.batch
    batch = SoaBatch.empty(n, dev)
    wl.gen_device(batch, 0, 0)
    res = torch.empty(n, dtype=torch.int32, device=dev)
    names = [v.strip() for v in args.variants.split(";")]
    clfs = {}
    envs = {v: dict(kv.split("=", 1) for kv in v.split(",") if "=" in kv) for v in names}

    class applied:  # the variant's environment, restored on exit
        def __init__(self, env):
            self.env = env

        def __enter__(self):
            self.saved = {k: os.environ.get(k) for k in self.env}
            os.environ.update(self.env)

        def __exit__(self, *a):
            for k, old in self.saved.items():
                if old is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = old

    shared = None
    for v in names:
        if args.launch and shared is not None:
            clfs[v] = shared
            continue
        with applied({} if args.launch else envs[v]):
            c = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
            wl.load_into(c, order=wl.shuffled_order() if args.key_order == "shuffled" else None)
            c.commit()
        info = c.info()
        print(f"[ab] {v}: {info['device_bytes'] / 2**20:.0f} MiB, compile {info['compile_ms']:.0f} ms, "
              f"upload {info['upload_ms']:.0f} ms, lists {info['n_lists']}, parts {info['dt_parts']}",
              file=sys.stderr, flush=True)
        clfs[v] = shared = c
    ref = None
    times = {v: [] for v in names}
    s = torch.cuda.current_stream()
    for r in range(args.rounds):
        for v in names:
            c = clfs[v]
            with applied(envs[v] if args.launch else {}):
                c.stats_reset()
                c.classify(batch, results=res)
                torch.cuda.synchronize()
                if r == 0:
                    got = (res.clone(), c.stats_read_all())
                    if ref is None:
                        ref = got
                    else:
                        assert torch.equal(got[0], ref[0]), f"variant {v}: result words differ"
                        assert (got[1] == ref[1]).all(), f"variant {v}: counters differ"
                for _ in range(args.iters):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(s)
                    c.classify(batch, results=res)
                    b.record(s)
                    b.synchronize()
                    times[v].append(a.elapsed_time(b))
    for v in names:
        t = times[v]
        print(json.dumps({"variant": v, "median_ms": round(statistics.median(t), 4), "min_ms": round(min(t), 4),
                          "gpps": round(n / statistics.median(t) / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
