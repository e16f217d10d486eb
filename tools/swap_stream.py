#!/usr/bin/env python3
"""configs[4] with live rule-table swaps mid-stream: classify throughput with commits between batches.

Loads the adversarial table (IPv6 /128 deepest-prefix hits, last-slot ICMPv6 type/code rules,
cross-family aliasing keys), then streams K resident batches through classify on one stream.
Between batches it applies E key edits — each rewrites an existing key's value with another
rule list (or deletes and re-adds it) — and commits them (an incremental epoch swap,
DESIGN.md §4).  Reports Gpps with no edits, and with E edits committed after every batch
(commit wall time included), plus the commit latency; the final per-rule totals are checked
against the sum of the per-batch packet counts (stats persist across swaps).
  python tools/swap_stream.py [--batch 16777216] [--batches 24] [--edits 1,100,1000]
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
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--batches", type=int, default=24)
    ap.add_argument("--edits", default="1,100,1000")
    args = ap.parse_args()
    import numpy as np
    import torch
    import infw
    from infw import workloads as W
    from infw.batch import SoaBatch

    dev = torch.device("cuda", 0)
    wl = W.Workload(W.CFG4_ADVERSARIAL)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 4096)
    wl.load_into(clf)
    t0 = time.time()
    clf.commit()
    print(json.dumps({"cfg": 4, "entries": wl.n_entries, "initial_commit_s": round(time.time() - t0, 2)}), flush=True)
    keys = wl.keys_bytes().reshape(-1, 24)
    tmpl = np.ascontiguousarray(wl.templates_bytes().reshape(-1, 1200))
    n = args.batch
    batches = [SoaBatch.empty(n, dev) for _ in range(2)]
    for j, b in enumerate(batches):
        wl.gen_device(b, j * n, 0)
    res = torch.empty(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    rng = np.random.default_rng(7)

    def edit_sets(edits):
        """Per batch: `edits` existing keys rewritten with other rule lists (one batch update), 1/16 of them deleted
        first and re-added by that update — drawn before the timed loop (the syncer's diff is an input here)."""
        out = []
        for _ in range(args.batches):
            idx = rng.integers(keys.shape[0], size=edits)  # repeats are fine
            dels = np.ascontiguousarray(keys[np.unique(idx[: edits // 16])])  # every key is present
            sel = np.ascontiguousarray(keys[idx])
            vi = rng.integers(tmpl.shape[0], size=edits).astype(np.uint32)
            out.append((dels, sel, vi))
        return out

    def run(edits):
        sets = edit_sets(edits) if edits else None
        clf.stats_reset()
        commit_ms = []
        torch.cuda.synchronize()
        ts = time.perf_counter()
        edit_ms = []
        for k in range(args.batches):
            clf.classify(batches[k & 1], results=res)
            if edits:
                e0 = time.perf_counter()
                dels, sel, vi = sets[k]
                clf.delete_batch_ptr(dels.ctypes.data, dels.shape[0])
                clf.update_batch_ptr(sel.ctypes.data, tmpl.ctypes.data, vi.ctypes.data, edits)
                c0 = time.perf_counter()
                edit_ms.append((c0 - e0) * 1e3)
                clf.commit()  # epoch swap: the next batch reads the new epoch, this one finishes on the old
                commit_ms.append((time.perf_counter() - c0) * 1e3)
        torch.cuda.synchronize()
        wall = time.perf_counter() - ts
        st = clf.stats_read_all()
        run.edit_ms = sorted(edit_ms)
        return wall, commit_ms, int(st[:, 0].sum() + st[:, 2].sum())

    run(0)  # warm
    run(1)  # warm the commit path (staging buffers, events)
    base, _, counted0 = run(0)
    out = {"batch": n, "batches": args.batches, "edits_per_commit": 0,
           "gpps": round(n * args.batches / base / 1e9, 2), "counted": counted0}
    print(json.dumps(out), flush=True)
    for e in [int(x) for x in args.edits.split(",")]:
        wall, cms, counted = run(e)
        cms.sort()
        print(json.dumps({"batch": n, "batches": args.batches, "edits_per_commit": e,
                          "gpps": round(n * args.batches / wall / 1e9, 2),
                          "commit_ms_median": round(cms[len(cms) // 2], 2), "commit_ms_max": round(cms[-1], 2),
                          "edit_ms_median": round(run.edit_ms[len(run.edit_ms) // 2], 2),
                          "commit_mode": clf.info()["commit_mode"], "full_reason": clf.info()["full_reason"],
                          "counted": counted}), flush=True)


if __name__ == "__main__":
    main()
