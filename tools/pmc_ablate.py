#!/usr/bin/env python3
"""Per-variant PMC averages of a tools/pmc_ablate.sh run: counters per launch and
per packet for every classify instantiation (kernel names carry the ablation code).
Usage: tools/pmc_ablate.py <tag> [n_packets]"""
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 27
    src = os.path.join(ROOT, "gpurun_out", f"pmcab_{tag}")
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for name in sorted(os.listdir(src)):
        p = os.path.join(src, name, f"{name}_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            if "classify" not in k:
                continue
            m = re.search(r"classify_kernel<(\d+), (\d+), (\d+)", k)
            key = f"ablate={m.group(3)}" if m else k[:60]
            vals[key][(r["Counter_Name"], r.get("Dispatch_Id", ""))].append(float(r["Counter_Value"]))
    out = {}
    for key, d in vals.items():
        per = collections.defaultdict(list)
        for (cname, _), v in d.items():
            per[cname].append(sum(v))  # one dispatch: sum over dimensions
        out[key] = {c: {"per_launch": sum(v) / len(v), "per_packet": sum(v) / len(v) / n} for c, v in per.items()}
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
