#!/usr/bin/env python3
"""Summarise tools/lds_ablate.sh (gpurun_out/lds_<tag>) into profiles/<tag>/lds_ablate.json: per variant the
classify kernel's average duration and its LDS counters per launch, and the attribution of bank-conflict cycles
to each LDS structure (default minus the variant without it)."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = {0: "default", 1: "no word cache", 2: "no IPv6 group cache", 4: "no LDS counters", 7: "none of the three"}


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", f"lds_{tag}")
    out = {"tag": tag, "variants": {}}
    for v in NAMES:
        d = os.path.join(src, f"v{v}")
        kt = glob.glob(os.path.join(d, "kt", "**", "kt_kernel_stats.csv"), recursive=True)
        pm = glob.glob(os.path.join(d, "lds", "**", "lds_counter_collection.csv"), recursive=True)
        if not kt or not pm:
            continue
        rows = [r for r in csv.DictReader(open(kt[0])) if "classify" in r["Name"]]
        main_row = max(rows, key=lambda r: int(r["Calls"]))
        name = main_row["Name"]
        acc = {}
        for r in csv.DictReader(open(pm[0])):
            if r["Kernel_Name"] == name:
                acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        avg = {k: sum(x) / len(x) for k, x in acc.items()}
        line = [l for l in open(os.path.join(d, "kt.stdout")) if l.startswith("{")]
        out["variants"][v] = {"what": NAMES[v], "kernel_avg_ns": float(main_row["AverageNs"]), "pmc": avg,
                              "bank_conflict_rate": avg["SQ_LDS_BANK_CONFLICT"] / max(avg["SQ_LDS_IDX_ACTIVE"], 1),
                              "build_id": json.loads(line[-1]).get("build_id") if line else None}
    base = out["variants"].get(0)
    if base:
        for v, r in out["variants"].items():
            if v:
                r["conflict_cycles_removed"] = base["pmc"]["SQ_LDS_BANK_CONFLICT"] - r["pmc"]["SQ_LDS_BANK_CONFLICT"]
                r["share_of_default_conflicts"] = r["conflict_cycles_removed"] / base["pmc"]["SQ_LDS_BANK_CONFLICT"]
    os.makedirs(os.path.join(ROOT, "profiles", tag), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "profiles", tag, "lds_ablate.json"), "w"), indent=1)
    for v, r in out["variants"].items():
        print(v, r["what"], round(r["kernel_avg_ns"] / 1e6, 4), "ms", "conflict rate", round(r["bank_conflict_rate"], 3),
              "share removed", round(r.get("share_of_default_conflicts", 0), 3))


if __name__ == "__main__":
    main()
