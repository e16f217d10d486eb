#!/usr/bin/env python3
"""Summarize tools/profile_lat.sh runs (gpurun_out/lat_<tag>) into one JSON: per classify launch, the L1->L2 read
latency, requests per packet and the SQ wave-state split per 64-packet tile (SQ_WAVE_CYCLES and the wait/active
counters are in 4-cycle units on gfx950; ratios are taken as measured).
Usage: tools/summarize_lat.py <out.json> <tag>[=label[:n_packets]] ...  (n_packets per launch, default 2^27)"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(tag):
    acc = collections.defaultdict(list)
    d = os.path.join(ROOT, "gpurun_out", f"lat_{tag}")
    for p in ("lat_tcp", "lat_ta", "lat_sq", "lat_wait"):
        f = os.path.join(d, p, f"{p}_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            if "classify_kernel" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    line = [l for l in open(os.path.join(d, "lat_tcp.stdout")) if l.startswith("{")]
    return {k: sum(v) / len(v) for k, v in acc.items()}, json.loads(line[-1]) if line else {}


def main():
    out = {}
    for arg in sys.argv[2:]:
        tag, _, label = arg.partition("=")
        label, _, ns = label.partition(":")
        n = int(ns) if ns else 1 << 27
        tiles = n / 64
        a, line = load(tag)
        wc = a.get("SQ_WAVE_CYCLES", 0.0)
        out[label or tag] = {
            "build_id": line.get("build_id"), "workload_key": line.get("config", {}).get("workload_key"),
            "kernel_ms_avg": line.get("roofline", {}).get("kernel_ms_avg"),
            "l1_l2_read_latency_cycles": a["TCP_TCC_READ_REQ_LATENCY_sum"] / a["TCP_TCC_READ_REQ_sum"],
            "l1_l2_read_requests_per_packet": a["TCP_TCC_READ_REQ_sum"] / n,
            "lds_bank_conflict_rate": (a["SQ_LDS_BANK_CONFLICT"] / a["SQ_LDS_IDX_ACTIVE"]
                                       if a.get("SQ_LDS_IDX_ACTIVE") else None),
            "per_tile": {k: a[c] / tiles for k, c in (("valu", "SQ_INSTS_VALU"), ("salu", "SQ_INSTS_SALU"),
                                                     ("lds", "SQ_INSTS_LDS"), ("vmem_rd", "SQ_INSTS_VMEM_RD"),
                                                     ("wave_cycles_x4", "SQ_WAVE_CYCLES")) if c in a},
            "wave_state_fraction": {k: a[c] / wc for k, c in (("dependency_wait", "SQ_WAIT_ANY"),
                                                              ("issue_wait", "SQ_WAIT_INST_ANY"),
                                                              ("lds_issue_wait", "SQ_WAIT_INST_LDS"),
                                                              ("active_any", "SQ_ACTIVE_INST_ANY"),
                                                              ("active_valu", "SQ_ACTIVE_INST_VALU"),
                                                              ("active_salu", "SQ_ACTIVE_INST_SCA"),
                                                              ("active_lds", "SQ_ACTIVE_INST_LDS")) if c in a and wc},
            "raw_per_launch": a,
        }
    json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
