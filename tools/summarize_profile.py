#!/usr/bin/env python3
"""Summarize a tools/profile.sh run (gpurun_out/prof_<tag>) into profiles/<tag>/.

Copies the rocprofv3 --stats summaries and writes summary.json with, for the
classify kernel: average duration (kernel trace), per-launch PMC values, and
the HBM traffic per launch corrected as MI355X_MICROARCH.md §HBM prescribes:
  FETCH_SIZE, WRITE_SIZE are in KiB; FETCH_SIZE reads exactly half the bytes of
  a wide coalesced streaming read (gfx950), exact for other shapes only after
  calibration.  The classify kernel's streamed input is known exactly
  (32 B/packet in the standard layout, algorithmic bytes - 4 in the family-compact one, both from the
  bench line), so   read_bytes = FETCH_SIZE*1024 + 0.5 * stream_bytes * n_packets
  (the un-counted half of the stream); gathers are taken at face value
  (64-B requests).  The uncorrected value is kept beside it.
Also writes profiles/traffic_<workload_key>.json (per-packet figures + kernel) that bench.py reads.
Usage: tools/summarize_profile.py <tag> [n_packets]
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 27
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    # the profiled command's bench line names the workload (profiles/traffic_<workload_key>.json, which bench.py
    # reads beside a line of the same workload, kernel and layout)
    bl = [l for l in open(os.path.join(src, "kt.stdout")) if l.startswith("{")] if os.path.exists(
        os.path.join(src, "kt.stdout")) else []
    line = json.loads(bl[-1]) if bl else {}
    key = line.get("config", {}).get("workload_key", "cfg2")
    if os.environ.get("PROFILE_KEY"):  # a line profiled before bench.py named its table size in the key
        key = os.environ["PROFILE_KEY"]
    layout = line.get("roofline", {}).get("layout", "standard")
    if layout == "compact" and not key.endswith("_compact") and "_frames" not in key:  # lines before round 4's key
        key += "_compact"
    if line:
        n = line["config"]["packets_per_gpu_per_step"]
        # an AF_XDP line launches once per interface ring: a launch classifies 1 / rings of the step's frames on
        # average, which is what the per-launch PMC averages below are divided by
        rings = line.get("roofline", {}).get("xdp_ring", {}).get("rings")
        if rings:
            n = n / rings
    stream_b = 32.0  # tuple bytes read per packet
    if layout == "compact":
        stream_b = line["roofline"]["algorithmic_bytes_per_packet"] - 4
    elif layout == "frames":  # infw_classify_frames: the 12 B of length/ifindex streams; the 64-B frame windows
        stream_b = 12.0       # (one per frame at the frame stride) are counted at face value, like gathers
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    for f in ("kt/kt_kernel_stats.csv", "kt/kt_domain_stats.csv"):
        p = os.path.join(src, f)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, os.path.basename(p)))
    out = {"tag": tag, "workload_key": key, "packets_per_launch": n, "kernels": {}}
    stats = list(csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv"))))
    # the profiled kernel: the classify instantiation launched most (a bench may run another one untimed, e.g. the
    # packer path's classify_c that --fused checks its results against); PMC rows are filtered to it as well
    cls = [r for r in stats if "classify" in r["Name"]]
    main_name = max(cls, key=lambda r: int(r["Calls"]))["Name"] if cls else ""
    # the two-phase form (classify.hip launch_split): phase 1 is a classify_kernel instantiation, phase 2 the
    # decide_kernel launched as often — one classification is the pair, so times and counters are summed over both
    calls = next((int(r["Calls"]) for r in stats if r["Name"] == main_name), 0)
    names = [main_name] + [r["Name"] for r in stats if "decide_kernel" in r["Name"] and int(r["Calls"]) == calls]
    names = list(dict.fromkeys(names))
    out["split"] = len(names) > 1
    for r in stats:
        if r["Name"] in names:
            out["kernels"][r["Name"][:80]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                              "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
    out["avg_ns_per_classification"] = sum(k["avg_ns"] for k in out["kernels"].values())
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for name in sorted(os.listdir(src)):
        p = os.path.join(src, name, f"{name}_counter_collection.csv")
        if not name.startswith("pmc") or not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            if r["Kernel_Name"] in names:
                pmc[r["Counter_Name"]][r["Kernel_Name"]].append(float(r["Counter_Value"]))
    # per classification: each kernel's average per launch, summed over the kernels of the pair
    avg = {k: sum(sum(v) / len(v) for v in per.values()) for k, per in pmc.items()}
    out["pmc_avg_per_launch"] = avg
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        raw = (avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
        corr = avg["FETCH_SIZE"] * 1024 + 0.5 * stream_b * n + avg["WRITE_SIZE"] * 1024
        out["hbm_bytes_per_launch_raw"] = raw
        out["hbm_bytes_per_launch"] = corr
        out["hbm_bytes_per_packet"] = corr / n
        out["hbm_bytes_per_packet_raw"] = raw / n
    if "TCC_HIT_sum" in avg:
        out["l2_hit_rate"] = avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
        out["l2_misses_per_packet"] = avg["TCC_MISS_sum"] / n
        out["l2_hits_per_packet"] = avg["TCC_HIT_sum"] / n
    if "SQ_LDS_BANK_CONFLICT" in avg:
        out["lds_bank_conflict_rate"] = avg["SQ_LDS_BANK_CONFLICT"] / max(1.0, avg["SQ_LDS_IDX_ACTIVE"])
    if "TCC_EA0_RDREQ_sum" in avg:  # fabric read requests: one per 128-B line (MI355X_MICROARCH.md §HBM)
        out["ea_rdreq_per_packet"] = avg["TCC_EA0_RDREQ_sum"] / n
    if "GRBM_GUI_ACTIVE" in avg and out["kernels"]:
        out["effective_clock_ghz"] = avg["GRBM_GUI_ACTIVE"] / 8 / out["avg_ns_per_classification"]
    if line:
        out["bench_line_under_kernel_trace"] = line
    json.dump(out, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    # the traffic file bench.py reads for this workload: every figure from this one profile
    if line and "hbm_bytes_per_packet" in out:
        # (the line rates the bench's random_line_model prices these counts with are measured by bench.py itself,
        # in its own process, before its timed loop — not stored here)
        tj = {"tag": tag, "workload_key": key, "build_id": line.get("build_id"), "kernel": line["roofline"]["kernel"],
              "layout": layout, "note": f"classify kernel, {key} bench command; see profiles/{tag}/summary.json"}
        for k in ("hbm_bytes_per_packet", "hbm_bytes_per_packet_raw", "l2_hits_per_packet", "l2_misses_per_packet",
                  "lds_bank_conflict_rate", "ea_rdreq_per_packet"):
            if k in out:
                tj[k] = out[k]
        json.dump(tj, open(os.path.join(ROOT, "profiles", f"traffic_{key}.json"), "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "bench_line_under_kernel_trace"}, indent=1))


if __name__ == "__main__":
    main()
