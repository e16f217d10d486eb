#!/usr/bin/env python3
"""Summarize tools/profile_lat.sh runs (gpurun_out/lat_<tag>) into one JSON: per classify launch, the memory path's
latency and occupancy and what bounds the kernel by Little's law at the L1 (TCP):

  in_flight_per_cu = (L1->L2 read requests per CU per cycle) x (average L1->L2 request latency, cycles)

with the CU's cycles taken from GRBM_GUI_ACTIVE per XCD (the clock the counters ran at).  A kernel whose in-flight
count sits at the same level across workloads whose bytes, hit rates and latencies differ is bound by the L1's
outstanding-request capacity: its rate = capacity / latency, and its levers are fewer requests per packet or a shorter
request latency — not bytes.  Also: rocprofv3's VmemLatency / LdsLatency (cycles per instruction), the SQ wave-state
split (4-cycle units on gfx950; fractions as measured), the TA/TD/TCP stall fractions of CU-cycles, L2 hits / misses
per packet.
Usage: tools/summarize_lat.py <out.json> <tag> [<tag> ...]   (tags as profile_lat.sh wrote them, e.g. r06g_cfg1)"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_CU, N_XCD = 256, 8


def load(tag):
    acc = collections.defaultdict(list)
    d = os.path.join(ROOT, "gpurun_out", f"lat_{tag}")
    for f in sorted(glob.glob(os.path.join(d, "*", "*_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if "classify_kernel" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    line = [l for l in open(os.path.join(d, "lat_tcp.stdout")) if l.startswith("{")]
    return {k: sum(v) / len(v) for k, v in acc.items()}, json.loads(line[-1])


def main():
    out = {}
    for tag in sys.argv[2:]:
        a, line = load(tag)
        n = line["config"]["packets_per_gpu_per_step"]
        cyc_xcd = a["GRBM_GUI_ACTIVE"] / N_XCD      # cycles of one launch, per XCD
        cu_cycles = cyc_xcd * N_CU
        req = a["TCP_TCC_READ_REQ_sum"]
        lat = a["TCP_TCC_READ_REQ_LATENCY_sum"] / req
        wc = a["SQ_WAVE_CYCLES"]
        out[tag] = {
            "build_id": line.get("build_id"), "workload_key": line["config"].get("workload_key"),
            "kernel": line["roofline"].get("kernel"), "packets_per_launch": n,
            "kernel_ms_avg_traced_run": line["roofline"].get("kernel_ms_avg"),
            "clock_GHz_from_grbm": round(cyc_xcd / (line["roofline"]["kernel_ms_avg"] * 1e-3) / 1e9, 3),
            "l1_l2_read_requests_per_packet": round(req / n, 4),
            "l1_l2_read_latency_cycles": round(lat, 1),
            "l1_l2_requests_per_cu_cycle": round(req / cu_cycles, 4),
            "l1_l2_in_flight_per_cu": round(req / cu_cycles * lat, 1),
            "l2_hits_per_packet": round(a["TCC_HIT_sum"] / n, 4),
            "l2_misses_per_packet": round(a["TCC_MISS_sum"] / n, 4),
            "vmem_latency_cycles": round(a["VmemLatency"], 1) if "VmemLatency" in a else None,
            "lds_latency_cycles": round(a["LdsLatency"], 1) if "LdsLatency" in a else None,
            "stall_fraction_of_cu_cycles": {k: round(a[c] / cu_cycles, 3) for k, c in (
                ("tcp_pending_data_from_l2", "TCP_PENDING_STALL_CYCLES_sum"),
                ("ta_address_stalled_by_tcp", "TA_ADDR_STALLED_BY_TC_CYCLES_sum"),
                ("td_stalled_by_tcp", "TD_TC_STALL_sum"),
                ("tcp_read_tag_conflict", "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum")) if c in a},
            "wave_state_fraction": {k: round(a[c] / wc, 3) for k, c in (
                ("waiting_on_counters", "SQ_WAIT_ANY"), ("issue_stalled", "SQ_WAIT_INST_ANY"),
                ("active", "SQ_ACTIVE_INST_ANY")) if c in a},
            "lds_bank_conflict_rate": (round(a["SQ_LDS_BANK_CONFLICT"] / a["SQ_LDS_IDX_ACTIVE"], 3)
                                       if a.get("SQ_LDS_IDX_ACTIVE") else None),
            "per_packet": {k: round(a[c] / n, 4) for k, c in (
                ("valu", "SQ_INSTS_VALU"), ("salu", "SQ_INSTS_SALU"), ("lds", "SQ_INSTS_LDS"),
                ("vmem_rd", "SQ_INSTS_VMEM_RD")) if c in a},
            "raw_per_launch": {k: round(v, 1) for k, v in sorted(a.items())},
        }
    json.dump(out, open(sys.argv[1], "w"), indent=1)
    for tag, s in out.items():
        print(tag, {k: s[k] for k in ("l1_l2_read_requests_per_packet", "l1_l2_read_latency_cycles",
                                      "l1_l2_in_flight_per_cu", "clock_GHz_from_grbm", "vmem_latency_cycles")},
              s["stall_fraction_of_cu_cycles"])


if __name__ == "__main__":
    main()
