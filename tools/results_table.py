#!/usr/bin/env python3
"""The results table of DESIGN.md §7.2 from one measurement pass: every bench line of profiles/<pass>/lines/*.log and,
where the pass profiled that workload, profiles/<pass>_<key>/summary.json (rocprofv3 kernel trace + PMC at the same
build).  Columns: packet rate; kernel time by HIP events (the line) and by the kernel trace (average over the traced
run's launches); roofline.frac (algorithmic bytes / HIP-event time / 8 TB/s); HBM bytes per packet from the PMC
(guide-corrected) against the algorithmic bytes; L2 hits / misses per packet; fabric line traffic = fabric read
requests (TCC_EA0_RDREQ) x 128 B per second against the stream bandwidth the same line measured in its own process,
and its inverse (the most the kernel could gain at today's lines per packet if every random line moved at the
streaming rate).  Lines whose build id differs from the profile's are refused.
Usage: tools/results_table.py <pass> [<override pass>]  (e.g. r06z r06K: lines present in profiles/<override>/lines,
and profiles <override>_<key>, replace the pass's own — re-measured after a host-side change at the same kernel build)
  -> markdown on stdout, JSON in profiles/<override or pass>/results.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = {  # bench_all.sh line -> gpu_pass.sh profile key
    "cfg2": "cfg2", "cfg2_compact": "cfg2c", "cfg1": "cfg1", "cfg1_compact": "cfg1c", "cfg4": "cfg4",
    "cfg4_1m": "cfg4m", "cfg2_uniform": "cfg2u", "cfg2_distinct": "cfg2d", "cfg2_frames_fused": "fused",
    "cfg2_frames": "frames", "cfg2_xdp_hbm": "xdphbm", "cfg3_n1": "cfg3",
}
ORDER = ["cfg2", "cfg2_compact", "cfg1", "cfg1_compact", "cfg4", "cfg4_1m", "cfg2_uniform", "cfg2_distinct",
         "cfg2_distinct_popularity_order", "cfg3_n1", "inproc_n1", "inproc_n8", "cfg2_frames", "cfg2_frames_fused",
         "cfg2_xdp_hbm", "cfg2_xdp_host", "cfg2_xdp_registered", "cfg2_xdp_host_packed",
         "cfg2_xdp_host_packed_interleaved", "cfg2_host_bursts", "cfg2_host_bursts32"]
LABEL = {
    "cfg2": "configs[2] (headline)", "cfg2_compact": "configs[2], family-compact", "cfg1": "configs[1]",
    "cfg1_compact": "configs[1], family-compact", "cfg4": "configs[4]", "cfg4_1m": "configs[4] at 1M prefixes",
    "cfg2_uniform": "configs[2], uniform sources", "cfg2_distinct": "configs[2], 1M distinct lists (two-phase)",
    "cfg2_distinct_popularity_order": "the same, keys in popularity order", "cfg3_n1": "configs[3]: 1B-packet job",
    "inproc_n1": "configs[3], in-process, 1 slot", "inproc_n8": "configs[3], in-process, 8 slots on one GPU",
    "cfg2_frames": "packer + classify from frames in HBM (two kernels)",
    "cfg2_frames_fused": "classified straight from frames in HBM", "cfg2_xdp_hbm": "AF_XDP rings, umem in HBM",
    "cfg2_xdp_host": "AF_XDP rings, umem in pinned host memory (device read)",
    "cfg2_xdp_registered": "AF_XDP rings, daemon's registered umem (device read)",
    "cfg2_xdp_host_packed": "AF_XDP rings, pageable umem, host-fed (ring order)",
    "cfg2_xdp_host_packed_interleaved": "the same, rings interleaved in one umem",
    "cfg2_host_bursts": "DPDK-style bursts, host-fed (one burst per port)",
    "cfg2_host_bursts32": "DPDK-style bursts of 32 frames, host-fed",
}


def last_json(path):
    return json.loads([l for l in open(path) if l.startswith("{")][-1])


def main():
    tag = sys.argv[1]
    over = sys.argv[2] if len(sys.argv) > 2 else None
    rows, out = [], {}
    for name in ORDER:
        p = os.path.join(ROOT, "profiles", tag, "lines", f"{name}.log")
        if over and os.path.exists(os.path.join(ROOT, "profiles", over, "lines", f"{name}.log")):
            p = os.path.join(ROOT, "profiles", over, "lines", f"{name}.log")
        if not os.path.exists(p):
            continue
        d = last_json(p)
        r = d.get("roofline", {})
        per_slot = d.get("per_slot")
        n = d["config"].get("packets_per_gpu_per_step") or sum(s["packets_per_step"] for s in per_slot)
        # in-process lines: N slots sharing the device, each slot's kernel time overlapping the others' (their
        # wall time per step stands for the launch)
        k_ms = r.get("kernel_ms_avg") or (d["ms_per_step"] if per_slot else None)
        row = {"line": name, "source": os.path.relpath(p, ROOT), "build_id": d.get("build_id"), "Gpps": d["value"] / 1e3,
               "kernel": r.get("kernel") or d.get("kernel"),
               "packets_per_launch": n, "kernel_ms_hip": k_ms, "frac": r.get("frac"), "bound": r.get("bound"),
               "algo_B": r.get("algorithmic_bytes_per_packet")}
        key = PROF.get(name)
        sp = None
        for t in ([over] if over else []) + [tag]:  # the override pass's profile of the workload first
            q = os.path.join(ROOT, "profiles", f"{t}_{key}", "summary.json") if key else None
            if q and os.path.exists(q):
                sp, ptag = q, t
                break
        if sp and os.path.exists(sp):
            s = json.load(open(sp))
            bl = s.get("bench_line_under_kernel_trace", {})
            assert bl.get("build_id") in (None, d.get("build_id")), (name, bl.get("build_id"), d.get("build_id"))
            stream = (r.get("line_rates") or {}).get("stream_GB_per_s")
            rings = (r.get("xdp_ring") or {}).get("rings") or 1  # AF_XDP: one launch per ring, the line's time per step
            row.update(rocprof_ms=s["avg_ns_per_classification"] * rings / 1e6, hbm_B=s["hbm_bytes_per_packet"],
                       hits=s["l2_hits_per_packet"], misses=s["l2_misses_per_packet"],
                       fabric_req=s["ea_rdreq_per_packet"], profile=f"profiles/{ptag}_{key}")
            if stream and k_ms:  # per step: the step's packets over the step's kernel time (AF_XDP: one launch per ring)
                tb = s["ea_rdreq_per_packet"] * 128 * n / (k_ms * 1e-3) / 1e9
                row.update(line_TBps=tb / 1e3, line_frac=tb / stream, headroom=stream / tb)
        rows.append(row)
        out[name] = row
    json.dump(out, open(os.path.join(ROOT, "profiles", over or tag, "results.json"), "w"), indent=1)

    def f(v, fmt):
        return format(v, fmt) if isinstance(v, (int, float)) else "—"
    print("| workload | kernel (registry name) | Gpps | kernel ms (HIP events) | kernel ms (rocprof) "
          "| frac | HBM B/pkt (PMC) vs algorithmic | L2 hits / misses per packet | line traffic (of stream) | headroom |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        gpps = f(r["Gpps"], ".3f") if r["Gpps"] < 2 else f(r["Gpps"], ".1f")
        hb = f"{r['hbm_B']:.1f} vs {r['algo_B']:.1f} ({r['hbm_B'] / r['algo_B']:.2f}×)" if "hbm_B" in r else "—"
        hm = f"{r['hits']:.2f} / {r['misses']:.2f}" if "hits" in r else "—"
        lt = f"{r['line_TBps']:.1f} TB/s ({r['line_frac']:.2f})" if "line_TBps" in r else "—"
        frac = f(r["frac"], ".3f") + (" (PCIe)" if r.get("bound") == "pcie" else "")
        print(f"| {LABEL[r['line']]} | `{r['kernel']}` | {gpps} | {f(r['kernel_ms_hip'], '.3f')} "
              f"| {f(r.get('rocprof_ms'), '.3f')} | {frac} | {hb} | {hm} | {lt} | {f(r.get('headroom'), '.2f')} |")


if __name__ == "__main__":
    main()
