#!/bin/bash
# Host-fed bench lines alternated R times on one box: on a shared host their spread is the other tenants' CPU use
# (each line reports its step spread and the host's load average).
# Usage (GPU box): tools/hostfed_lines.sh <out_dir> [R] [feed ...]
#   feed = <xdp-ring>:<umem order>[:<burst size>], default: host-packed:ring host-packed:packet
#   (e.g. host-bursts:ring for DPDK-style bursts, one per interface; host-bursts:ring:32 for rx_burst-sized ones)
set -u
OUT=${1:?out}; R=${2:-2}; shift; [ $# -gt 0 ] && shift
FEEDS=${*:-host-packed:ring host-packed:packet}
mkdir -p $OUT
for r in $(seq 1 $R); do
  for f in $FEEDS; do
    IFS=: read -r ring order bs <<< "$f"
    tag=${ring}_${order}${bs:+_b$bs}_$r
    timeout -k 10 300 python bench.py --xdp-ring $ring --umem-order $order ${bs:+--burst-size $bs} --no-cpu-baseline \
        --steps 20 --warmup 3 > $OUT/$tag.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$OUT/$tag.log') if l.startswith('{')][-1]); h=d['roofline']['xdp_ring']['host_feed']; print('$tag', d['value'], h['step_ms_min'], h['step_ms_median'], h['step_ms_max'], h['host_loadavg_1m'])"
  done
done
