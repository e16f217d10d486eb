#!/bin/bash
# The two host-fed bench lines (bench.py --xdp-ring host-packed, ring and interleaved umem order), alternated R times on
# one box: on a shared host their spread is the other tenants' CPU use (each line reports its step spread and the host's
# load average).  Usage (GPU box): tools/hostfed_lines.sh <out_dir> [R]
set -u
OUT=${1:?out}; R=${2:-2}
mkdir -p $OUT
for r in $(seq 1 $R); do
  for o in ring packet; do
    timeout -k 10 300 python bench.py --xdp-ring host-packed --umem-order $o --no-cpu-baseline --steps 20 --warmup 3 \
        > $OUT/host_packed_${o}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$OUT/host_packed_${o}_$r.log') if l.startswith('{')][-1]); h=d['roofline']['xdp_ring']['host_feed'] if 'xdp_ring' in d['roofline'] else d['config']['xdp_ring']['host_feed']; print('$o', $r, d['value'], h['step_ms_min'], h['step_ms_median'], h['step_ms_max'], h['host_loadavg_1m'])"
  done
done
