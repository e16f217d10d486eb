#!/bin/bash
# configs[2] under each per-context table option (results identical; the counters' digest is printed), alternated
# twice on one box.  Usage (GPU box): tools/opt_sweep.sh [out_dir]   (default gpurun_out/opts)
set -u
O=${1:-gpurun_out/opts}; mkdir -p $O
for r in 1 2; do
  for o in "" "--opt dt_parts=8" "--opt dt_parts=4" "--opt dt_half=1" "--opt dt_half=0" "--opt d16=1" "--opt dt_adapt=0"; do
    tag=$(echo "base $o" | tr ' =' '__')
    timeout -k 10 200 python bench.py $o --no-cpu-baseline --no-line-rates --steps 20 --warmup 3 > $O/${tag}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/${tag}_$r.log') if l.startswith('{')][-1]); print('$tag', $r, d['value'], d['roofline']['kernel'], d['roofline']['kernel_ms_avg'], d['config']['stats_digest'][:12])"
  done
done
