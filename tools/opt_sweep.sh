#!/bin/bash
# configs[2] under per-context options (results identical; tools-only sweep), alternated twice
set -u
O=gpurun_out/r06K_opts; mkdir -p $O
for r in 1 2; do
  for o in "" "--opt dt_parts=8" "--opt dt_parts=4" "--opt dt_half=1" "--opt dt_half=0" "--opt d16=1" "--opt dt_adapt=0"; do
    tag=$(echo "base $o" | tr ' =' '__')
    timeout -k 10 200 python bench.py $o --no-cpu-baseline --no-line-rates --steps 20 --warmup 3 > $O/${tag}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/${tag}_$r.log') if l.startswith('{')][-1]); print('$tag', $r, d['value'], d['roofline']['kernel'], d['roofline']['kernel_ms_avg'], d['config']['stats_digest'][:12])"
  done
done
