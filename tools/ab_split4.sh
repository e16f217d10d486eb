#!/bin/bash
# Decide-kernel workgroups per CU 1 vs 2 (the default) on configs[2] with one rule list per key, alternated twice.
# Usage (GPU box): tools/ab_split4.sh <tag>  -> gpurun_out/<tag>/ab_split4/
set -u
O=gpurun_out/${1:-ab}/ab_split4
mkdir -p $O
for rep in 1 2; do
  for bpc in 1 2; do
    INFW_DECIDE_BPC=$bpc timeout -k 10 300 python -u bench.py --templates 1000000 --no-cpu-baseline --steps 20 \
        --warmup 3 > $O/bpc${bpc}_r$rep.log 2>&1 || exit $?
    echo "bpc$bpc r$rep $(tail -1 $O/bpc${bpc}_r$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms_avg"])')"
  done
done
echo ab-split4-ok
