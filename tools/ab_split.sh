#!/bin/bash
# A/B of the two-phase classify form on configs[2] with one rule list per key (bench --templates 1000000), on one
# box in one call: the fused kernel and the split form at 4 value parts (the 2-GiB entry-line budget) and at 16
# (budget 16 GiB), in the reference loader's random update order, plus the fused kernel in popularity order (the
# round-3 reference point), alternated twice.  Usage (GPU box): tools/ab_split.sh <tag>  -> gpurun_out/<tag>/ab_split/
set -u
O=gpurun_out/${1:-ab}/ab_split
mkdir -p $O
run() {  # name, env..., -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --templates 1000000 --no-cpu-baseline --steps 20 --warmup 3 "$@" \
      > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -1 $O/$name.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms_avg"], d["config"]["tables"]["dt_parts"])' 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
}
for rep in 1 2; do
  run fused_r$rep INFW_SPLIT=0 --
  run split4_r$rep INFW_SPLIT=1 --
  run split16_r$rep INFW_SPLIT=1 INFW_DT_BUDGET_MB=16384 --
  run fused_pop_r$rep INFW_SPLIT=0 -- --key-order workload
done
echo ab-split-ok
