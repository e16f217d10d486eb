#!/bin/bash
# A/B of the two-phase classify form against the fused kernel on the other gather-bound workloads, one box, one call,
# alternated twice: configs[2] (interned lists, the headline), configs[2] with uniform sources, configs[4] at 1M
# prefixes.  Usage (GPU box): tools/ab_split2.sh <tag>  -> gpurun_out/<tag>/ab_split2/
set -u
O=gpurun_out/${1:-ab}/ab_split2
mkdir -p $O
run() {  # name, env..., -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 3 "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -1 $O/$name.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms_avg"])' 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
}
for rep in ${REPS:-1 2}; do
  run cfg2_fused_r$rep INFW_SPLIT=0 --
  run cfg2_split_r$rep INFW_SPLIT=1 --
  run cfg2u_fused_r$rep INFW_SPLIT=0 -- --uniform
  run cfg2u_split_r$rep INFW_SPLIT=1 -- --uniform
  run cfg4m_fused_r$rep INFW_SPLIT=0 -- --cfg 4 --prefixes 1000000
  run cfg4m_split_r$rep INFW_SPLIT=1 -- --cfg 4 --prefixes 1000000
done
echo ab-split2-ok
