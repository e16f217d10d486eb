#!/bin/bash
# The two-phase form's knobs on configs[2] with one rule list per key (random update order), one box, alternated
# twice: decide-kernel workgroups per CU (INFW_DECIDE_BPC 2 / 3 / 4) and 8 value parts (entry-line budget 4 GiB)
# against the default 4.  Usage (GPU box): tools/ab_split3.sh <tag>  -> gpurun_out/<tag>/ab_split3/
set -u
O=gpurun_out/${1:-ab}/ab_split3
mkdir -p $O
run() {
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
  run split4_bpc4_r$rep INFW_SPLIT=1 --
  run split4_bpc2_r$rep INFW_SPLIT=1 INFW_DECIDE_BPC=2 --
  run split4_bpc3_r$rep INFW_SPLIT=1 INFW_DECIDE_BPC=3 --
  run split8_r$rep INFW_SPLIT=1 INFW_DT_BUDGET_MB=4096 --
done
echo ab-split3-ok
