#!/bin/bash
# The /16-word LDS cache halved (INFW_D16_CACHE=small) against the default on the workloads with /16
# words — configs[1] and configs[4] — alternated twice on one box.  Usage: tools/ab_d16cache.sh <tag>
set -u
O=gpurun_out/${1:-ab}/ab_d16cache
mkdir -p $O
run() {
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --warmup 3 "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -1 $O/$name.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms_avg"])' 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
}
for rep in 1 2; do
  run cfg1_default_r$rep INFW_D16_CACHE=small -- --cfg 1 --batch 67108864
  run cfg1_big_r$rep INFW_D16_CACHE=big -- --cfg 1 --batch 67108864
  run cfg4_default_r$rep INFW_D16_CACHE=small -- --cfg 4
  run cfg4_big_r$rep INFW_D16_CACHE=big -- --cfg 4
done
echo ab-d16cache-ok
