#!/bin/bash
# configs[1] launch shapes: the default 768 x 2 (24 waves per CU, 4096-entry /16-word LDS cache) against 512 x 4 and
# 512 x 3 (32 / 24 waves, the generic instantiations: no /16-word cache), alternated twice.  Usage: tools/ab_cfg1_shape.sh <tag>
set -u
O=gpurun_out/${1:-ab}/ab_cfg1_shape
mkdir -p $O
run() {
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --cfg 1 --batch 67108864 --no-cpu-baseline --steps 30 --warmup 3 "$@" \
      > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -1 $O/$name.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms_avg"], d["roofline"]["kernel"])' 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
}
for rep in 1 2; do
  run default_r$rep INFW_NONE=1 --
  run b512x4_r$rep INFW_BLOCK=512 INFW_BLOCKS_PER_CU=4 --
  run b512x3_r$rep INFW_BLOCK=512 INFW_BLOCKS_PER_CU=3 --
done
echo ab-cfg1-shape-ok
