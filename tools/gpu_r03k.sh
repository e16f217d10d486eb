#!/bin/bash
# Round-3 pass K: configs[1] with /16 words profiled (kernel trace + PMC incl. the SQ counters); the automatic
# threshold checked at configs[2] with 100k and 300k prefixes (INFW_D16=0 vs 1 in one process).
set -u
O=gpurun_out/r03k
mkdir -p $O
PROFILE_DEEP=1 bash tools/profile.sh r03k_cfg1 --cfg 1 --steps 5 --warmup 1 --no-cpu-baseline || exit 1
ab() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python -u tools/ab_tables.py --variants "INFW_D16=0;INFW_D16=1" "$@" > $O/ab_$name.txt 2>&1
  local rc=$?; echo "ab $name rc=$rc"; cat $O/ab_$name.txt | tail -3
  [ $rc -eq 0 ] || exit $rc
}
ab cfg2_100k --cfg 2 --prefixes 100000
ab cfg2_300k --cfg 2 --prefixes 300000
echo all-ok
