#!/bin/bash
# Round-3 pass L: /16 words with the LDS word cache filled from their answers — parity, then INFW_D16=0 vs 1 in
# one process on configs[1], [4] and [2] at 100k / 300k prefixes (where the choice threshold sits).
set -u
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "d16 or classify_frames_on_device or parity_configs or compact_layout or lds_cache" > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
ab() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python -u tools/ab_tables.py --variants "INFW_D16=0;INFW_D16=1" "$@" > $O/ab_$name.txt 2>&1
  local rc=$?; echo "ab $name rc=$rc"; cat $O/ab_$name.txt | tail -2
  [ $rc -eq 0 ] || exit $rc
}
ab cfg1 --cfg 1
ab cfg4 --cfg 4
ab cfg2_100k --cfg 2 --prefixes 100000
ab cfg2_300k --cfg 2 --prefixes 300000
echo all-ok
