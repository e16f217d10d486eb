#!/bin/bash
# Round-3 pass J: /16 words in front of DIR-24-8 — GPU parity, then same-process A/Bs (INFW_D16=0 vs 1) on
# configs[1], [4] (100k and 1M prefixes) and [2] (1M: the compiler would not choose them).
set -u
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "d16 or classify_frames_on_device or parity_configs or compact_layout or incremental or commits_while or many_ifindexes or lds_cache or clustered" \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
ab() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python -u tools/ab_tables.py --variants "INFW_D16=0;INFW_D16=1" "$@" > $O/ab_$name.txt 2>&1
  local rc=$?; echo "ab $name rc=$rc"; cat $O/ab_$name.txt | tail -3
  [ $rc -eq 0 ] || exit $rc
}
ab cfg1 --cfg 1 --batch 67108864
ab cfg4 --cfg 4
ab cfg2 --cfg 2
ab cfg4m --cfg 4 --prefixes 1000000
echo all-ok
