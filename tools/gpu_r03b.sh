#!/bin/bash
# Round-3 pass B: the new GPU tests, configs[4] at 1M prefixes (bench line + CPU baseline), swap stream,
# and the headline profile at this build.  Stops at the first failing step.
set -u
O=gpurun_out/r03b
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step gpu_new 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "e2e or past_part or four_slot or headline_scale"
step bench_cfg4m 500 python bench.py --cfg 4 --prefixes 1000000
step swap_stream 300 python tools/swap_stream.py --edits 1,100,1000
bash tools/profile.sh r03_cfg2 || exit 1
echo all-ok
