#!/bin/bash
# Round-3 pass C: LDS attribution, profiles of configs[4] at 1M prefixes and of uniform-source configs[2],
# swap stream with batch deletes.
set -u
mkdir -p gpurun_out/r03c
timeout -k 10 300 python tools/swap_stream.py --edits 100,1000 > gpurun_out/r03c/swap_stream.log 2>&1 || exit 1
echo swap rc=0
bash tools/lds_ablate.sh r03 || exit 1
bash tools/profile.sh r03_cfg4m --cfg 4 --prefixes 1000000 --steps 5 --warmup 1 --no-cpu-baseline || exit 1
bash tools/profile.sh r03_cfg2u --uniform --steps 5 --warmup 1 --no-cpu-baseline || exit 1
echo all-ok
