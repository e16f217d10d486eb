#!/bin/bash
# Round-3 pass H: the headline and configs[4]@1M profiles at the flat-index build (tables.cpp is part of the build
# id), then commit latency at configs[2] with one and four device slots.
set -u
mkdir -p gpurun_out/r03h
bash tools/profile.sh r03h_cfg2 || exit 1
bash tools/profile.sh r03h_cfg4m --cfg 4 --prefixes 1000000 --steps 5 --warmup 1 --no-cpu-baseline || exit 1
timeout -k 10 300 python tools/commit_latency.py > gpurun_out/r03h/commit_latency.jsonl 2>&1 || exit 1
timeout -k 10 300 python tools/commit_latency.py --slots 4 --sizes 1,100,1000 > gpurun_out/r03h/commit_latency_4slots.jsonl 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r03h/bench.log 2>&1 || exit 1
tail -1 gpurun_out/r03h/bench.log
echo all-ok
