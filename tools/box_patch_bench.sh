#!/bin/bash
# Host cost of incremental commits on the GPU box's CPU (no GPU use): tools/patch_bench.cpp per phase.
set -u
mkdir -p gpurun_out/pb
for c in 4 2; do
  PB_TRACE=1 PB_MICRO=1 timeout -k 10 240 tools/micro/patch_bench $c 1000 20 \
    > gpurun_out/pb/cfg$c.log 2>&1 || exit 1
  grep -v '^\[patch\]' gpurun_out/pb/cfg$c.log; grep '^\[patch\]' gpurun_out/pb/cfg$c.log | tail -3
done
