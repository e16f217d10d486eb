#!/bin/bash
# Round-3 pass Q: launch shapes (waves per CU) on configs[2]'s one-list-per-key variant with the table loaded in
# random order — is its 1.77x slowdown against popularity order (same misses) latency that more waves would hide?
set -u
mkdir -p gpurun_out/r03q
timeout -k 10 500 python -u tools/tune.py --templates 1000000 --key-order shuffled --variants "768:0:2,512:0:3,512:0:4" \
  > gpurun_out/r03q/tune_distinct_shuffled.txt 2>&1
rc=$?; tail -4 gpurun_out/r03q/tune_distinct_shuffled.txt; exit $rc
