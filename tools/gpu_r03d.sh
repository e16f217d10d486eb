#!/bin/bash
# Round-3 pass D: packed LDS counters — GPU tests, then same-box A/B against the previous build (abtree/).
set -u
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests failed; exit 1; }
echo tests ok
bash tools/ab_libs.sh $O/ab_cfg2 abtree/libinfw_prev.so prev packed 3 --no-cpu-baseline --steps 30 > $O/ab_cfg2.txt || exit 1
echo ab cfg2 ok
bash tools/ab_libs.sh $O/ab_cfg4 abtree/libinfw_prev.so prev packed 3 --cfg 4 --no-cpu-baseline --steps 30 > $O/ab_cfg4.txt || exit 1
echo ab cfg4 ok
