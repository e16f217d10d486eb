#!/bin/bash
# Round-3 pass R: value parts per (list, class) on the one-list-per-key variant loaded in random order — fewer
# parts shrink the 7.2 GB of entry lines (fewer pages for the hot lists) at the price of leaf lines.
set -u
mkdir -p gpurun_out/r03r
timeout -k 10 900 python -u tools/ab_tables.py --templates 1000000 --key-order shuffled --rounds 3 --iters 3 \
  --variants "INFW_DT_PARTS=16;INFW_DT_PARTS=4;INFW_DT_PARTS=1" > gpurun_out/r03r/ab_parts_distinct_shuffled.txt 2>&1
rc=$?; tail -5 gpurun_out/r03r/ab_parts_distinct_shuffled.txt; exit $rc
