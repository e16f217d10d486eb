#!/bin/bash
# Round-3 pass C: line-read microbenchmark + PMC, LDS attribution, profiles of configs[4] at 1M prefixes and of
# uniform-source configs[2] at this build.
set -u
bash tools/micro/line_pmc.sh r03 || exit 1
bash tools/lds_ablate.sh r03 || exit 1
bash tools/profile.sh r03_cfg4m --cfg 4 --prefixes 1000000 --steps 5 --warmup 1 --no-cpu-baseline || exit 1
bash tools/profile.sh r03_cfg2u --uniform --steps 5 --warmup 1 --no-cpu-baseline || exit 1
echo all-ok
