#!/bin/bash
# Round-3 pass E: every workload line, then the headline and configs[4]@1M profiles, at the final kernel build.
set -u
bash tools/bench_all.sh gpurun_out/r03e_all || exit 1
bash tools/profile.sh r03e_cfg2 || exit 1
bash tools/profile.sh r03e_cfg4m --cfg 4 --prefixes 1000000 --steps 5 --warmup 1 --no-cpu-baseline || exit 1
echo all-ok
