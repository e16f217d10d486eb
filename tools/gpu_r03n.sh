#!/bin/bash
# Round-3 pass N: kernel trace + PMC of the headline, configs[1], configs[4] and configs[4]@1M at the /16-word
# build (the traffic files bench.py attaches carry its build id).
set -u
bash tools/profile.sh r03n_cfg2 || exit 1
bash tools/profile.sh r03n_cfg1 --cfg 1 --steps 5 --warmup 1 --no-cpu-baseline || exit 1
bash tools/profile.sh r03n_cfg4 --cfg 4 --steps 5 --warmup 1 --no-cpu-baseline || exit 1
bash tools/profile.sh r03n_cfg4m --cfg 4 --prefixes 1000000 --steps 5 --warmup 1 --no-cpu-baseline || exit 1
mkdir -p gpurun_out/r03n
# table update order: shuffled (the default, like the reference's Go map range) and the generator's popularity
# order, for the one workload where it places the hot rule lists (one list per key)
for ko in shuffled workload; do
  timeout -k 10 300 python bench.py --templates 1000000 --no-cpu-baseline --steps 20 --key-order $ko \
    > gpurun_out/r03n/cfg2_distinct_$ko.log 2>&1 || exit 1
  tail -1 gpurun_out/r03n/cfg2_distinct_$ko.log | cut -c1-120
done
echo all-ok
