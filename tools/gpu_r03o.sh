#!/bin/bash
# Round-3 pass O: the remaining bench lines profiled at the /16-word build — uniform sources, the distinct-lists
# variant in both table update orders (shuffled is bench.py's default), and the fused frames kernel.
set -u
bash tools/profile.sh r03o_cfg2u --uniform --steps 5 --warmup 1 --no-cpu-baseline || exit 1
bash tools/profile.sh r03o_cfg2d_wl --templates 1000000 --key-order workload --steps 5 --warmup 1 --no-cpu-baseline || exit 1
bash tools/profile.sh r03o_cfg2d --templates 1000000 --steps 5 --warmup 1 --no-cpu-baseline || exit 1
bash tools/profile.sh r03o_fused --from-frames 128 --fused --steps 5 --warmup 1 --no-cpu-baseline || exit 1
echo all-ok
