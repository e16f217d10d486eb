#!/bin/bash
# Round-3 pass ZA (final build): kernel trace + PMC of uniform sources, the distinct-lists variant (random update
# order, bench.py's default) and the fused frames kernel.
set -u
bash tools/profile.sh r03za3_cfg2u --uniform --steps 5 --warmup 1 --no-cpu-baseline || exit 1
bash tools/profile.sh r03za3_cfg2d --templates 1000000 --steps 5 --warmup 1 --no-cpu-baseline || exit 1
bash tools/profile.sh r03za3_fused --from-frames 128 --fused --steps 5 --warmup 1 --no-cpu-baseline || exit 1
echo all-ok
