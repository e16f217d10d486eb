#!/bin/bash
# Round-3 pass T (final build): kernel trace + PMC of the headline, configs[1], configs[4], configs[4]@1M.
set -u
bash tools/profile.sh r03z3_cfg2 || exit 1
bash tools/profile.sh r03z3_cfg1 --cfg 1 --steps 5 --warmup 1 --no-cpu-baseline || exit 1
bash tools/profile.sh r03z3_cfg4 --cfg 4 --steps 5 --warmup 1 --no-cpu-baseline || exit 1
bash tools/profile.sh r03z3_cfg4m --cfg 4 --prefixes 1000000 --steps 5 --warmup 1 --no-cpu-baseline || exit 1
echo all-ok
