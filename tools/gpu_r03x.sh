#!/bin/bash
# Round-3 pass X: experiment — the LDS word cache holding /16 words in the kD16 kernels (build in abtree/):
# parity with it, then alternating bench runs against the tree's build on configs[1] and configs[4].
set -u
O=gpurun_out/r03x
mkdir -p $O
LIB=abtree/ingress-node-firewall_amd/lib/libinfw.so
INFW_LIB=$LIB timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "d16 or parity_configs or lds_cache or compact_layout" > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh $O/cfg1 $LIB d16cache tree 3 --cfg 1 --batch 67108864 --no-cpu-baseline --steps 30 || exit 1
bash tools/ab_libs.sh $O/cfg4 $LIB d16cache tree 3 --cfg 4 --no-cpu-baseline --steps 30 || exit 1
echo all-ok
