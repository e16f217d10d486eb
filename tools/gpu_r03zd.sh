#!/bin/bash
# Round-3 pass ZD: experiment — LDS counters for rule ids < 128 only (higher ids straight to the device counters),
# the freed LDS back to a 512-entry IPv6 group cache (abtree/ build): parity, then alternating bench runs.
set -u
O=gpurun_out/r03zd
mkdir -p $O
LIB=abtree/ingress-node-firewall_amd/lib/libinfw.so
INFW_LIB=$LIB timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "counter_paths or survey_probes or parity_configs or lds_cache or frozen or golden" > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh $O/cfg2 $LIB c128_b512 tree 4 --no-cpu-baseline --steps 30 || exit 1
echo all-ok
