#!/bin/bash
# Round-3 pass ZB: the LDS /16-word cache under contention (new GPU test) and the other /16-word tests.
set -u
mkdir -p gpurun_out/r03zb
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "lds_d16_cache or lds_cache or d16" > gpurun_out/r03zb/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r03zb/pytest_gpu.log; exit $rc
