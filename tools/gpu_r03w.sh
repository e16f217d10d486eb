#!/bin/bash
# Round-3 pass W: incremental commits on the device with /16 words forced on (and the default).
set -u
mkdir -p gpurun_out/r03w
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "incremental_commits_on_device or d16" > gpurun_out/r03w/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r03w/pytest_gpu.log; exit $rc
