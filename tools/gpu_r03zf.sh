#!/bin/bash
# Round-3 pass ZF: the C++ host side end to end on the device (loader -> commit -> infw_classify_host ->
# UpdateMetrics), plus the suite's other control-plane GPU tests.
set -u
mkdir -p gpurun_out/r03zf
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "cpp_loader or ebpfsyncer or e2e or classify_host" > gpurun_out/r03zf/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r03zf/pytest_gpu.log; exit $rc
