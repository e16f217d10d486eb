#!/bin/bash
# Round-3 pass G: host patch cost and the live-swap stream at configs[4] on the flat-index pending map, then the
# GPU incremental-commit tests.
set -u
mkdir -p gpurun_out/r03g
bash tools/box_patch_bench.sh > gpurun_out/r03g/patch_bench.log 2>&1 || exit 1
cat gpurun_out/r03g/patch_bench.log | grep -v '^\[patch\] checks'
INFW_COMMIT_TRACE=1 timeout -k 10 300 python tools/swap_stream.py > gpurun_out/r03g/swap_stream.log 2> gpurun_out/r03g/commit_trace.log
rc=$?; echo "swap rc=$rc"; cat gpurun_out/r03g/swap_stream.log; tail -2 gpurun_out/r03g/commit_trace.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "incremental or swap or commit or image or dist" > gpurun_out/r03g/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r03g/pytest.log
exit $rc
