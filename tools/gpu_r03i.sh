#!/bin/bash
# Round-3 pass I (re-entry after the container was re-created): the whole GPU suite, smoke() and the headline
# bench line at HEAD, plus the configs[4]@1M profile whose summary was lost with the old container.
set -u
mkdir -p gpurun_out/r03i
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r03i/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03i/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/r03i/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r03i/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r03i/bench.log 2>&1 || exit 1
tail -1 gpurun_out/r03i/bench.log
bash tools/profile.sh r03i_cfg4m --cfg 4 --prefixes 1000000 --steps 5 --warmup 1 --no-cpu-baseline || exit 1
echo all-ok
