#!/bin/bash
# Round-3 pass ZH (tree at the end of the round): the whole GPU suite, smoke() and the default bench line, as the
# round-end driver runs them.
set -u
O=gpurun_out/r03zh
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench_default.log
[ $rc -eq 0 ] || exit $rc
echo all-ok
