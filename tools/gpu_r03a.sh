#!/bin/bash
# Round-3 first GPU pass: GPU tests, smoke, headline bench (standalone and through the spawn launcher),
# commit latency at 1 and 4 device slots.  Stops at the first failing step.
set -u
O=gpurun_out/r03a
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py
step bench_spawn 400 python bench.py --gpus 1 --spawn --no-cpu-baseline
step commit_1slot 400 python tools/commit_latency.py --sizes 100,1000 --slots 1
step commit_4slot 400 python tools/commit_latency.py --sizes 100,1000 --slots 4
echo all-ok
