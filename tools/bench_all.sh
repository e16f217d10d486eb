#!/bin/bash
# Every bench.py workload line on the current build (on the GPU box).  Usage: tools/bench_all.sh <out_dir>
set -u
OUT=${1:-gpurun_out/bench_all}
mkdir -p $OUT
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run cfg2 --steps 30
run cfg2_compact --layout compact --no-cpu-baseline --steps 30
run cfg1 --cfg 1 --batch 67108864 --no-cpu-baseline --steps 30
run cfg4 --cfg 4 --no-cpu-baseline --steps 30
run cfg4_1m --cfg 4 --prefixes 1000000 --no-cpu-baseline --steps 30
run cfg2_uniform --uniform --no-cpu-baseline --steps 30
run cfg2_distinct --templates 1000000 --no-cpu-baseline --steps 20
run cfg2_distinct_popularity_order --templates 1000000 --key-order workload --no-cpu-baseline --steps 20
run cfg2_frames --from-frames 128 --no-cpu-baseline --steps 20
run cfg2_frames_fused --from-frames 128 --fused --no-cpu-baseline --steps 20
run cfg3_n1 --global-packets 1073741824 --no-cpu-baseline --steps 10 --warmup 2
for f in $OUT/*.log; do
  python3 -c "import json; l=[x for x in open('$f') if x.startswith('{')]; d=json.loads(l[-1]); r=d['roofline']; print('$(basename $f .log)', d['value'], r['kernel_ms_avg'], r['frac'], r.get('from_frames', {}).get('pack_kernel_ms_avg', ''))"
done
