#!/bin/bash
# Same-box alternating A/Bs of bench lines (one call, REPS rounds of every arm).  Arms differ only in bench.py
# arguments — table forms through --opt NAME=VALUE (include/infw.h infw_set_option; the library reads no
# environment), launch inputs through bench flags.
# Usage (GPU box): tools/ab.sh <tag> <experiment>  -> gpurun_out/<tag>/ab_<experiment>/<arm>_r<rep>.log; prints
# "<arm>_r<rep> rc=<rc> <Mpps> <kernel ms> <extra>" per run and stops at the first failing run.
#   keyorder   configs[2]: the reference loader's random update order (default) vs the generator's popularity order
#              (--key-order workload: hot rule lists get adjacent ids, so their decision lines sit together)
#   split      configs[2] with one rule list per key: fused vs the two-phase form (option split)
#   fstride    classification straight from frames (--fused) at frame strides 80 (header snapshots back to back: the
#              window of every other frame straddles two 64-B sectors) / 128 / 256 / 512 B
set -u
TAG=${1:?tag}; EXP=${2:?experiment}
O=gpurun_out/$TAG/ab_$EXP
mkdir -p $O
BASE=()     # bench arguments every arm of the experiment shares
EXTRA=''    # python expression on the bench line d printed after the timings
run() {  # arm, bench args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps ${STEPS:-20} --warmup 3 "${BASE[@]}" "$@" \
      > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -1 $O/$name.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms_avg'], ${EXTRA:-''})" 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
}
arms() {  # one round of the experiment's arms
  case $EXP in
    keyorder)
      run shuffled_$1
      run workload_$1 --key-order workload ;;
    split)
      run fused_$1 --opt split=0
      run split_$1 --opt split=1 ;;
    fstride)
      run s80_$1 --from-frames 80 --fused
      run s128_$1 --from-frames 128 --fused
      run s256_$1 --from-frames 256 --fused
      run s512_$1 --from-frames 512 --fused ;;
    *) echo "unknown experiment $EXP" >&2; exit 2 ;;
  esac
}
case $EXP in
  split) BASE=(--templates 1000000); EXTRA="d['config']['tables']['dt_parts']" ;;
esac
for rep in ${REPS:-1 2}; do arms r$rep; done
echo ab-$EXP-ok
