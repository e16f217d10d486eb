#!/bin/bash
# Same-box alternating A/Bs of bench lines (one call, REPS rounds of every arm; round 4's experiments as data).
# Usage (GPU box): tools/ab.sh <tag> <experiment>  -> gpurun_out/<tag>/ab_<experiment>/<arm>_r<rep>.log; prints
# "<arm>_r<rep> rc=<rc> <Mpps> <kernel ms> <extra>" per run and stops at the first failing run.
#   split      configs[2] with one rule list per key: fused vs the two-phase form at 4 and 16 value parts (random
#              update order), plus fused in popularity order
#   split2     two-phase vs fused on the other gather-bound lines: configs[2], uniform sources, configs[4] at 1M
#   split3     two-phase knobs: decide workgroups per CU 2 / 3 / 4 (INFW_DECIDE_BPC), 8 value parts
#   split4     decide workgroups per CU 1 vs 2
#   d16cache   the /16-word LDS cache halved (INFW_D16_CACHE=small) vs the default, configs[1] and [4]
#   cfg1_shape configs[1] launch shapes: 768 x 2 (default) vs 512 x 4 and 512 x 3
set -u
TAG=${1:?tag}; EXP=${2:?experiment}
O=gpurun_out/$TAG/ab_$EXP
mkdir -p $O
BASE=()     # bench arguments every arm of the experiment shares
EXTRA=''    # python expression on the bench line d printed after the timings
run() {  # arm, env..., -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps ${STEPS:-20} --warmup 3 "${BASE[@]}" \
      "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -1 $O/$name.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms_avg'], ${EXTRA:-''})" 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
}
arms() {  # one round of the experiment's arms
  case $EXP in
    split)
      run fused_$1 INFW_SPLIT=0 --
      run split4_$1 INFW_SPLIT=1 --
      run split16_$1 INFW_SPLIT=1 INFW_DT_BUDGET_MB=16384 --
      run fused_pop_$1 INFW_SPLIT=0 -- --key-order workload ;;
    split2)
      run cfg2_fused_$1 INFW_SPLIT=0 --
      run cfg2_split_$1 INFW_SPLIT=1 --
      run cfg2u_fused_$1 INFW_SPLIT=0 -- --uniform
      run cfg2u_split_$1 INFW_SPLIT=1 -- --uniform
      run cfg4m_fused_$1 INFW_SPLIT=0 -- --cfg 4 --prefixes 1000000
      run cfg4m_split_$1 INFW_SPLIT=1 -- --cfg 4 --prefixes 1000000 ;;
    split3)
      run split4_bpc4_$1 INFW_SPLIT=1 INFW_DECIDE_BPC=4 --
      run split4_bpc2_$1 INFW_SPLIT=1 INFW_DECIDE_BPC=2 --
      run split4_bpc3_$1 INFW_SPLIT=1 INFW_DECIDE_BPC=3 --
      run split8_$1 INFW_SPLIT=1 INFW_DT_BUDGET_MB=4096 -- ;;
    split4)
      run bpc1_$1 INFW_DECIDE_BPC=1 --
      run bpc2_$1 INFW_DECIDE_BPC=2 -- ;;
    d16cache)
      run cfg1_small_$1 INFW_D16_CACHE=small -- --cfg 1 --batch 67108864
      run cfg1_big_$1 INFW_D16_CACHE=big -- --cfg 1 --batch 67108864
      run cfg4_small_$1 INFW_D16_CACHE=small -- --cfg 4
      run cfg4_big_$1 INFW_D16_CACHE=big -- --cfg 4 ;;
    cfg1_shape)
      run default_$1 INFW_NONE=1 --
      run b512x4_$1 INFW_BLOCK=512 INFW_BLOCKS_PER_CU=4 --
      run b512x3_$1 INFW_BLOCK=512 INFW_BLOCKS_PER_CU=3 -- ;;
    *) echo "unknown experiment $EXP" >&2; exit 2 ;;
  esac
}
case $EXP in
  split|split3|split4) BASE=(--templates 1000000); EXTRA="d['config']['tables']['dt_parts']" ;;
  cfg1_shape) BASE=(--cfg 1 --batch 67108864); STEPS=${STEPS:-30}; EXTRA="d['roofline']['kernel']" ;;
esac
for rep in ${REPS:-1 2}; do arms r$rep; done
echo ab-$EXP-ok
