#!/bin/bash
# rocprofv3 evidence for one round: kernel trace + stats, then one PMC pass per
# counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
# Usage (on the GPU box): tools/profile.sh <tag> [bench args...]
# Stops at the first run that crashes / times out (rc >= 124).
set -u
TAG=${1:-r01}; shift || true
ARGS=${*:-"--steps 5 --warmup 1 --no-cpu-baseline"}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 420 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $ARGS \
      > $OUT/$name.stdout 2> $OUT/$name.stderr
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run kt --kernel-trace --stats
run pmc_fetch --pmc FETCH_SIZE
run pmc_write --pmc WRITE_SIZE
run pmc_lds --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES
run pmc_l2 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
run pmc_dram --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum
if [ "${PROFILE_DEEP:-0}" = "1" ]; then
  run pmc_sq --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM
  run pmc_tcc --pmc TCC_BUSY_avr TCC_TAG_STALL_sum
fi
echo done
