#!/bin/bash
# Memory-path latency and unit-busy counters of one bench workload (rocprofv3's derived VmemLatency / LdsLatency —
# in-flight VMEM / LDS instructions integrated over time ÷ instructions, in cycles — then four PMC passes, each within gfx950's per-block
# limits: 4 TCP + 1 GRBM; 2 TA + 2 TCC + 4 SQ; 8 SQ; 8 SQ + 2 TD).  Usage (GPU box): tools/profile_lat.sh <tag> [bench args...]
# -> gpurun_out/lat_<tag>/{lat_tcp,lat_ta}/
set -u
TAG=${1:?tag}; shift
ARGS=${*:-""}
OUT=gpurun_out/lat_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 420 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $ARGS --steps 5 \
      --warmup 1 --no-cpu-baseline --no-line-rates > $OUT/$name.stdout 2> $OUT/$name.stderr
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run lat_vmem --pmc VmemLatency
run lat_ldsl --pmc LdsLatency
run lat_l2 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
run lat_tcp --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE
run lat_ta --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_BUSY_avr TCC_TAG_STALL_sum SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES
run lat_sq --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS
run lat_wait --pmc SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TD_TD_BUSY_sum TD_TC_STALL_sum
echo done
