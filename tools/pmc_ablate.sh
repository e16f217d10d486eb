#!/bin/bash
# L2 / memory-side counters per classify ablation variant (INFW_ABLATE codes):
# one rocprofv3 --pmc pass per counter group over tools/tune.py, then
# tools/pmc_ablate.py groups the dispatches by kernel instantiation.
# Usage (on the GPU box): tools/pmc_ablate.sh <tag> [ablate codes, default 0,2,1,8]
set -u
TAG=${1:-abl}; CODES=${2:-0,2,1,8}
OUT=gpurun_out/pmcab_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 tools/tune.py \
      --ablate $CODES --rounds 1 --iters 1 > $OUT/$name.stdout 2> $OUT/$name.stderr
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run l2 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum
run ea --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
run tcp --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
echo done
