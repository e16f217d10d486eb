#!/bin/bash
# LDS bank-conflict attribution of the default classify kernel (configs[2]): the same bench command with
# INFW_LDS_ABLATE = 0 (default), 1 (no DIR-24-8 word cache), 2 (no IPv6 group cache), 4 (no LDS counters),
# 7 (none of the three); per variant a kernel trace and one PMC pass of the LDS counters.
# Usage (GPU box): tools/lds_ablate.sh <tag> [bench args...]; summarise here with tools/summarize_lds.py <tag>.
set -u
TAG=${1:-lds}; shift || true
ARGS=${*:-"--steps 5 --warmup 1 --no-cpu-baseline"}
OUT=gpurun_out/lds_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in 0 1 2 4 7; do
  mkdir -p $OUT/v$v
  for pass in kt lds; do
    if [ $pass = kt ]; then P="--kernel-trace --stats"; else P="--pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES"; fi
    INFW_LDS_ABLATE=$v timeout -k 10 300 rocprofv3 $P -d $OUT/v$v/$pass -o $pass --output-format csv -- \
        python3 bench.py $ARGS > $OUT/v$v/$pass.stdout 2> $OUT/v$v/$pass.stderr
    rc=$?
    echo "v$v $pass rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
echo done
