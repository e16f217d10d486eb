#!/bin/bash
# tools/micro/line per read form: rates, then L2 / L1 request counters per form at an L2-resident (1 MiB) and an
# HBM-sized (2 GiB) table.  Usage (GPU box): tools/micro/line_pmc.sh <tag>
set -u
OUT=gpurun_out/line_${1:-r03}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 ./tools/micro/line > $OUT/rates.jsonl 2> $OUT/rates.stderr || exit $?
echo rates rc=0
for f in 1 2 4 8; do
  for mib in 1 2048; do
    for grp in "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
      name=f${f}_m${mib}_$(echo $grp | cut -d' ' -f1)
      timeout -k 10 60 rocprofv3 --pmc $grp -d $OUT/$name -o $name --output-format csv -- ./tools/micro/line $f $mib \
          > $OUT/$name.stdout 2> $OUT/$name.stderr
      rc=$?; echo "$name rc=$rc"
      if [ $rc -ne 0 ]; then exit $rc; fi
    done
  done
done
