#!/bin/bash
# Same-box A/B of two libinfw builds (on the GPU box): alternating bench.py runs, library A via INFW_LIB.
# Usage: tools/ab_libs.sh <out_dir> <libA.so> <nameA> <nameB> [rounds] [bench args...]
set -u
OUT=$1; LIBA=$2; NA=$3; NB=$4; R=${5:-3}; shift 5 2>/dev/null || shift $#
ARGS=${*:-"--no-cpu-baseline --steps 30"}
mkdir -p $OUT
for r in $(seq 1 $R); do
  INFW_LIB=$LIBA timeout -k 10 200 python bench.py $ARGS > $OUT/${NA}_$r.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py $ARGS > $OUT/${NB}_$r.log 2>&1 || exit 1
done
for f in $OUT/*_[0-9]*.log; do
  python3 -c "import json,sys; l=[x for x in open('$f') if x.startswith('{')]; d=json.loads(l[-1]); print('$(basename $f)', d['value'], d['roofline']['kernel_ms_avg'])"
done
