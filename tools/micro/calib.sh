#!/bin/bash
# PMC calibration of random-gather traffic: the gather microbenchmark with a known
# number of random lookups (grid*512*64*6 launches) into a 1 GiB table (every lookup a
# distinct-line L2 miss), W = 4 and 64 bytes, one counter group per pass.
set -u
OUT=gpurun_out/calib
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for w in 4 64; do
  for grp in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_MISS_sum TCC_REQ_sum"; do
    name=w${w}_$(echo $grp | cut -d' ' -f1)
    timeout -k 10 120 rocprofv3 --pmc $grp -d $OUT/$name -o $name --output-format csv -- ./tools/micro/gather $w 1024 \
        > $OUT/$name.stdout 2> $OUT/$name.stderr
    rc=$?; echo "$name rc=$rc"
    if [ $rc -ge 124 ]; then exit $rc; fi
  done
done
