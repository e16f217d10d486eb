#!/bin/bash
# Every bench.py workload line on the current build (on the GPU box).  Usage: tools/bench_all.sh <out_dir> [names]
set -u
OUT=${1:-gpurun_out/bench_all}
shift || true
ONLY=" $* "  # optional: the line names to run (default: all)
mkdir -p $OUT
run() {  # name, args...
  local name=$1; shift
  if [ "$ONLY" != "  " ] && [[ "$ONLY" != *" $name "* ]]; then return 0; fi
  timeout -k 10 300 python bench.py "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run cfg2 --steps 30
run cfg2_compact --layout compact --no-cpu-baseline --steps 30
run cfg1 --cfg 1 --batch 67108864 --no-cpu-baseline --steps 30
run cfg1_compact --cfg 1 --batch 67108864 --layout compact --no-cpu-baseline --steps 30
run cfg4 --cfg 4 --no-cpu-baseline --steps 30
run cfg4_1m --cfg 4 --prefixes 1000000 --no-cpu-baseline --steps 30
run cfg2_uniform --uniform --no-cpu-baseline --steps 30
run cfg2_distinct --templates 1000000 --no-cpu-baseline --steps 20
run cfg2_distinct_popularity_order --templates 1000000 --key-order workload --no-cpu-baseline --steps 20
run cfg2_frames --from-frames 128 --no-cpu-baseline --steps 20
run cfg2_frames_fused --from-frames 128 --fused --no-cpu-baseline --steps 20
run cfg2_xdp_hbm --xdp-ring hbm --no-cpu-baseline --steps 20
run cfg2_xdp_host --xdp-ring host --no-cpu-baseline --steps 10 --warmup 2
run cfg2_xdp_registered --xdp-ring registered --no-cpu-baseline --steps 10 --warmup 2
# the host-fed path: umem and rings in pageable memory, packed by the library's host threads (infw_classify_xdp_host)
run cfg2_xdp_host_packed --xdp-ring host-packed --no-cpu-baseline --steps 10 --warmup 2
run cfg2_xdp_host_packed_interleaved --xdp-ring host-packed --umem-order packet --no-cpu-baseline --steps 10 --warmup 2
# the same frames as DPDK-style bursts (a pointer, data_len and pkt_len per frame: infw_classify_bursts_host)
run cfg2_host_bursts --xdp-ring host-bursts --no-cpu-baseline --steps 10 --warmup 2
run cfg2_host_bursts32 --xdp-ring host-bursts --burst-size 32 --no-cpu-baseline --steps 10 --warmup 2
run cfg3_n1 --global-packets 1073741824 --no-cpu-baseline --steps 10 --warmup 2
# the library's one-process shape: one context over N device slots (all on this GPU), a thread + stream per slot
run inproc_n1 --in-process --gpus 1 --slots-on-gpu0 --global-packets 1073741824 --steps 5 --warmup 1 --no-line-rates
run inproc_n8 --in-process --gpus 8 --slots-on-gpu0 --global-packets 1073741824 --steps 5 --warmup 1 --no-line-rates
for f in $OUT/*.log; do
  python3 -c "import json; l=[x for x in open('$f') if x.startswith('{')]; d=json.loads(l[-1]); r=d.get('roofline', {}); print('$(basename $f .log)', d['value'], r.get('kernel_ms_avg', [s['kernel_ms_avg'] for s in d.get('per_slot', [])]), r.get('frac', ''), r.get('from_frames', {}).get('pack_kernel_ms_avg', ''), d['config'].get('stats_digest', '')[:12])"
done
