#!/bin/bash
# Same-box A/B of the host packer's build-time knobs (csrc/hostfeed.cpp INFW_PACK_PF / INFW_PACK_NT): libraries built
# beforehand into exp/ (see the round-6 notes in DESIGN.md §7.3), loaded through INFW_LIB, alternated R times over the
# host-fed sweep in ring and packet umem order.  Usage (GPU box): tools/hostfeed_ab.sh <out_dir> [R] [variant ...]
set -u
OUT=${1:?out}; R=${2:-2}; shift 2 || true
VARIANTS=${*:-"base pf64 pf64nt"}
mkdir -p $OUT
for r in $(seq 1 $R); do
  for v in $VARIANTS; do
    lib=""; [ $v != base ] && lib=$PWD/exp/libinfw_$v.so
    for o in ring packet; do
      INFW_LIB=$lib timeout -k 10 300 python -u tools/xdp_host_sweep.py --order $o --threads 1,16 --chunks 524288 \
          --per-call 65536 --reps 5 > $OUT/${v}_${o}_$r.jsonl 2>> $OUT/err.log || exit $?
      python3 -c "
import json
rows=[json.loads(l) for l in open('$OUT/${v}_${o}_$r.jsonl')]
t={(x.get('threads'), x.get('per_call')): x['Mpps'] for x in rows[1:]}
print('$v', '$o', $r, 't1', t.get((1, None)), 't16', t.get((16, None)), 'call64k', t.get(('auto', 65536)), 'load', rows[-1]['loadavg_1m'])"
    done
  done
done
