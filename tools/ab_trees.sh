#!/bin/bash
# Same-box A/B between two builds: an older commit's tree, built here, against the current tree.
#   bash tools/ab_trees.sh prepare <commit>      (CPU container) build <commit> into abtree/old (git-ignored; travels
#                                                  with the gpurun snapshot — remove ./abtree from .gpurunignore first)
#   gpurun -- bash tools/ab_trees.sh run <tag> [bench.py args]   alternating old/new bench lines, 2 rounds,
#                                                  into gpurun_out/<tag>/{old,new}_<r>.log
# Used for profiles/r05h (the frames-fused line before and after the AF_XDP instantiation change).
set -u
ROOT=$(cd "$(dirname "$0")/.." && pwd)
case ${1:?prepare|run} in
  prepare)
    C=${2:?commit}
    WT=$(mktemp -d /tmp/abtree.XXXXXX)
    git -C "$ROOT" worktree add -f "$WT" "$C" >/dev/null || exit 1
    make -C "$WT" -j8 >/dev/null || exit 1
    rm -rf "$ROOT/abtree/old" && mkdir -p "$ROOT/abtree/old"
    tar -C "$WT" --exclude=./.git --exclude=./profiles --exclude=./ingress-node-firewall_amd/build -cf - . |
      tar -C "$ROOT/abtree/old" -xf - || exit 1
    git -C "$ROOT" worktree remove --force "$WT"
    echo "abtree/old = $C" ;;
  run)
    TAG=${2:?tag}; shift 2
    O=$ROOT/gpurun_out/$TAG; mkdir -p "$O"
    for r in 1 2; do
      (cd "$ROOT/abtree/old" && timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 20 "$@") > "$O/old_$r.log" 2>&1 || exit 1
      (cd "$ROOT" && timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 20 "$@") > "$O/new_$r.log" 2>&1 || exit 1
      for f in old_$r new_$r; do
        python3 -c "import json; [print('$f', d['build_id'], d['roofline']['kernel'], d['per_rank'][0]['kernel_ms_avg']) for d in (json.loads(l) for l in open('$O/$f.log') if l.startswith('{'))]"
      done
    done ;;
  *) echo "usage: $0 prepare <commit> | run <tag> [bench args]" >&2; exit 2 ;;
esac
