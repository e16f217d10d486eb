#!/bin/bash
# Round-3 pass ZC: experiment — the headline kernel with a 4096-entry word cache and a 256-entry IPv6 group cache
# (abtree/ build) against the tree's 2048 + 512, alternating bench runs at configs[2].
set -u
O=gpurun_out/r03zc
mkdir -p $O
LIB=abtree/ingress-node-firewall_amd/lib/libinfw.so
bash tools/ab_libs.sh $O/cfg2 $LIB c4096_b256 tree 4 --no-cpu-baseline --steps 30 || exit 1
echo all-ok
