#!/bin/bash
# Round-3 pass V: dependent pairs of random reads over a growing span (tools/micro/dep.hip).
set -u
mkdir -p gpurun_out/r03v
timeout -k 10 300 ./tools/micro/dep > gpurun_out/r03v/dep_pairs.jsonl 2>&1
rc=$?; cat gpurun_out/r03v/dep_pairs.jsonl; exit $rc
