#!/bin/bash
# Round-3 pass P: random 16-B gathers with a fixed footprint (64 MiB, 1 GiB) spread over 1..12 GiB of address
# span — does the line rate fall with span (address translation), as configs[2]'s one-list-per-key tables suggest?
set -u
mkdir -p gpurun_out/r03p
timeout -k 10 300 ./tools/micro/gather bigspread > gpurun_out/r03p/gather_bigspread.jsonl 2>&1
rc=$?; cat gpurun_out/r03p/gather_bigspread.jsonl; exit $rc
