#!/bin/bash
# One GPU pass, parameterised (replaces round 3's ~40 one-off tools/gpu_r03*.sh).  Runs on the GPU box via gpurun:
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash tools/gpu_pass.sh <tag> <step> [<step> ...]
# steps (in the order given; the pass stops at the first failing step, and no GPU step follows a fault or timeout):
#   suite        pytest -m gpu (as the driver runs it, with per-test timeouts) and __graft_entry__.smoke()
#   test:<a,b>   pytest -m gpu -k "a or b" (one test group)
#   bench        the default bench line (what the driver's BENCH record runs)
#   lines        every bench.py workload line (tools/bench_all.sh); lines:<a,b,..> a subset
#   line:<key>   one workload line: key as in prof:<key>
#   prof:<key>   rocprofv3 kernel trace + PMC passes of one workload (tools/profile.sh) into gpurun_out/prof_<tag>_<key>;
#                keys: cfg2 cfg2c cfg1 cfg4 cfg4m cfg2u cfg2d cfg2dw fused cfg3 cfg2w fused80 fused256 fused512 xdphbm frames
#   lat:<key>    latency-attribution PMC passes of one workload (tools/profile_lat.sh)
#   micro        tools/micro/gather (random-gather rates by table size; built here beforehand)
#   commit       commit latency, 1 and 4 device slots, and live swaps mid-stream (tools/commit_latency.py, swap_stream.py)
#   pcie / hostpack / hoststream   the host-fed feed's microbenchmarks and infw_classify_host (tools/micro, tools/host_stream.py)
# Output: gpurun_out/<tag>/ (logs); summarise profiles afterwards with tools/summarize_profile.py <tag>_<key>.
set -u
TAG=${1:?tag}; shift
O=gpurun_out/$TAG
mkdir -p $O

args_of() {  # bench.py arguments of a workload key
  case $1 in
    cfg2)   echo "" ;;
    cfg2c)  echo "--layout compact" ;;
    cfg1)   echo "--cfg 1 --batch 67108864" ;;
    cfg1c)  echo "--cfg 1 --batch 67108864 --layout compact" ;;
    cfg4)   echo "--cfg 4" ;;
    cfg4m)  echo "--cfg 4 --prefixes 1000000" ;;
    cfg2u)  echo "--uniform" ;;
    cfg2d)  echo "--templates 1000000" ;;
    cfg2dw) echo "--templates 1000000 --key-order workload" ;;
    cfg2w)  echo "--key-order workload" ;;
    xdphbm) echo "--xdp-ring hbm" ;;
    xdphp)  echo "--xdp-ring host-packed --steps 10 --warmup 2" ;;
    xdphb)  echo "--xdp-ring host-bursts --steps 10 --warmup 2" ;;
    xdphb32) echo "--xdp-ring host-bursts --burst-size 32 --steps 10 --warmup 2" ;;
    fused80)  echo "--from-frames 80 --fused" ;;
    fused256) echo "--from-frames 256 --fused" ;;
    fused512) echo "--from-frames 512 --fused" ;;
    fused)  echo "--from-frames 128 --fused" ;;
    frames) echo "--from-frames 128" ;;
    cfg3)   echo "--global-packets 1073741824 --steps 10 --warmup 2" ;;
    *) echo "unknown workload key $1" >&2; return 1 ;;
  esac
}

step() {
  local s=$1 rc=0
  case $s in
    suite)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
          > $O/pytest_gpu.log 2>&1 || rc=$?
      tail -3 $O/pytest_gpu.log
      [ $rc -eq 0 ] || return $rc
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || rc=$?
      tail -1 $O/smoke.log ;;
    test:*)  # test:a,b,c -> pytest -k "a or b or c" (no spaces: the step list is word-split on the way in)
      local k=${s#test:} lg=$O/pytest_$(echo ${s#test:} | tr , _).log
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
          -k "$(echo $k | sed 's/,/ or /g')" > $lg 2>&1 || rc=$?
      tail -3 $lg ;;
    sweep|sweep:*)  # infw_classify_xdp_host over packer threads x chunk (tools/xdp_host_sweep.py); sweep:<args joined by +>
      local sa=""; [ "$s" != sweep ] && sa=$(echo ${s#sweep:} | tr + ' ')
      timeout -k 10 600 python -u tools/xdp_host_sweep.py --trace $sa >> $O/xdp_host_sweep.jsonl 2>> $O/xdp_host_sweep.trace || rc=$?
      tail -30 $O/xdp_host_sweep.jsonl ;;
    bench)
      timeout -k 10 300 python -u bench.py > $O/bench_default.log 2>&1 || rc=$?
      tail -1 $O/bench_default.log | cut -c1-400 ;;
    lines)
      bash tools/bench_all.sh $O/lines || rc=$? ;;
    lines:*)  # a comma-separated subset of tools/bench_all.sh's lines
      bash tools/bench_all.sh $O/lines $(echo ${s#lines:} | tr , ' ') || rc=$? ;;
    line:*)
      local a; a=$(args_of ${s#line:}) || return 2
      timeout -k 10 300 python -u bench.py $a --no-cpu-baseline > $O/line_${s#line:}.log 2>&1 || rc=$?
      tail -1 $O/line_${s#line:}.log | cut -c1-300 ;;
    prof:*)
      local a; a=$(args_of ${s#prof:}) || return 2
      [ "${s#prof:}" = cfg3 ] && a="--global-packets 1073741824"
      bash tools/profile.sh ${TAG}_${s#prof:} $a --steps 5 --warmup 1 --no-cpu-baseline || rc=$? ;;
    lat:*)       # latency attribution PMC passes of one workload (tools/profile_lat.sh) into gpurun_out/lat_<tag>_<key>
      local a; a=$(args_of ${s#lat:}) || return 2
      bash tools/profile_lat.sh ${TAG}_${s#lat:} $a || rc=$? ;;
    micro)
      timeout -k 10 300 ./tools/micro/gather > $O/gather.jsonl 2>&1 || rc=$? ;;
    pcie)     # GPU reads of pinned host memory and the SDMA 2D header gather (tools/micro/pcie.hip, built beforehand)
      timeout -k 10 300 ./tools/micro/pcie > $O/pcie.jsonl 2>&1 || rc=$?
      tail -4 $O/pcie.jsonl ;;
    hostpack) # the host packer alone on the box's cores (CPU only; tools/micro/hostpack.cpp, built beforehand)
      (nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; lscpu | grep -E "Model name|^CPU\(s\)|NUMA node\(s\)") > $O/host_cpu.txt 2>&1
      timeout -k 10 300 ./tools/micro/hostpack --umem-gib 8 --descs 16 --threads 1,4,8,16 > $O/hostpack.jsonl 2>&1 || rc=$?
      tail -4 $O/hostpack.jsonl ;;
    hostpackx) # the packer's per-core rate by input order and output memory (32 GiB umem, 2048-B chunks)
      for cfg in "--keep 1 --out vector" "--keep 4 --out vector" "--keep 4 --out pinned" "--keep 4 --out registered" \
                 "--keep 1 --shuffle --out pinned"; do
        timeout -k 10 300 ./tools/micro/hostpack --umem-gib 32 --descs 16 --thp 1 --threads 1,16 $cfg \
            >> $O/hostpackx.jsonl 2>&1 || { rc=$?; break; }
      done
      tail -12 $O/hostpackx.jsonl ;;
    commit)   # commit latency at configs[2] scale, one and four device slots (tools/commit_latency.py)
      timeout -k 10 300 python -u tools/commit_latency.py > $O/commit_latency.jsonl 2>&1 || rc=$?
      [ $rc -eq 0 ] && { timeout -k 10 300 python -u tools/commit_latency.py --slots 4 > $O/commit_latency_4slots.jsonl 2>&1 || rc=$?; }
      [ $rc -eq 0 ] && { timeout -k 10 300 python -u tools/swap_stream.py > $O/swap_stream.log 2>&1 || rc=$?; }
      tail -3 $O/commit_latency.jsonl; tail -4 $O/swap_stream.log ;;
    hoststream) # infw_classify_host: SoA tuples in host memory, chunked H2D / classify / D2H
      timeout -k 10 300 python -u tools/host_stream.py --per-call 1024,4096,16384,65536,262144,1048576 \
          > $O/host_stream.json 2>&1 || rc=$?
      tail -8 $O/host_stream.json ;;
    *) echo "unknown step $s"; return 2 ;;
  esac
  echo "step $s rc=$rc"
  return $rc
}

for s in "$@"; do
  step $s || { echo "pass $TAG stopped at $s"; exit 1; }
done
echo "pass $TAG all-ok"
