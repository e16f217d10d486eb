set -o pipefail
mkdir -p gpurun_out/r05d
timeout -k 10 600 python -u -m pytest tests/test_gpu_xdp.py tests/test_abi_cpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05d/pytest_xdp.log 2>&1 || { tail -30 gpurun_out/r05d/pytest_xdp.log; exit 1; }
tail -3 gpurun_out/r05d/pytest_xdp.log
timeout -k 10 300 python -u bench.py --xdp-ring hbm --no-cpu-baseline > gpurun_out/r05d/xdp_hbm.log 2>&1 || { tail -20 gpurun_out/r05d/xdp_hbm.log; exit 1; }
tail -1 gpurun_out/r05d/xdp_hbm.log | cut -c1-300
timeout -k 10 400 python -u bench.py --xdp-ring host --no-cpu-baseline > gpurun_out/r05d/xdp_host.log 2>&1 || { tail -20 gpurun_out/r05d/xdp_host.log; exit 1; }
tail -1 gpurun_out/r05d/xdp_host.log | cut -c1-300
