set -u
O=gpurun_out/r05j; mkdir -p $O
C="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $C -d $O/tlb_fused -o tlb_fused --output-format csv -- python3 bench.py --from-frames 128 --fused --no-cpu-baseline --steps 3 --warmup 1 > $O/tlb_fused.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc $C -d $O/tlb_cfg2 -o tlb_cfg2 --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/tlb_cfg2.log 2>&1 || exit 1
echo ok
