# MFMA ceiling (no memory) and gemm_ws ablations at the FFN-up shape
set -u
mkdir -p gpurun_out
O=gpurun_out/r03_ws_ablate.jsonl
: > $O
timeout -k 5 120 t-one_amd/mfma_peak 4000 >> $O 2>&1 || exit $?
for d in 5 1 3 7 6; do echo "dbg=$d" >> $O; timeout -k 5 90 env ROWSCALE=1 XSDBG=$d t-one_amd/gemm_bench_ablate 40960 384 3072 2 -200 1 20 >> $O 2>&1 || exit $?; done
echo done
