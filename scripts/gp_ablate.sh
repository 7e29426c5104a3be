# gemm_p ablations at the FFN-up shape (M = 20480): full, no epilogue, no MFMA, no DMA, no epi+DMA, no MFMA+DMA
set -u
mkdir -p gpurun_out
out=gpurun_out/gp_ablate.log
: > $out
export ROWSCALE=1
for r in 1 2; do
  timeout -k 10 120 ./t-one_amd/gemm_bench 20480 384 3072 2 90,490,890,1690,2090,2490,690,2890 1 50 >> $out 2>&1 || { echo "rc=$?"; cat $out; exit 1; }
done
cat $out
