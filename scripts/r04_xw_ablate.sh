# gemm_xw ablations at the FFN-up shape (M = 40960 / 20480): full kernel with the spread DMA (0), the gemm_xs DMA
# schedule (64), and components removed (1 no epilogue, 2 no MFMA, 4 no DMA, 16 no W reads; timing only).
# gemm_xs (-10) first as the reference.  Output: gpurun_out/r04_xw_ablate.jsonl
set -u
mkdir -p gpurun_out
out=gpurun_out/r04_xw_ablate.jsonl; : > $out
A=./t-one_amd/gemm_bench_ablate
for M in 40960 20480; do
  echo "# xs M=$M" >> $out
  ROWSCALE=1 timeout -k 5 60 $A $M 384 3072 2 -10 1 30 >> $out 2>&1 || exit 1
  for d in 0 64 128 1 2 3 16 0 64 128; do
    echo "# xw dbg=$d M=$M" >> $out
    ROWSCALE=1 XSDBG=$d timeout -k 5 60 $A $M 384 3072 2 -300 1 30 >> $out 2>&1 || exit 1
  done
done
cat $out | cut -c1-150
