# fp8 FFN down (gemm_mx RESID, K = 1536, N = 384): K-loop vs epilogue split.  MXDBG bits: 1 no epilogue,
# 4 no MFMA, 16 / 32 force 256 / 128-row X tiles
set -u
mkdir -p gpurun_out
O=gpurun_out/r03_mx_resid_ablate.jsonl
: > $O
for M in 40960 20480; do
  for d in 0 1 4 5 32 33 36 37; do
    echo "M=$M MXDBG=$d" >> $O
    MXDBG=$d timeout -k 5 90 t-one_amd/gemm_bench_ablate $M 1536 384 1 99 1 50 >> $O 2>&1 || exit $?
  done
done
echo done
