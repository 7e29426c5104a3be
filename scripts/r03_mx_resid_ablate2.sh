# fp8 FFN down (gemm_mx RESID, K = 1536, N = 384): what the K loop's 42 us are made of.  MXDBG = 256 x kernel DBG
# bits: 1 no epilogue, 4 no MFMA, 8 no LDS fragment reads, 16 no DMA after the first two K-steps
set -u
mkdir -p gpurun_out
O=gpurun_out/${OUT:-r03_mx_resid_ablate2}.jsonl
: > $O
for r in ${ROUNDS:-1 2}; do
for M in 40960 20480; do
  for c in ${CODES:-0 1 5 13 21 29}; do
    echo "M=$M DBG=$c" >> $O
    MXDBG=$((256 * c)) timeout -k 5 90 t-one_amd/gemm_bench_ablate $M 1536 384 1 99 1 50 >> $O 2>&1 || exit $?
  done
done
done
echo done
