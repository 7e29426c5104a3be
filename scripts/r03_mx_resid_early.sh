# fp8 FFN down (gemm_mx RESID): E = QPT (the whole K-step t + 2 issued after step t's stage-freeing barrier,
# MXDBG bit 8 -> DBG 64) vs E = QPT / 2; with / without epilogue (bit 1), 256 / 128-row X tiles (32)
set -u
mkdir -p gpurun_out
O=gpurun_out/r03_mx_resid_early.jsonl
: > $O
for r in 1 2; do
for M in 40960 20480; do
  for d in 0 8 1 9 32 40; do
    echo "M=$M MXDBG=$d" >> $O
    MXDBG=$d timeout -k 5 90 t-one_amd/gemm_bench_ablate $M 1536 384 1 99 1 50 >> $O 2>&1 || exit $?
  done
done
done
echo done
