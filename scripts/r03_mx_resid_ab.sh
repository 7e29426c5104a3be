# A/B of gemm_mx (MXFP8 FFN down, K = 1536, N = 384, RESID) before / after the running tile position
# (gemm_bench_old = previous commit, gemm_bench = working tree); two alternating rounds each
set -u
mkdir -p gpurun_out
O=gpurun_out/r03_mx_resid_ab.jsonl
: > $O
for r in 1 2; do
  for b in gemm_bench_old gemm_bench; do
    for M in 40960 20480; do
      echo "$b M=$M round=$r" >> $O
      timeout -k 5 90 t-one_amd/$b $M 1536 384 1 99 1 50 >> $O 2>&1 || exit $?
    done
  done
done
echo done
