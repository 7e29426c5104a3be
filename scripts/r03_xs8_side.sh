# gemm_xs8 (fp8 FFN up, K = 384) with the vectorised launch-time W-scale / bias copy vs the previous build
set -u
mkdir -p gpurun_out
O=gpurun_out/r03_xs8_side.jsonl
: > $O
for r in 1 2 3; do
  for b in gemm_bench_old gemm_bench; do
    for M in 40960 20480 10240; do
      echo "$b up M=$M" >> $O; timeout -k 5 90 env ROWSCALE=1 t-one_amd/$b $M 384 3072 2 98 1 50 >> $O 2>&1 || exit $?
    done
  done
done
echo done
