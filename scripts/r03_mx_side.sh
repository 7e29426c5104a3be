# gemm_mx with the batched, prefetched side data vs the previous build (gemm_bench_old: before the running tile
# positions); then the fp8 GPU tests
set -u
mkdir -p gpurun_out
O=gpurun_out/${OUT:-r03_mx_side}.jsonl
: > $O
for r in 1 2; do
  for b in gemm_bench_old gemm_bench; do
    echo "$b qkv M=40960" >> $O; timeout -k 5 90 env ROWSCALE=1 t-one_amd/$b 40960 384 1152 0 99 1 50 >> $O 2>&1 || exit $?
    echo "$b qkv N=384 M=40960" >> $O; timeout -k 5 90 env ROWSCALE=1 t-one_amd/$b 40960 384 384 0 99 1 50 >> $O 2>&1 || exit $?
    echo "$b up M=2560" >> $O; timeout -k 5 90 env ROWSCALE=1 t-one_amd/$b 2560 384 3072 2 99 1 50 >> $O 2>&1 || exit $?
    echo "$b down M=40960" >> $O; timeout -k 5 90 t-one_amd/$b 40960 1536 384 1 99 1 50 >> $O 2>&1 || exit $?
    echo "$b down M=20480" >> $O; timeout -k 5 90 t-one_amd/$b 20480 1536 384 1 99 1 50 >> $O 2>&1 || exit $?
    echo "$b down M=5120" >> $O; timeout -k 5 90 t-one_amd/$b 5120 1536 384 1 99 1 50 >> $O 2>&1 || exit $?
  done
done
CODES="1 3 29 31" ROUNDS=1 OUT=${OUT:-r03_mx_side}_ablate bash scripts/r03_mx_resid_ablate2.sh || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "fp8" > gpurun_out/${OUT:-r03_mx_side}_tests.log 2>&1
echo "tests rc=$?"
