# bf16 GEMM variant sweep at the B=2048 encoder shapes (tools/gemm_bench.hip).
set -u
mkdir -p gpurun_out
B=${B:-2048}
M10=$((B * 10)); M5=$((B * 5))
V=${V:-0,3,6,7,16,19,22,23,32,39,48,55}
run() { timeout -k 10 120 ./t-one_amd/gemm_bench "$@" >> gpurun_out/gemm_sweep.log 2>&1 || { echo "rc=$? on $*"; exit 1; }; }
run $M10 384 3072 2 $V
run $M5 384 3072 2 $V
run $M10 1536 384 1 $V
run $M10 384 1152 0 $V
run $M10 384 384 1 $V
run $M10 384 768 3 $V
echo done
