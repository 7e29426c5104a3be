# GEMM variant sweep at the encoder shapes (tools/gemm_bench.hip).  B=2048 bf16 variants, B=256 fp32 (-2).
set -u
mkdir -p gpurun_out
B=${B:-2048}
M10=$((B * 10)); M5=$((B * 5))
V=${V:-0,7,3,6,-1}
F=${F:-256}
F10=$((F * 10)); F5=$((F * 5))
run() { timeout -k 10 120 ./t-one_amd/gemm_bench "$@" >> gpurun_out/gemm_sweep.log 2>&1 || { echo "rc=$? on $*"; exit 1; }; }
run $M10 384 3072 2 $V
run $M5 384 3072 2 $V
run $M10 1536 384 1 $V
run $M10 384 1152 0 $V
run $M10 384 384 1 $V
run $M10 384 768 3 $V
if [ "$F" != 0 ]; then
  run $F10 384 3072 2 -2
  run $F5 384 3072 2 -2
  run $F10 1536 384 1 -2
  run $F10 384 1152 0 -2
  run $F10 384 384 1 -2
  run $F10 384 768 3 -2
fi
echo done
