# fp32-by-bf16-split GEMM (gemm_x3, variants 50-55) vs the exact-fp32 MFMA kernels at the fp32 B=256
# encoder shapes; full-precision fp32 operands, fp64 reference (FULLF32=1).
set -u
mkdir -p gpurun_out
out=gpurun_out/x3_sweep.jsonl
: > $out
run() {  # rowscale M K N epi variants
  ROWSCALE=$1 FULLF32=1 timeout -k 10 60 ./t-one_amd/gemm_bench $2 $3 $4 $5 $6 1 20 >> $out 2>&1 || { echo "fail $*"; exit 1; }
}
run 1 2560 384 3072 2 -3,50,51,52,53,54,55
run 0 2560 1536 384 1 -3,30,50,51,52,53,54,55
run 1 2560 384 1152 0 -3,30,50,51,52,53,54,55
run 1 2560 384 768 3 -3,31,50,51,52,53,54,55
run 0 2560 384 384 1 -3,30,50,51,52,53,54,55
run 1 1280 384 3072 2 -3,50,51,52,53,54,55
run 0 1280 384 384 1 -3,30,50,51,52,53,54,55
cat $out
