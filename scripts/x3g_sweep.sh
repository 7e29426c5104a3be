# GLU / SwiGLU projections of the reduced layers at B = 256 (M = 1280): current tiles vs 64x32 (bench 82)
set -u
mkdir -p gpurun_out
out=gpurun_out/x3g_sweep.jsonl
: > $out
run() {  # rowscale M K N epi variants
  ROWSCALE=$1 FULLF32=1 timeout -k 10 60 ./t-one_amd/gemm_bench $2 $3 $4 $5 $6 1 20 >> $out 2>&1 || { echo "fail $*"; exit 1; }
}
# variant 82 (XT<64,32,1,1,4,2>) was removed after this sweep
run 1 1280 384 768 3 71,82
run 1 2560 384 768 3 71,82
run 1 1280 384 3072 2 76,82
run 1 1280 384 1152 0 76,80,82
cat $out
