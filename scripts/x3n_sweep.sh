# narrow x3 tiles (variants 9-11 = bench 79-81) vs the 64x64 default (70) for the N = 384 projections
set -u
mkdir -p gpurun_out
out=gpurun_out/x3n_sweep.jsonl
: > $out
run() {  # rowscale M K N epi variants [nsplit]
  ROWSCALE=$1 FULLF32=1 timeout -k 10 60 ./t-one_amd/gemm_bench $2 $3 $4 $5 $6 ${7:-1} 20 >> $out 2>&1 || { echo "fail $*"; exit 1; }
}
run 0 1280 384 384 1 70,79,80,81
run 0 2560 384 384 1 70,79,80,81
run 0 2560 1536 384 1 70,79,80,81
run 0 1280 1536 384 1 70,79,80,81
run 0 1280 1536 384 1 50,59 2
run 1 1280 384 384 0 70,79,80,81
cat $out
