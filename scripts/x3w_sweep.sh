# gemm_x3 two-waves-per-SIMD variants (56-59) vs the current picks
set -u
mkdir -p gpurun_out
out=gpurun_out/x3w_sweep.jsonl
: > $out
run() { ROWSCALE=$1 FULLF32=1 timeout -k 10 60 ./t-one_amd/gemm_bench $2 $3 $4 $5 $6 1 20 >> $out 2>&1 || { echo "fail $*"; exit 1; }; }
run 1 2560 384 3072 2 53,56,57,58
run 0 2560 1536 384 1 50,56,57,58
run 1 2560 384 1152 0 54,56,57,58
run 1 2560 384 768 3 51,56,57,58
run 0 2560 384 384 1 50,56,57,58
run 1 1280 384 3072 2 53,56,57,58
run 0 1280 1536 384 1 50,56,57,58
cat $out
