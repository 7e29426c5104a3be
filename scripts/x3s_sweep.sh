# gemm_x3 with a pre-split A (variants 60-65) vs in-register split (50-55) and exact fp32 (-3)
set -u
mkdir -p gpurun_out
out=gpurun_out/x3s_sweep.jsonl
: > $out
run() { ROWSCALE=$1 FULLF32=1 timeout -k 10 60 ./t-one_amd/gemm_bench $2 $3 $4 $5 $6 1 20 >> $out 2>&1 || { echo "fail $*"; exit 1; }; }
run 1 2560 384 3072 2 -3,53,61,63,65
run 0 2560 1536 384 1 -3,50,60,61,62,63,64,65
run 1 2560 384 1152 0 -3,54,60,61,62,63,64,65
run 1 2560 384 768 3 -3,51,61,63,65
run 1 2560 384 384 0 -3,50,60,62,63,64
run 1 1280 384 3072 2 -3,53,61,63,65
run 0 1280 1536 384 1 -3,50,60,62,63,64
cat $out
