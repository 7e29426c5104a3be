# split-K for the split-fp32 FFN down-projection (M x 1536 -> 384, RESID) and the other K=384 RESID
set -u
mkdir -p gpurun_out
out=gpurun_out/x3k_sweep.jsonl
: > $out
run() { FULLF32=1 timeout -k 10 60 ./t-one_amd/gemm_bench $1 $2 $3 $4 $5 $6 20 >> $out 2>&1 || { echo "fail $*"; exit 1; }; }
run 2560 1536 384 1 50 1
for ns in 2 3 4 6; do run 2560 1536 384 1 50,54,56 $ns; done
run 1280 1536 384 1 50 1
for ns in 2 4; do run 1280 1536 384 1 50,54,56 $ns; done
run 2560 384 384 1 50 1
for ns in 2 3; do run 2560 384 384 1 50,54,56 $ns; done
cat $out
