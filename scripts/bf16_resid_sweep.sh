# bf16 RESID projections of the reduced layers (M = 10240) and the full layers (M = 20480)
set -u
mkdir -p gpurun_out
out=gpurun_out/bf16_resid_sweep.jsonl
: > $out
run() { timeout -k 10 60 ./t-one_amd/gemm_bench $1 $2 $3 $4 $5 1 20 >> $out 2>&1 || { echo "fail $*"; exit 1; }; }
run 10240 1536 384 1 -1,14,0,1,3,5,7,8,21,23,24,25,40,41,42,43
run 10240 384 384 1 -1,14,0,1,3,5,7,8,21,23,24,25,40,41,42,43
run 20480 1536 384 1 -1,14,0,1,3,4,21,23,24,25,41,43
run 20480 384 384 1 -1,14,0,1,3,4,21,23,24,25,41,43
cat $out
