# MXFP8 GEMMs (gemm_mx, variant 99) vs the bf16 routes at the encoder shapes, B = 2048
set -u
mkdir -p gpurun_out
out=gpurun_out/mx_sweep.log
: > $out
run() { timeout -k 10 120 ./t-one_amd/gemm_bench "$@" >> $out 2>&1 || { echo "rc=$? on $*"; cat $out; exit 1; }; }
ROWSCALE=1 run 20480 384 3072 2 92,99 1 30
ROWSCALE=1 run 10240 384 3072 2 92,99 1 30
ROWSCALE=0 run 20480 1536 384 1 -1,99 1 30
ROWSCALE=0 run 10240 1536 384 1 -1,99 1 30
ROWSCALE=1 run 20480 384 1152 0 -1,99 1 30
ROWSCALE=1 run 20480 384 384 0 -1,99 1 30
cat $out
