# gemm_t vs the 128x128 LDS-DMA kernel at the B=2048 encoder shapes (ROWSCALE=1 where the session folds RMSNorm)
set -u
mkdir -p gpurun_out
out=gpurun_out/gsweep2.log
: > $out
run() { timeout -k 10 120 ./t-one_amd/gemm_bench "$@" >> $out 2>&1 || { echo "rc=$? on $*"; tail -3 $out; exit 1; }; }
ROWSCALE=1 run 20480 384 3072 2 14,20,21,22,23
ROWSCALE=1 run 10240 384 3072 2 14,20,21,22,23
run 20480 1536 384 1 14,21,23
run 10240 1536 384 1 14,21,23
ROWSCALE=1 run 20480 384 1152 0 14,21,23
run 20480 384 384 1 14,21,23
ROWSCALE=1 run 20480 384 768 3 14,20,21,22,23
cat $out
