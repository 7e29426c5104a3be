set -u
mkdir -p gpurun_out
out=gpurun_out/gsweep3.log
: > $out
run() { timeout -k 10 120 ./t-one_amd/gemm_bench "$@" >> $out 2>&1 || { echo "rc=$? on $*"; tail -3 $out; exit 1; }; }
ROWSCALE=1 run 20480 384 3072 2 20,24,25,14
ROWSCALE=1 run 10240 384 3072 2 20,24,25,14
run 20480 1536 384 1 14,24,25
run 10240 1536 384 1 14,24,25
ROWSCALE=1 run 20480 384 1152 0 14,24,25
run 20480 384 384 1 14,24,25
ROWSCALE=1 run 20480 384 768 3 14,24,25
cat $out
