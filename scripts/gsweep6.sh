set -u
mkdir -p gpurun_out
out=gpurun_out/gsweep6.log
: > $out
run() { timeout -k 10 120 ./t-one_amd/gemm_bench "$@" >> $out 2>&1 || { echo "rc=$? on $*"; tail -3 $out; exit 1; }; }
run 160 1536 384 0 -1,42
run 320 384 384 1 -1,42
ROWSCALE=1 run 320 384 1152 0 -1,42
run 2560 1536 384 0 -2,30
cat $out
