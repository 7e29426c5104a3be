set -u
mkdir -p gpurun_out
out=gpurun_out/gsweep4.log
: > $out
run() { timeout -k 10 120 ./t-one_amd/gemm_bench "$@" >> $out 2>&1 || { echo "rc=$? on $*"; tail -3 $out; exit 1; }; }
# fp32 B=256 shapes: -2 = current fp32 path (with split-K), 30..33 = gemm_f32t variants
ROWSCALE=1 run 2560 384 384 0 -2,30,32,33
run 2560 384 384 1 -2,30,32,33
run 1280 384 384 1 -2,30,32,33
run 2560 1536 384 1 -2,30,32,33
run 1280 1536 384 1 -2,30,32,33
ROWSCALE=1 run 2560 384 768 3 -2,31
ROWSCALE=1 run 2560 384 1152 0 -2,30,31,33
ROWSCALE=1 run 2560 384 3072 2 -2,31
ROWSCALE=1 run 1280 384 3072 2 -2,31
cat $out
