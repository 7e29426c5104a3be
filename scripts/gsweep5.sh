set -u
mkdir -p gpurun_out
out=gpurun_out/gsweep5.log
: > $out
run() { timeout -k 10 120 ./t-one_amd/gemm_bench "$@" >> $out 2>&1 || { echo "rc=$? on $*"; tail -3 $out; exit 1; }; }
# bf16 B=2048 small-N shapes: -1 = current routing, 40..43 = K-split kernel on bf16 operands
ROWSCALE=1 run 20480 384 384 0 -1,40,42,43
run 20480 384 384 1 -1,40,42,43
run 10240 384 384 1 -1,40,42,43
run 20480 1536 384 1 -1,40,42,43
run 10240 1536 384 1 -1,40,42,43
ROWSCALE=1 run 20480 384 1152 0 -1,40,41,43
ROWSCALE=1 run 20480 384 768 3 -1,41
ROWSCALE=1 run 10240 384 768 3 -1,41
cat $out
