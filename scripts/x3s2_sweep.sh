# gemm_x3 small-LDS tile variants (12-16: several workgroups per CU) vs the routed ones at the fp32 B=256 shapes
set -u
mkdir -p gpurun_out
out=gpurun_out/x3s2_sweep.jsonl
: > $out
B=./t-one_amd/gemm_bench
run() { FULLF32=1 NOC2=1 timeout -k 10 60 $B "$@" >> $out 2>&1 || { echo "fail $*"; cat $out; exit 1; }; }
V=70,80,82,83,84,85,86
run 2560 384 384 1 $V 1 50
run 1280 384 384 1 $V 1 50
run 2560 1536 384 1 $V 1 50
run 1280 1536 384 1 $V 1 50
ROWSCALE=1 run 2560 384 1152 0 76,$V 1 50
ROWSCALE=1 run 2560 384 768 3 71,73,75,83,85 1 50
ROWSCALE=1 run 1280 384 768 3 71,73,75,83,85 1 50
ROWSCALE=1 run 2560 384 3072 2 77,83,85 1 50
ROWSCALE=1 run 1280 384 3072 2 76,83,85 1 50
cat $out
