# gemm_pp (ping-pong fp32 split) vs gemm_x3 at the fp32 B=256 FFN-up shapes; ablations of pp variant 0
# (dbg: +400 no MFMA, +1600 no DMA, +3200 no epilogue).  PP=1 maps variants 50-59 onto gemm_pp.
# gemm_bench_noslp: gemm_t.hip (x3) built with -fno-slp-vectorize (no packed-fp32 VALU in the split).
set -u
mkdir -p gpurun_out
out=gpurun_out/pp_sweep.jsonl
: > $out
run() { local B=$1; shift; FULLF32=1 NOC2=1 PP=1 timeout -k 10 60 $B "$@" >> $out 2>&1 || { echo "fail $*"; cat $out; exit 1; }; }
B=./t-one_amd/gemm_bench; BN=./t-one_amd/gemm_bench_noslp
echo '# pp' >> $out
ROWSCALE=1 run $B 2560 384 3072 2 50,51,52,450,1650,3250,2050 1 50
echo '# x3 slp / noslp' >> $out
ROWSCALE=1 run $B 2560 384 3072 2 77,77 1 50
ROWSCALE=1 run $BN 2560 384 3072 2 77,77 1 50
ROWSCALE=1 run $B 1280 384 3072 2 76 1 50
ROWSCALE=1 run $BN 1280 384 3072 2 76 1 50
run $B 2560 1536 384 1 70 1 50
run $BN 2560 1536 384 1 70 1 50
ROWSCALE=1 run $B 2560 384 768 3 71 1 50
ROWSCALE=1 run $BN 2560 384 768 3 71 1 50
cat $out
