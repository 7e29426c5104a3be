# gemm_pp with register staging (variants 6-8: global -> VGPR -> ds_write) vs LDS-DMA (0, 1, 2) and gemm_x3 (77 / 76),
# FFN-up shapes at B = 256 (T = 10 / 5); +25600 = lockstep schedule
set -u
mkdir -p gpurun_out
out=gpurun_out/pp_rg.jsonl
: > $out
B=./t-one_amd/gemm_bench
run() { FULLF32=1 NOC2=1 PP=1 timeout -k 10 60 $B "$@" >> $out 2>&1 || { echo "fail $*"; cat $out; exit 1; }; }
ROWSCALE=1 run 2560 384 3072 2 77,50,56,57,58,25656,77,56,57 1 50
ROWSCALE=1 run 1280 384 3072 2 76,52,58,25658,76,58 1 50
ROWSCALE=1 run 2560 384 1152 0 76,58,25658 1 50
cat $out
