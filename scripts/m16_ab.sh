# gemm_x3 with the products on v_mfma_f32_16x16x32_bf16 (x3 variants 12 / 13 = 7 / 6 with M16) vs 32x32x16,
# at the fp32 B=256 shapes (FFN up T=10 / T=5, fused q|k|v), alternating to cancel drift
set -u
mkdir -p gpurun_out
out=gpurun_out/m16_ab.jsonl
: > $out
B=./t-one_amd/gemm_bench
run() { FULLF32=1 NOC2=1 timeout -k 10 60 $B "$@" >> $out 2>&1 || { echo "fail $*"; cat $out; exit 1; }; }
ROWSCALE=1 run 2560 384 3072 2 77,82,77,82,77,82 1 50
ROWSCALE=1 run 1280 384 3072 2 76,83,76,83 1 50
ROWSCALE=1 run 2560 384 1152 0 76,83,76,83 1 50
ROWSCALE=1 run 20480 384 3072 2 77,82,77,82 1 20
cat $out
