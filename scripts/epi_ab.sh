# FFN-up (SwiGLU, fp32 out) epilogue cost in gemm_x3 / gemm_pp: full, no epilogue (+3200), fast exp/rcp
# activation (+204800)
set -u
mkdir -p gpurun_out
out=gpurun_out/epi_ab.jsonl
: > $out
B=./t-one_amd/gemm_bench
FULLF32=1 NOC2=1 PP=1 ROWSCALE=1 timeout -k 10 60 $B 2560 384 3072 2 77,3277,204877,50,3250,204850,77,204877 1 50 >> $out 2>&1
FULLF32=1 NOC2=1 PP=1 ROWSCALE=1 timeout -k 10 60 $B 1280 384 3072 2 76,3276,204876 1 50 >> $out 2>&1
FULLF32=1 NOC2=1 PP=1 ROWSCALE=1 timeout -k 10 60 $B 2560 384 768 3 71,3271,204871 1 50 >> $out 2>&1
cat $out
