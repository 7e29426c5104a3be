# gemm_sm (small-M exact fp32) vs the split kernels it replaces at the B = 1 / B = 4 shapes of the fp32 step:
# -2 = gemm() fp32 routing (now gemm_sm for M <= 64), 55 / 59 = gemm_x3 variants 5 / 9 (the previous routes);
# FULLF32=1: full-precision operands, fp64 reference.  Output: gpurun_out/r04_sm_check.jsonl
set -u
mkdir -p gpurun_out
out=gpurun_out/r04_sm_check.jsonl; : > $out
run() { echo "# $*" >> $out; FULLF32=1 timeout -k 5 60 ./t-one_amd/gemm_bench "$@" >> $out 2>&1 || { echo "rc=$?"; exit 1; }; }
ROWSCALE=1 run 10 384 3072 2 -2,55,-2 1 50
ROWSCALE=1 run 5 384 3072 2 -2,55 1 50
ROWSCALE=1 run 40 384 3072 2 -2,55 1 50
run 10 1536 384 1 -2,59,-2 1 50
run 5 1536 384 1 -2,59 1 50
ROWSCALE=1 run 10 384 1152 0 -2,59 1 50
run 10 384 384 1 -2,59 1 50
ROWSCALE=1 run 10 384 768 3 -2,51 1 50
run 40 384 768 0 -2,59 1 50
run 20 384 768 0 -2,59 1 50
run 10 2176 384 0 -2,59 1 50
run 5 1536 384 0 -2,59 1 50
run 60 384 3072 2 -2,55 1 50
cat $out
