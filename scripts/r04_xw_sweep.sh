# gemm_xw (32x32x16 MFMA, cross-item pipeline) vs gemm_xs at the FFN-up / pw1 shapes; microbenchmark, one process
# per shape, variants alternated.  Output: gpurun_out/r04_xw_sweep.jsonl
set -u
mkdir -p gpurun_out
out=gpurun_out/r04_xw_sweep.jsonl; : > $out
run() { echo "# $*" >> $out; ROWSCALE=1 timeout -k 5 60 ./t-one_amd/gemm_bench "$@" >> $out 2>&1 || { echo "rc=$?"; exit 1; }; }
for M in 40960 20480 10240; do run $M 384 3072 2 -10,-300,-10,-300 1 30; done
run 40960 384 3072 2 -316,-312,-308,-324 1 30
run 40960 384 768 3 -10,-300,-10,-300 1 30
run 20480 384 768 3 -10,-300,-10,-300 1 30
cat $out
