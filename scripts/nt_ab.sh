# bf16 FFN up on gemm_t (20 = 256x256, 22 = 256x128) with plain vs non-temporal h stores (+200), plus PMC fetch
set -u
mkdir -p gpurun_out
out=gpurun_out/nt_ab.jsonl
: > $out
B=./t-one_amd/gemm_bench
for pass in 1 2; do
for M in 10240 20480 40960; do
  ROWSCALE=1 timeout -k 10 60 $B $M 384 3072 2 20,220 1 20 >> $out 2>&1 || echo "fail $M"
done
ROWSCALE=1 timeout -k 10 60 $B 2560 384 3072 2 22,222 1 20 >> $out 2>&1 || echo "fail 2560"
done
cat $out
