# bf16 FFN up (SwiGLU, N = 3072, K = 384) across M: gemm_p (90 = XCD-contiguous, 97 = 2D XCD blocks, the default
# where the tiles divide) vs gemm_t tiles (20 = 256x256, 21 = 128x256, 22 = 256x128, 23 = 128x128); two passes
set -u
mkdir -p gpurun_out
out=gpurun_out/ffnup_route.jsonl
: > $out
B=./t-one_amd/gemm_bench
for pass in 1 2; do
for M in 1280 2560 3840 5120 7680 10240 20480 40960; do
  ROWSCALE=1 timeout -k 10 60 $B $M 384 3072 2 -1,90,97,20,21,22,23 1 20 >> $out 2>&1 || echo "fail $M"
done
done
cat $out
