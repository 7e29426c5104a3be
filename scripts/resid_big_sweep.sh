# bf16 RESID projections (N = 384) at config 3 / 4 batches (M = 10240 .. 40960): routed kernel (-1) vs gemm_t
# tiles (21 = 128x256, 23 = 128x128) and the LDS-DMA tiles (14 = 128x128 4x2, 0/1 = 128x128 2x2 S2/S3, 7 = 64x128)
set -u
mkdir -p gpurun_out
out=gpurun_out/resid_big.jsonl
: > $out
B=./t-one_amd/gemm_bench
for pass in 1 2; do
for M in 10240 20480 40960; do
  timeout -k 10 60 $B $M 1536 384 1 -1,21,23,14,0,1,7 1 20 >> $out 2>&1 || echo "fail $M"
  timeout -k 10 60 $B $M 384 384 1 -1,21,23,14,0,1,7 1 20 >> $out 2>&1 || echo "fail $M"
done
done
cat $out
