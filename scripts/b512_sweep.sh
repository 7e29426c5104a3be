# bf16 RESID projections (N = 384) at the config-4 per-GPU batch (B = 512 at N = 8: M = 5120 / 2560): the routed
# kernel (-1 = gemm_f32t 64x64 with bf16 operands) vs LDS-DMA tiles (7-9 64x128, 14 128x128) with split-K,
# persistent (11, 12) and the transposed persistent kernels (20-23)
set -u
mkdir -p gpurun_out
out=gpurun_out/b512_sweep.jsonl
: > $out
B=./t-one_amd/gemm_bench
run() { timeout -k 10 60 $B "$@" >> $out 2>&1 || { echo "fail $*"; }; }
for MK in "5120 1536" "2560 1536" "5120 384" "2560 384"; do
  run $MK 384 1 -1,7,8,9,14,11,12,20,21,22,23 1 30
  run $MK 384 1 7,8,14 2 30
  run $MK 384 1 7,8,14 3 30
  run $MK 384 1 7,8 4 30
done
# the other B = 512 shapes: q|k|v (N = 1152, rowscale, bf16 out), pw1 (GLU), FFN up
ROWSCALE=1 run 5120 384 1152 0 -1,14,7,8,20,21,22,23 1 30
ROWSCALE=1 run 5120 384 768 3 -1,14,7,20,21,22,23,90 1 30
ROWSCALE=1 run 2560 384 768 3 -1,14,7,20,21,22,23 1 30
ROWSCALE=1 run 5120 384 3072 2 -1,20,21,22,23,90,91 1 30
ROWSCALE=1 run 2560 384 3072 2 -1,20,21,22,23,90,91 1 30
cat $out
