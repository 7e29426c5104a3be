#!/bin/bash
# fp32-split GEMM shapes of the B = 256 step: round-1 routing (-2: gemm() with W planes) vs the
# K-tile ring kernel (gemm_r3, variants 40-49).  FULLF32=1: full fp32 operands, fp64 reference.
set -e
B=t-one_amd/gemm_bench
export FULLF32=1 NOC2=1
run() { timeout -k 5 60 $B "$@"; }
for M in 2560 1280; do
  ROWSCALE=1 run $M 384 3072 2 -2,40,41,47,48 1 50     # FFN up (SwiGLU)
  run $M 1536 384 1 -2,42,43,44,49 1 50                # FFN down (residual)
  run $M 384 384 1 -2,42,43,44,49 1 50                 # attention out / pw2
  ROWSCALE=1 run $M 384 768 3 -2,45,46,41 1 50         # pw1 (GLU)
  ROWSCALE=1 run $M 384 384 0 -2,42,43,44,49 1 50      # q (STORE, row scale)
  ROWSCALE=1 run $M 384 1152 0 -2,45,42,41 1 50        # fused qkv
done
run 10240 384 768 0 -2,41,45,40 1 50                   # k|v of layer 15
run 5120 384 768 0 -2,41,45,40 1 50                    # k|v of layer 14
run 2560 2176 384 0 -2,42,43,49 1 50                   # subsampling Linear
