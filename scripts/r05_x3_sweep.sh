#!/bin/bash
# fp32-mode (split) GEMM tile sweep at config 2's shapes (M = 2560 full layers, 1280 reduced): every gemm_x3 tile
# (50-61), the fp32-W ring kernel (40-49) and the current route (-2), FULLF32 operands; NOC2 (no shadow in fp32 mode).
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_x3_sweep.jsonl
: > $out
run() {  # M K N epi rowscale variants
  ROWSCALE=$5 FULLF32=1 NOC2=1 timeout -k 10 120 ./t-one_amd/gemm_bench $1 $2 $3 $4 $6 1 30 | sed "s/}\$/, \"rowscale\": $5}/" >> $out || exit $?
}
X3="-2,50,51,52,53,54,55,56,57,58,59,60,61"
R3="40,41,42,43,44,45,46,47,48,49"
for M in 1280 2560; do
  run $M 384 768 3 1 "$X3,$R3"      # pw1 (GLU)
  run $M 384 3072 2 1 "$X3,$R3"     # FFN up (SwiGLU)
  run $M 1536 384 1 0 "$X3,$R3"     # FFN down (RESID)
  run $M 384 384 1 0 "$X3,$R3"      # attn-out / pw2 (RESID)
  run $M 384 1152 0 1 "$X3,$R3"     # q|k|v of layers 0 / 7 (STORE)
  run $M 384 384 0 1 "$X3,$R3"      # v (STORE)
done
echo done
