#!/bin/bash
# fp32-mode route candidates, 3 interleaved repetitions: FFN up (SwiGLU) at M = 2560 / 3328 (300 / 400 ms full layers)
# and 1536 (400 ms reduced), q|k|v N = 1152 at M = 1280 / 1536 / 2560 / 3328, plus the 400 ms RESID / GLU shapes.
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_x3_sweep2.jsonl
: > $out
run() {  # M K N epi rowscale variants
  ROWSCALE=$5 FULLF32=1 NOC2=1 timeout -k 10 120 ./t-one_amd/gemm_bench $1 $2 $3 $4 $6 1 40 | sed "s/}\$/, \"rowscale\": $5}/" >> $out || exit $?
}
for rep in 1 2 3; do
  for M in 2560 3328 1536; do run $M 384 3072 2 1 "-2,56,57,58"; done
  for M in 1280 1536 2560 3328; do run $M 384 1152 0 1 "-2,51,52,56,61"; done
  for M in 1536 3328; do
    run $M 384 768 3 1 "-2,51,55,61"
    run $M 1536 384 1 0 "-2,50,59"
    run $M 384 384 1 0 "-2,50,59"
  done
done
echo done
