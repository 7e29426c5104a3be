#!/bin/bash
# gemm_xw (bf16 FFN up SwiGLU, pw1 GLU) microbenchmark: the tree's build against gemm_bench_prev (the previous commit)
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_xw_ab.jsonl
: > $out
for rep in 1 2; do
  for bin in gemm_bench_prev gemm_bench; do
    for shape in "40960 384 3072 2" "20480 384 3072 2" "40960 384 768 3"; do
      ROWSCALE=1 timeout -k 10 120 ./t-one_amd/$bin $shape -300 1 20 | sed "s/}\$/, \"bin\": \"$bin\"}/" >> $out || exit $?
    done
  done
done
cat $out
