#!/bin/bash
# gemm_xw epilogue grouping: 1 (tree), 2, 4 parts per slot (every 3 / 6 / 12 K-steps)
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_xw_epg.jsonl
: > $out
for rep in 1 2; do
  for bin in gemm_bench gemm_bench_epg2 gemm_bench_epg4; do
    for shape in "40960 384 3072 2" "20480 384 3072 2" "40960 384 768 3"; do
      ROWSCALE=1 timeout -k 10 120 ./t-one_amd/$bin $shape -300 1 20 | sed "s/}\$/, \"bin\": \"$bin\"}/" >> $out || exit $?
    done
  done
done
cat $out
