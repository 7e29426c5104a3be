#!/bin/bash
# gemm_rp ablations (gemm_bench_ablate, RP_ABLATE): full, 1 no epilogue, 4 no K loop, 8 no DMA, 16 no MFMA,
# 32 no residual loads, and combinations; M = 40960 / 20480, K = 1536 / 384.
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_rp_ablate.jsonl
: > $out
for MK in "40960 1536" "40960 384" "20480 1536"; do
  set -- $MK
  for dbg in 0 1 4 8 16 32 9 17 24 25 48; do
    vv=$((dbg * 400 + 90))
    RES16=1 timeout -k 10 120 ./t-one_amd/gemm_bench_ablate $1 $2 384 1 $vv 1 30 | sed "s/}\$/, \"dbg\": $dbg}/" >> $out || exit $?
  done
done
cat $out
