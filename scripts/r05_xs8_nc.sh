#!/bin/bash
# gemm_xs8 run length (XSNC W tiles per work item, 0 = auto) sweep after the counted-wait change
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_xs8_nc.jsonl
: > $out
for rep in 1 2; do
  for M in 40960 20480 10240; do
    for nc in 0 4 6 8 12 16 24 48; do
      XSNC=$nc ROWSCALE=1 timeout -k 10 60 ./t-one_amd/gemm_bench $M 384 3072 2 98 1 20 | sed "s/}\$/, \"nc\": $nc}/" >> $out || exit $?
    done
  done
done
cat $out
