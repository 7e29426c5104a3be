#!/bin/bash
# gemm_xw run length (W tiles per work item) sweep after the counted-wait changes: auto (-300) and nc = 4..48
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_xw_nc.jsonl
: > $out
for rep in 1 2; do
  for M in 40960 20480 10240; do
    for v in -300 -304 -306 -308 -312 -316 -324 -348; do
      ROWSCALE=1 timeout -k 10 60 ./t-one_amd/gemm_bench $M 384 3072 2 $v 1 20 | sed "s/}\$/, \"v\": $v}/" >> $out || exit $?
    done
  done
done
cat $out
