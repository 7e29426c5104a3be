#!/bin/bash
# gemm_xw ablations with counted LDS waits (XW_ABLATE build; timing only for dbg != 0): 1 no epilogue, 2 no MFMA,
# 3 neither, 4 no W DMA after the prologue, 16 no W fragment reads, 64 ping-pong schedule, 192 ping-pong (waves 0-3
# order for all)
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_xw_ablate2.jsonl
: > $out
for rep in ${REPS:-1 2}; do
  for M in 40960 20480; do
    for dbg in ${DBGS:-0 1 2 3 4 16 19 64 192}; do
      ROWSCALE=1 XSDBG=$dbg timeout -k 10 60 ./t-one_amd/gemm_bench_ablate $M 384 3072 2 -300 1 20 | sed "s/}\$/, \"dbg\": $dbg}/" >> $out || exit $?
    done
  done
done
cat $out
