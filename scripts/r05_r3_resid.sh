#!/bin/bash
# fp32 RESID shapes of the B = 256 step after the counted-wait change: routed gemm() (-2) against every gemm_r3
# variant (40-49, fp32 W streamed and split in registers); FULLF32: fp64 reference
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_r3_resid.jsonl
: > $out
export FULLF32=1 NOC2=1
for M in 2560 1280; do
  for KN in "1536 384" "384 384"; do
    set -- $KN
    for v in -2 40 41 42 43 44 45 46 47 48 49; do
      timeout -k 5 60 ./t-one_amd/gemm_bench $M $1 $2 1 $v 1 50 | sed "s/}\$/, \"v\": $v}/" >> $out || true
    done
  done
done
cat $out
