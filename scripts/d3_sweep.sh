#!/bin/bash
# gemm_d3 (fp32 split, fragment-packed operands straight into registers) against the routed fp32 kernels at the N = 384
# shapes of the fp32 step (300 ms: M = 2560 / 1280 at B = 256; 400 ms: 3328 / 1536; smaller batches), and the fp32
# SwiGLU epilogue writing FFN down's A packed (CPACK)
set -u
out=gpurun_out/${1:-d3}_sweep.jsonl
mkdir -p gpurun_out; : > $out
V=-2,-500,-501,-502,-503,-504,-505,-506,-507,-508,-509
for M in ${MS:-2560 1280 3328 1536 640 320 128}; do
  for K in 384 1536; do
    PACKX=1 FULLF32=1 timeout -k 10 120 t-one_amd/gemm_bench $M $K 384 1 $V 1 200 >> $out || { echo "fail M=$M K=$K"; exit 1; }
  done
done
for M in 2560 1280; do
  for c in 0 1; do
    CPACK=$c FULLF32=1 timeout -k 10 120 t-one_amd/gemm_bench $M 384 3072 2 -2 1 200 | sed "s/^{/{\"cpack\": $c, /" >> $out || exit 1
  done
done
cut -c1-150 $out
