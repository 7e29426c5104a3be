#!/bin/bash
# gemm_d3 (fragment-packed A, PACKX=1; second line of each M) vs the routed fp32 kernel (gemm_r3, -2) for the k|v projection
# of layers 14 / 15 at B = 256 (M = B (S + T) = 10240 / 5120, N = 768); the first variant of each run reads cold
set -u
for M in 10240 5120; do
  FULLF32=1 NOC2=1 timeout -k 10 120 t-one_amd/gemm_bench $M 384 768 0 -504,-2,-500,-501,-503,-504,-507,-508 1 200 | grep '^{' | cut -c1-120
  PACKX=1 FULLF32=1 NOC2=1 timeout -k 10 120 t-one_amd/gemm_bench $M 384 768 0 -504,-500,-501,-503,-504,-505,-507,-508,-509 1 200 | grep '^{' | cut -c1-120
done
