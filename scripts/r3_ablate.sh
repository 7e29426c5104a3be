#!/bin/bash
# gemm_r3 ablations (RESID epilogue; dbg bits: 1 no MFMA, 2 no split, 4 no LDS-DMA, 8 no epilogue):
# variant + 400 * dbg.  x3 (-2) for reference.
set -e
B=t-one_amd/gemm_bench
export FULLF32=1 NOC2=1
run() { timeout -k 5 60 $B "$@"; }
for V in 40 42 49; do
  L=""
  for D in 0 1 2 3 4 6 8 12 13; do L="$L,$((V + 400 * D))"; done
  run 2560 384 3072 1 -2${L} 1 50
  run 2560 1536 384 1 -2${L} 1 50
done
