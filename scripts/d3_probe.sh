#!/bin/bash
# gemm_d3 timing probes: coalesced W (dbg 16) / X (dbg 32) / both, against the plain kernel (wrong results, timing only)
set -u
out=gpurun_out/${1:-d3}_probe.jsonl
mkdir -p gpurun_out; : > $out
for M in 2560 1280; do
  for K in 384 1536; do
    for d in 0 16 32 48; do
      XSDBG=$d timeout -k 10 120 t-one_amd/gemm_bench $M $K 384 1 -500,-503,-504 1 200 | sed "s/^{/{\"dbg\": $d, /" >> $out || exit 1
    done
  done
done
cut -c1-110 $out
