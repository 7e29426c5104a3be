#!/bin/bash
# exact-fp32 MFMA tiles (gemm_f32t, variants 30-33) against the routed fp32 split kernels (-2) on the K = 384 shapes of the
# fp32 B = 256 step: attn-out / pw2 (RESID, N = 384), pw1 (GLU, N = 768, row factor), q|k|v (STORE, N = 1152, row factor)
set -u
mkdir -p gpurun_out
out=gpurun_out/${1:-f32t}_probe.jsonl
: > $out
for M in 2560 1280; do
  FULLF32=1 NOC2=1 timeout -k 10 120 t-one_amd/gemm_bench $M 384 384 1 -2,30,31,32,33 1 50 >> $out || exit 1
  FULLF32=1 NOC2=1 ROWSCALE=1 timeout -k 10 120 t-one_amd/gemm_bench $M 384 768 3 -2,30,31,32,33 1 50 >> $out || exit 1
  FULLF32=1 NOC2=1 ROWSCALE=1 timeout -k 10 120 t-one_amd/gemm_bench $M 384 1152 0 -2,30,31,32,33 1 50 >> $out || exit 1
done
cat $out
