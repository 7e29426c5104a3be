#!/bin/bash
# gemm_xs8 after the VALU trims (precomputed DMA offsets, scales before the ring, integer lane-group amax, scalar fp32
# SwiGLU without SLP packing): SwiGLU M = 40960 / 20480 timing (+ no-epilogue / no-MFMA ablations), then the fp8 GPU tests
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_xs8_valu.jsonl
: > $out
for rep in 1 2; do
  for d in 0 1 2; do
    NOREF=1 ROWSCALE=1 MXDBG=$d timeout -k 10 60 ./t-one_amd/gemm_bench_ablate 40960 384 3072 2 98 1 20 | sed "s/}\$/, \"dbg\": $d}/" >> $out || exit $?
  done
done
ROWSCALE=1 timeout -k 10 120 ./t-one_amd/gemm_bench 4096 384 3072 2 98 1 5 >> $out || exit $?
cat $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "fp8 or mx or xs8" > gpurun_out/r05_xs8_valu_tests.log 2>&1 || { tail -30 gpurun_out/r05_xs8_valu_tests.log; exit 1; }
tail -3 gpurun_out/r05_xs8_valu_tests.log
BASE_LIB=t-one_amd/libtonehip_prev.so LEGS="fp8 4096" STEPS=100 bash scripts/r05_ab.sh xs8_valu
