#!/bin/bash
# fp8 FFN down on the row-panel kernel (gemm_rp_mx) vs gemm_mx (microbenchmark, fp16 residual), the fp8 / bf16 GPU
# parity tests, and the fp8 B = 4096 step sequence
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r05_rpmx.jsonl
: > $out
for M in 40960 20480 10240; do
  for rep in 1 2; do
    RES16=1 timeout -k 10 60 ./t-one_amd/gemm_bench $M 1536 384 1 99 1 30 | sed 's/}$/, "kernel": "gemm_mx"}/' >> $out || exit $?
    RPMX=1 RES16=1 timeout -k 10 60 ./t-one_amd/gemm_bench $M 1536 384 1 99 1 30 | sed 's/}$/, "kernel": "gemm_rp_mx"}/' >> $out || exit $?
  done
done
cat $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_400ms.py -x -v --timeout 300 --timeout-method thread \
  -k "bf16 or fp8 or large or ragged or lowprec" > gpurun_out/r05_rpmx_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05_rpmx_tests.log; [ $rc -ne 0 ] && exit $rc
SEQ=seq bash scripts/step_breakdown.sh fp8_b4096_rpmx --precision fp8 --batch 4096 || exit $?
head -16 gpurun_out/step_fp8_b4096_rpmx.txt
