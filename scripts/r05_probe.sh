#!/bin/bash
# Round 5: the row-panel RESID kernel (gemm_rp, variants 90-98) against the LDS-DMA 128x128 tile (variant 14, the
# round-4 route) on the family's four shapes with the fp16 residual; the low-precision GPU parity tests; one-step
# sequences of the bf16 B = 4096 step.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r05_rp_sweep.jsonl
: > $out
for MK in "40960 1536" "20480 1536" "40960 384" "20480 384" "10240 1536" "10240 384"; do
  set -- $MK
  RES16=1 timeout -k 10 120 ./t-one_amd/gemm_bench $1 $2 384 1 14,90,93,94,95,96,97,98 1 30 >> $out || exit $?
done
cat $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "bf16 or fp8 or large or ragged or lowprec or stagewise" > gpurun_out/r05_rp_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05_rp_tests.log; [ $rc -ne 0 ] && exit $rc
SEQ=seq bash scripts/step_breakdown.sh bf16_b4096_seq --precision bf16 --batch 4096 || exit $?
head -30 gpurun_out/step_bf16_b4096_seq.txt
echo done
