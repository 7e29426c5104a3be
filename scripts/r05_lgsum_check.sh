#!/bin/bash
# permlane lane-group reductions in attention_rec / gemm_sm: the GPU suite, then bf16 B = 4096 and fp32 B = 1 steps
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_lgsum_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r05_lgsum_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r05_lgsum_gpu_tests.log
bash scripts/step_breakdown.sh bf16_lgsum --precision bf16 --batch 4096 || exit 1
grep -E "attention|sub_conv" gpurun_out/step_bf16_lgsum.txt
bash scripts/step_breakdown.sh fp32_b1_lgsum --batch 1 || exit 1
head -3 gpurun_out/step_fp32_b1_lgsum.txt; tail -1 gpurun_out/step_fp32_b1_lgsum.txt
