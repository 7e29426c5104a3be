#!/bin/bash
# tests/test_gpu_kernels.py (GEMM routes through gemm_bench, non-GEMM kernels through kernel_check), then the same
# sub_conv checks against kernel_check_nobar (sub_conv_bf16's slab barrier removed: expected to FAIL), then the fused
# norm's cost in the row-panel kernel (gemm_bench timing, NORMW=0 / 1).  Tag: gpurun_out/<tag>_*.
set -u
tag=${1:-kt}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_kernel_tests.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -3 gpurun_out/${tag}_kernel_tests.log; grep "^FAILED" gpurun_out/${tag}_kernel_tests.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
if [ -x t-one_amd/kernel_check_nobar ]; then
  TONE_KERNEL_CHECK=$PWD/t-one_amd/kernel_check_nobar timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -v -k sub_conv --timeout 120 --timeout-method thread > gpurun_out/${tag}_nobar.log 2>&1
  echo "nobar rc=$? (expected 1)"; grep -E "passed|failed" gpurun_out/${tag}_nobar.log | tail -2; grep -o "'flat': [0-9.e+-]*" gpurun_out/${tag}_nobar.log | head -5
fi
for n in 0 1; do
  for K in 1536 384; do
    NORMW=$n RES16=1 timeout -k 10 120 t-one_amd/gemm_bench 40960 $K 384 1 90 1 50 | tail -1
  done
done > gpurun_out/${tag}_rp_norm_cost.jsonl
cat gpurun_out/${tag}_rp_norm_cost.jsonl
exit $rc
