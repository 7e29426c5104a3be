#!/bin/bash
# blocked FFN hidden (round 6): gemm_bench timing of gemm_xw SWIGLU / gemm_rp FFN down with HBLK=0 / 1, the kernel
# tests, then one profiled bf16 B = 4096 step with TONE_H_BLOCKED=0 / 1 on this box.  Tag: gpurun_out/<tag>_*
set -u
tag=${1:-hb}
mkdir -p gpurun_out
for h in 0 1; do
  for M in 40960 20480; do
    HBLK=$h ROWSCALE=1 timeout -k 10 120 t-one_amd/gemm_bench $M 384 3072 2 -300 1 50 | tail -1 || exit 1
    HBLK=$h RES16=1 timeout -k 10 120 t-one_amd/gemm_bench $M 1536 384 1 90 1 50 | tail -1 || exit 1
    HBLK=$h RES16=1 NORMW=1 timeout -k 10 120 t-one_amd/gemm_bench $M 1536 384 1 90 1 50 | tail -1 || exit 1
  done
done > gpurun_out/${tag}_gemm.jsonl
cat gpurun_out/${tag}_gemm.jsonl
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_kernel_tests.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -2 gpurun_out/${tag}_kernel_tests.log; grep "^FAILED" gpurun_out/${tag}_kernel_tests.log | head
[ $rc -ne 0 ] && exit $rc
TONE_H_BLOCKED=0 bash scripts/step_breakdown.sh ${tag}_rowmajor_bf16_b4096 --precision bf16 --batch 4096 || exit 1
bash scripts/step_breakdown.sh ${tag}_blocked_bf16_b4096 --precision bf16 --batch 4096 || exit 1
for v in rowmajor blocked; do echo "== $v"; head -8 gpurun_out/step_${tag}_${v}_bf16_b4096.txt; tail -1 gpurun_out/step_${tag}_${v}_bf16_b4096.txt; done
