#!/bin/bash
set -u
tag=${1:-d3f}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v -k "d3 or packed or fp32_routes" --timeout 300 --timeout-method thread > gpurun_out/${tag}_kt.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -1 gpurun_out/${tag}_kt.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_400ms.py tests/test_gpu_ring.py tests/test_decode.py tests/test_pipeline_dropin.py -m gpu -v -k "not bf16 and not fp8 and not lowprec" --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/${tag}_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/${tag}_tests.log | head; [ $rc -ne 0 ] && exit $rc
bash scripts/d3_ab.sh ${tag} || exit 1
bash scripts/step_breakdown.sh ${tag}_fp32_b256 --precision fp32 --batch 256 || exit 1
bash scripts/step_breakdown.sh ${tag}_fp32_400ms --precision fp32 --batch 256 --chunk-samples 3200 || exit 1
head -8 gpurun_out/step_${tag}_fp32_b256.txt; tail -1 gpurun_out/step_${tag}_fp32_b256.txt
head -8 gpurun_out/step_${tag}_fp32_400ms.txt; tail -1 gpurun_out/step_${tag}_fp32_400ms.txt
