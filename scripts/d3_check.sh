#!/bin/bash
# gemm_d3 in the fp32 step: small-M sweep, the fp32 GPU parity tests, one profiled fp32 B = 256 step
set -u
tag=${1:-d3}
mkdir -p gpurun_out
MS="320 128 100" bash scripts/d3_sweep.sh ${tag} > /dev/null || { echo "sweep failed"; exit 1; }
grep -c error gpurun_out/${tag}_sweep.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v -k "d3 or packed or fp32_routes" --timeout 300 --timeout-method thread > gpurun_out/${tag}_kt.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -2 gpurun_out/${tag}_kt.log; grep -E "^(FAILED|ERROR)" gpurun_out/${tag}_kt.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_400ms.py tests/test_gpu_ring.py tests/test_decode.py -m gpu -v -k "not bf16 and not fp8 and not lowprec" --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${tag}_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/${tag}_tests.log | head -20
[ $rc -ne 0 ] && exit $rc
bash scripts/step_breakdown.sh ${tag}_fp32_b256 --precision fp32 --batch 256 || exit 1
head -12 gpurun_out/step_${tag}_fp32_b256.txt; tail -1 gpurun_out/step_${tag}_fp32_b256.txt
