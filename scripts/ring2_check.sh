#!/bin/bash
# resident state with the MHSA caches: ring tests, kernel checks of the ring kernels, one profiled bf16 B = 4096 step.
set -u
tag=${1:-ring2}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ring.py -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_ring_tests.log 2>&1
rc=$?; echo "ring tests rc=$rc"; tail -2 gpurun_out/${tag}_ring_tests.log; grep -E "^(FAILED|E  )" gpurun_out/${tag}_ring_tests.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v -k "ring or kv" --timeout 300 --timeout-method thread > gpurun_out/${tag}_kt.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -2 gpurun_out/${tag}_kt.log; grep -E "^(FAILED|E  )" gpurun_out/${tag}_kt.log | head -20
[ $rc -ne 0 ] && exit $rc
for c in kv_bf16 kv_ring_bf16; do timeout -k 10 120 t-one_amd/kernel_check $c 4096 10 30; timeout -k 10 120 t-one_amd/kernel_check $c 4096 5 15; done | cut -c1-200
bash scripts/step_breakdown.sh ${tag}_ring_bf16_b4096 --precision bf16 --batch 4096 --state ring || exit 1
grep -E "kv_assemble|dwconv" gpurun_out/step_${tag}_ring_bf16_b4096.txt; tail -1 gpurun_out/step_${tag}_ring_bf16_b4096.txt
