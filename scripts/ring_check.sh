#!/bin/bash
# resident (ring) state: the ring tests, the dwconv kernel checks (flat and ring, with their launch times), then one
# profiled bf16 B = 4096 step per form.  Tag: gpurun_out/<tag>_*
set -u
tag=${1:-ring}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ring.py -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_ring_tests.log 2>&1
rc=$?; echo "ring tests rc=$rc"; tail -3 gpurun_out/${tag}_ring_tests.log; grep -E "^(FAILED|E  )" gpurun_out/${tag}_ring_tests.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v -k dwconv --timeout 300 --timeout-method thread > gpurun_out/${tag}_dw_tests.log 2>&1
rc=$?; echo "dwconv tests rc=$rc"; tail -2 gpurun_out/${tag}_dw_tests.log
for c in dwconv_bf16 dwconv_ring_bf16; do for T in 10 5; do timeout -k 10 120 t-one_amd/kernel_check $c 4096 $T; done; done > gpurun_out/${tag}_dw_times.jsonl
cat gpurun_out/${tag}_dw_times.jsonl
exit $rc
