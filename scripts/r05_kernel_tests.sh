#!/bin/bash
# tests/test_gpu_kernels.py against the build before the gemm_rp_mx barrier fix (gemm_bench_head: expected to fail
# the fp8 RESID K = 384 cases) and against the tree's build (expected to pass)
set -u
mkdir -p gpurun_out
TONE_GEMM_BENCH=$PWD/t-one_amd/gemm_bench_head timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -q --timeout 300 --timeout-method thread > gpurun_out/r05_kernel_tests_head.log 2>&1
echo "head rc=$?"; grep -E "passed|failed" gpurun_out/r05_kernel_tests_head.log | tail -3; grep "^FAILED" gpurun_out/r05_kernel_tests_head.log | head
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v --timeout 300 --timeout-method thread > gpurun_out/r05_kernel_tests.log 2>&1
rc=$?; echo "tree rc=$rc"; tail -3 gpurun_out/r05_kernel_tests.log; exit $rc
