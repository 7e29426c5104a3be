#!/bin/bash
# tests/test_gpu_kernels.py on the tree (all kernel-level cases)
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py -v --timeout 300 --timeout-method thread > gpurun_out/r05_kernel_tests2.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r05_kernel_tests2.log | tail -15; exit $rc
