#!/bin/bash
# test_lowprec_stagewise_large_batch on the build before the gemm_rp_mx barrier fix (libtonehip_prev.so: expected to
# fail the fp8 case) and on the tree
set -u
mkdir -p gpurun_out
TONEHIP_LIB=$PWD/t-one_amd/libtonehip_prev.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k lowprec_stagewise -v --timeout 300 --timeout-method thread > gpurun_out/r05_stagewise_prev.log 2>&1
echo "prev rc=$?"; grep -E "PASSED|FAILED|AssertionError" gpurun_out/r05_stagewise_prev.log | head -8
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k lowprec_stagewise -v --timeout 300 --timeout-method thread > gpurun_out/r05_stagewise.log 2>&1
rc=$?; echo "tree rc=$rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r05_stagewise.log | tail -5; exit $rc
