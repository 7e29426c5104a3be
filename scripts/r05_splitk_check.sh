#!/bin/bash
# fp32 FFN down on the 3-way K split at the 400 ms shapes: the 400 ms + fp32 parity tests, then the step A/B against
# the previous tree (fp32 B = 256 at 400 ms and 300 ms)
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_400ms.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "400ms or fp32 or ragged" > gpurun_out/r05_splitk_tests.log 2>&1 || { tail -30 gpurun_out/r05_splitk_tests.log; exit 1; }
tail -3 gpurun_out/r05_splitk_tests.log
BASE_LIB=t-one_amd/libtonehip_prev.so LEGS="fp32 256 3200;fp32 256" STEPS=150 bash scripts/r05_ab.sh splitk
