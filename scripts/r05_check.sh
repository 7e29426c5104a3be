#!/bin/bash
# the GPU suite, then a step A/B of the tree's library against t-one_amd/libtonehip_prev.so (LEGS, default the three
# headline legs); tag = $1
set -u
tag=${1:-check}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_${tag}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r05_${tag}_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r05_${tag}_gpu_tests.log
BASE_LIB=t-one_amd/libtonehip_prev.so LEGS="${LEGS:-fp32 256;bf16 4096;fp8 4096}" STEPS=${STEPS:-100} bash scripts/r05_ab.sh $tag
