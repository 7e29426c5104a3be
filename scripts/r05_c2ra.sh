#!/bin/bash
# conv2 taps with the next tap's fragments read ahead (sub_conv_bf16 / conv2_bf16) vs the previous commit's build
# (libtonehip_prev.so = 1b9dac2): GPU suite, bf16 B = 4096 and fp8 B = 4096 per-kernel A/B
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_c2ra_tests.log 2>&1 || { tail -30 gpurun_out/r05_c2ra_tests.log; exit 1; }
tail -2 gpurun_out/r05_c2ra_tests.log
bash scripts/r05_step_ab.sh c2ra_bf16_b4096 --precision bf16 --batch 4096 || exit 1
bash scripts/r05_step_ab.sh c2ra_fp8_b4096 --precision fp8 --batch 4096
