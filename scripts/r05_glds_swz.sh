#!/bin/bash
# gemm_glds with the (row >> 1) & 7 chunk swizzle (conflict-free ds_read_b128 groups on 128-byte rows) vs
# libtonehip_prev.so (1b9dac2): GPU suite, per-kernel A/B at bf16 B = 4096 and B = 2048, LDS-conflict PMC pass
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_glds_tests.log 2>&1 || { tail -30 gpurun_out/r05_glds_tests.log; exit 1; }
tail -2 gpurun_out/r05_glds_tests.log
bash scripts/r05_step_ab.sh glds_bf16_b4096 --precision bf16 --batch 4096 || exit 1
bash scripts/r05_step_ab.sh glds_bf16_b2048 --precision bf16 --batch 2048 || exit 1
bash scripts/r05_pmc_lds.sh
