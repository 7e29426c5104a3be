#!/bin/bash
# gemm_xw with counted LDS waits (DMA from inline asm, no conditional LDS ops in the steady state, bias in the
# accumulators, X rows pre-scaled by the row factor) vs gemm_bench_prev; then the GPU suite and a bf16 B = 4096
# per-kernel A/B against libtonehip_prev.so
set -u
bash scripts/r05_xw_ab.sh || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_xw_lgkm_tests.log 2>&1 || { tail -30 gpurun_out/r05_xw_lgkm_tests.log; exit 1; }
tail -2 gpurun_out/r05_xw_lgkm_tests.log
bash scripts/r05_step_ab.sh xwlgkm_bf16_b4096 --precision bf16 --batch 4096
