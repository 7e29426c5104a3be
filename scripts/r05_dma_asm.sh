#!/bin/bash
# every LDS-DMA from inline asm (counted LDS waits in every kernel): GPU suite, then per-kernel A/B against
# libtonehip_prev.so on the fp32 B = 256 headline, bf16 B = 4096 and fp8 B = 4096 steps
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_dma_asm_tests.log 2>&1 || { tail -30 gpurun_out/r05_dma_asm_tests.log; exit 1; }
tail -2 gpurun_out/r05_dma_asm_tests.log
bash scripts/r05_step_ab.sh dmaasm_fp32_b256 || exit 1
bash scripts/r05_step_ab.sh dmaasm_bf16_b4096 --precision bf16 --batch 4096 || exit 1
bash scripts/r05_step_ab.sh dmaasm_fp8_b4096 --precision fp8 --batch 4096
