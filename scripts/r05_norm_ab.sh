#!/bin/bash
# FFN2 down with / without the fused norm inside the bf16 B = 4096 step (one-step sequences)
set -u
export TMPDIR=/tmp
SEQ=seq bash scripts/step_breakdown.sh bf16_b4096_norm1 --precision bf16 --batch 4096 || exit $?
TONE_RP_NORM=0 SEQ=seq bash scripts/step_breakdown.sh bf16_b4096_norm0 --precision bf16 --batch 4096 || exit $?
for t in norm1 norm0; do echo $t; grep -E "rp_kernel|rmsnorm" gpurun_out/step_bf16_b4096_$t.txt | tail -70 | awk '{print $1}' | tr '\n' ' '; echo; tail -1 gpurun_out/step_bf16_b4096_$t.txt 2>/dev/null; grep total gpurun_out/step_bf16_b4096_$t.txt; done
