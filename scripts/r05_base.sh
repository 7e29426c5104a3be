#!/bin/bash
# Round-5 start: unprofiled default bench + one-step breakdowns (bf16 / fp8 B = 4096) on the round-start tree.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-base}
timeout -k 10 600 python -u bench.py > gpurun_out/r05_${tag}_bench.json 2> gpurun_out/r05_${tag}_bench.err || exit $?
echo bench done
bash scripts/step_breakdown.sh bf16_b4096 --precision bf16 --batch 4096 || exit $?
bash scripts/step_breakdown.sh fp8_b4096 --precision fp8 --batch 4096 || exit $?
echo breakdowns done
