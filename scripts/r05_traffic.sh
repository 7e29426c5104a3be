#!/bin/bash
# round-5 HBM traffic summaries (FFN up + RESID family) for the bench's legs: PMC passes, then the summaries
set -u
for leg in "fp32 256" "bf16 4096" "fp8 4096" "bf16 2048"; do
  set -- $leg
  bash scripts/pmc_traffic.sh $1 $2 || exit $?
  python3 scripts/traffic_summary.py gpurun_out/pmc_$1 $1 $2 > gpurun_out/r05_traffic_$1_b$2.json || exit $?
  cat gpurun_out/r05_traffic_$1_b$2.json
done
