#!/bin/bash
# closing evidence, part 2: one profiled step per bench leg, then the PMC traffic summaries the bench line quotes
# (profiles/<round>_traffic_<prec>_b<batch>.json via scripts/pmc_traffic.sh + traffic_summary.py)
set -u
tag=${1:-r06_final}
rnd=${2:-r06}
bash scripts/step_breakdown.sh ${tag}_fp32_b256 || exit 1
bash scripts/step_breakdown.sh ${tag}_fp32_400ms_b256 --chunk-samples 3200 || exit 1
bash scripts/step_breakdown.sh ${tag}_bf16_b4096 --precision bf16 --batch 4096 || exit 1
bash scripts/step_breakdown.sh ${tag}_fp8_b4096 --precision fp8 --batch 4096 || exit 1
bash scripts/step_breakdown.sh ${tag}_fp32_b1 --batch 1 || exit 1
for t in fp32_b256 fp32_400ms_b256 bf16_b4096 fp8_b4096 fp32_b1; do echo "== $t $(tail -1 gpurun_out/step_${tag}_$t.txt)"; done
for pb in "fp32 256" "bf16 4096" "fp8 4096" "bf16 2048"; do
  set -- $pb
  bash scripts/pmc_traffic.sh $1 $2 || exit 1
  python scripts/traffic_summary.py gpurun_out/pmc_$1 $1 $2 > gpurun_out/${rnd}_traffic_$1_b$2.json || exit 1
  cut -c1-300 gpurun_out/${rnd}_traffic_$1_b$2.json
done
