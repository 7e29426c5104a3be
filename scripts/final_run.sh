#!/bin/bash
# closing evidence: suite + smoke + default bench + headline kernel stats, then one-step breakdowns of the
# bench legs (fp32 B = 256 headline, fp32 400 ms B = 256, bf16 / fp8 B = 4096, fp32 B = 1)
set -u
tag=${1:-final}
bash scripts/suite.sh $tag || exit $?
bash scripts/step_breakdown.sh ${tag}_fp32_b256 || exit 1
bash scripts/step_breakdown.sh ${tag}_fp32_400ms_b256 --chunk-samples 3200 || exit 1
bash scripts/step_breakdown.sh ${tag}_bf16_b4096 --precision bf16 --batch 4096 || exit 1
bash scripts/step_breakdown.sh ${tag}_fp8_b4096 --precision fp8 --batch 4096 || exit 1
bash scripts/step_breakdown.sh ${tag}_fp32_b1 --batch 1 || exit 1
for t in fp32_b256 fp32_400ms_b256 bf16_b4096 fp8_b4096 fp32_b1; do echo "== $t"; tail -1 gpurun_out/step_${tag}_$t.txt; done
