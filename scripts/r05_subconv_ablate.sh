set -u
for d in ${DBGS:-0 1 4 5}; do
  TONE_SUBCONV_DBG=$d bash scripts/step_breakdown.sh bf16_sc$d --precision bf16 --batch 4096 || exit 1
  grep sub_conv gpurun_out/step_bf16_sc$d.txt | head -1
done
