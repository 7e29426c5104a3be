# microbenchmarks (dwconv state stream, RESID output bytes), the fp16-residual A/B, one-step breakdowns
set -u
export TMPDIR=/tmp
bash scripts/r04_dwconv.sh || exit $?
bash scripts/r04_resid_bytes.sh || exit $?
bash scripts/r04_ab.sh res16 || exit $?
bash scripts/step_breakdown.sh bf16_b4096 --precision bf16 --batch 4096 || exit $?
bash scripts/step_breakdown.sh fp8_b4096 --precision fp8 --batch 4096 || exit $?
head -30 gpurun_out/step_fp8_b4096.txt
