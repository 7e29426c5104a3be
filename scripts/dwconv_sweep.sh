# dwconv workgroup-shape sweep (TONE_DWCONV_VARIANT): bf16 B=2048 and fp32 B=256 bench values.
set -u
mkdir -p gpurun_out
for v in 0 1 2 3; do
  TONE_DWCONV_VARIANT=$v timeout -k 10 200 python bench.py --precision bf16 --batch 2048 --cpu-baseline-s 0 --alt 0 > gpurun_out/dw_bf16_$v.log 2>&1 || exit $?
  echo "bf16 v=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dw_bf16_$v.log)"
  TONE_DWCONV_VARIANT=$v timeout -k 10 200 python bench.py --cpu-baseline-s 0 --alt 0 > gpurun_out/dw_fp32_$v.log 2>&1 || exit $?
  echo "fp32 v=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dw_fp32_$v.log)"
done
