# In-step A/B of the X-stationary bf16 FFN-up / pw1 kernels: gemm_xs (TONE_XW=0) vs gemm_xw with the interleaved
# schedule (TONE_XW=1) at bf16 B = 4096 and B = 2048: bench lines + one-step rocprof breakdowns
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for xw in 0 1; do
  for B in 4096 2048; do
    TONE_XW=$xw timeout -k 10 300 python bench.py --precision bf16 --batch $B --steps 100 --cpu-baseline-s 0 --alt 0 --config4 0 --config5 0 > gpurun_out/r04_xwstep_${xw}_$B.json 2> gpurun_out/r04_xwstep_${xw}_$B.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r04_xwstep_${xw}_$B.json'));r=d['roofline'];print('xw=$xw B=$B', d['value'], d['ms_per_step'], r['families_us_per_step'].get('gemm_ffn_up'), r['families_us_per_step'].get('gemm_pw1'), r['encoder_gemm_frac'])"
  done
  TONE_XW=$xw bash scripts/step_breakdown.sh xw${xw}_bf16_b4096 --precision bf16 --batch 4096 || exit $?
done
head -6 gpurun_out/step_xw0_bf16_b4096.txt gpurun_out/step_xw1_bf16_b4096.txt
