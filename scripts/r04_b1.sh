# B = 1 drop-in latency A/B: gemm_sm's cross-workgroup K split on / off (TONE_SM_NOSPLIT), one-step breakdowns, and
# the GPU tests that run the small-M GEMMs
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in split nosplit split; do
  if [ $v = nosplit ]; then export TONE_SM_NOSPLIT=1; else unset TONE_SM_NOSPLIT; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 2 --alt 0 --config4 0 --config5 0 --cpu-baseline-s 0 > gpurun_out/b1_$v.json 2> gpurun_out/b1_$v.err || { tail -5 gpurun_out/b1_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/b1_$v.json')); print('$v', d['latency_b1']['device_step_median_ms'], d['latency_b1']['dropin_numpy_median_ms'], d['value'])"
done
unset TONE_SM_NOSPLIT
bash scripts/step_breakdown.sh fp32_b1 --batch 1 || exit $?
head -24 gpurun_out/step_fp32_b1.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "dropin or ragged or small or b1 or golden or stagewise or fp32" --timeout 300 --timeout-method thread > gpurun_out/r04_b1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_b1_tests.log; exit $rc
