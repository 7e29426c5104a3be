#!/bin/bash
# TONE_NORM4 A/B: RMSNorm (no MXFP8 output) on 32 lanes per row with 16-byte runs vs one wave per row with single
# elements: kernel_check timing + every-element errors, the norm / parity / ring tests with it on, then the fp32 headline
# step, same box, interleaved.  Measured and NOT kept (76.0 -> 70.6 us per fp32 step, within the bench's noise); the
# rmsnorm4 kernel and TONE_NORM4 were removed after this run (profiles/r06_norm4_ab.txt)
set -u
tag=${1:-n4}
mkdir -p gpurun_out; out=gpurun_out/${tag}_ab.txt; : > $out
for x in 0 1; do
  for a in "rmsnorm 2560" "rmsnorm_pk 2560" "rmsnorm 1280" "rmsnorm_r16 20480" "rmsnorm_pk 100"; do
    echo "norm4=$x $a: $(TONE_NORM4=$x timeout -k 10 120 t-one_amd/kernel_check $a | grep '^{' | tail -1 | cut -c1-230)" | tee -a $out
  done
done
TONE_NORM4=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_400ms.py tests/test_gpu_ring.py -m gpu -q -k "rmsnorm or parity or ring or 400 or step or oracle" --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "norm4 tests rc=$rc: $(tail -1 gpurun_out/${tag}_tests.log)" | tee -a $out; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for x in 0 1; do
    TONE_NORM4=$x timeout -k 10 300 python bench.py --steps 60 --warmup 5 --cpu-baseline-s 0 --alt 0 --config4 0 --config5 0 > gpurun_out/${tag}_b.log 2>&1 || { tail -5 gpurun_out/${tag}_b.log; exit 1; }
    tail -1 gpurun_out/${tag}_b.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(json.dumps({'norm4': $x, 'fp32_b256_value': r['value'], 'ms_per_step': r['ms_per_step']}))" | tee -a $out
  done
done
for x in 0 1; do
  TONE_NORM4=$x bash scripts/step_breakdown.sh ${tag}_f$x --precision fp32 --batch 256 || exit 1
  echo "norm4=$x fp32: $(grep -E 'rmsnorm' gpurun_out/step_${tag}_f$x.txt | cut -c1-80) | $(tail -1 gpurun_out/step_${tag}_f$x.txt)" | tee -a $out
done
