#!/bin/bash
# TONE_HEAD_MFMA A/B: the CTC head on the exact-fp32 MFMA (head_mfma_kernel) vs the LDS-fed FMA kernel (head_kernel):
# kernel_check timing + every-element errors, the head / parity / ring tests with it on, then the fp32 headline and the
# bf16 B = 4096 step, same box, interleaved
set -u
tag=${1:-hm}
mkdir -p gpurun_out; out=gpurun_out/${tag}_ab.txt; : > $out
for x in 0 1; do
  for a in "head 2560" "head 2570" "head_r16 40960" "head_r16 20480"; do
    echo "mfma=$x $a: $(TONE_HEAD_MFMA=$x timeout -k 10 120 t-one_amd/kernel_check $a | grep '^{' | tail -1 | cut -c1-220)" | tee -a $out
  done
done
TONE_HEAD_MFMA=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_400ms.py tests/test_gpu_ring.py -m gpu -q -k "head or parity or ring or 400 or step or oracle" --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "mfma tests rc=$rc: $(tail -1 gpurun_out/${tag}_tests.log)" | tee -a $out; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for x in 0 1; do
    TONE_HEAD_MFMA=$x timeout -k 10 300 python bench.py --steps 60 --warmup 5 --cpu-baseline-s 0 --alt 0 --config4 0 --config5 0 > gpurun_out/${tag}_b.log 2>&1 || { tail -5 gpurun_out/${tag}_b.log; exit 1; }
    tail -1 gpurun_out/${tag}_b.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(json.dumps({'head_mfma': $x, 'fp32_b256_value': r['value'], 'ms_per_step': r['ms_per_step']}))" | tee -a $out
  done
done
for x in 0 1; do
  TONE_HEAD_MFMA=$x bash scripts/step_breakdown.sh ${tag}_f$x --precision fp32 --batch 256 || exit 1
  TONE_HEAD_MFMA=$x bash scripts/step_breakdown.sh ${tag}_b$x --precision bf16 --batch 4096 || exit 1
  echo "mfma=$x fp32: $(grep -E 'head' gpurun_out/step_${tag}_f$x.txt | cut -c1-80) | $(tail -1 gpurun_out/step_${tag}_f$x.txt)" | tee -a $out
  echo "mfma=$x bf16: $(grep -E 'head' gpurun_out/step_${tag}_b$x.txt | cut -c1-80) | $(tail -1 gpurun_out/step_${tag}_b$x.txt)" | tee -a $out
done
