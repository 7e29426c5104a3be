#!/bin/bash
# the fp32 rowscale projections on gemm_d3n over the packed residual copy: kernel tests, fp32 parity tests, same-box A/B
# of TONE_D3X (headline and 400 ms), one profiled fp32 B = 256 step
set -u
tag=${1:-d3x}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v -k "d3 or packed or _pk or reduce or upsample or rmsnorm or fp32_routes" --timeout 300 --timeout-method thread > gpurun_out/${tag}_kt.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -1 gpurun_out/${tag}_kt.log; grep -E "^(FAILED|ERROR)" gpurun_out/${tag}_kt.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_400ms.py tests/test_gpu_ring.py tests/test_decode.py tests/test_pipeline_dropin.py -m gpu -v -k "not bf16 and not fp8 and not lowprec" --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/${tag}_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/${tag}_tests.log | head; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/${tag}_ab.jsonl
for i in 1 2; do
  for d in 0 1; do
    for c in 2400 3200; do
      TONE_D3X=$d timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-s 0 --alt 0 --config4 0 --config5 0 --chunk-samples $c > gpurun_out/${tag}_b.log 2>&1 || { tail -5 gpurun_out/${tag}_b.log; exit 1; }
      tail -1 gpurun_out/${tag}_b.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(json.dumps({'d3x': $d, 'chunk': $c, 'value': r['value'], 'ms_per_step': r['ms_per_step']}))" >> gpurun_out/${tag}_ab.jsonl
    done
  done
done
cat gpurun_out/${tag}_ab.jsonl
bash scripts/step_breakdown.sh ${tag}_fp32_b256 --precision fp32 --batch 256 || exit 1
head -14 gpurun_out/step_${tag}_fp32_b256.txt; tail -1 gpurun_out/step_${tag}_fp32_b256.txt
