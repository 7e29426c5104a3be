#!/bin/bash
# MXFP8 activations with one binade of headroom (E = floor(log2 amax) - 7) and the scaled conversion: the fp8 tests,
# then a same-box A/B of the fp8 / bf16 B = 4096 steps against the library built before the change (TONEHIP_LIB)
set -u
tag=${1:-q7}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v -k "mx or q8 or xs8 or rmsnorm" --timeout 300 --timeout-method thread > gpurun_out/${tag}_kt.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -1 gpurun_out/${tag}_kt.log; grep -E "^(FAILED|ERROR)" gpurun_out/${tag}_kt.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_400ms.py tests/test_gpu_ring.py -m gpu -v -k "fp8 or lowprec or nan" --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/${tag}_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/${tag}_tests.log | head; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/${tag}_ab.jsonl
for i in 1 2; do
  for lib in t-one_amd/libtonehip_abq.so t-one_amd/libtonehip.so; do
    TONEHIP_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-s 0 --alt 0 --config4 0 --config5 0 --precision fp8 --batch 4096 > gpurun_out/${tag}_b.log 2>&1 || { tail -5 gpurun_out/${tag}_b.log; exit 1; }
    tail -1 gpurun_out/${tag}_b.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(json.dumps({'lib': '$lib', 'value': r['value'], 'ms_per_step': r['ms_per_step']}))" >> gpurun_out/${tag}_ab.jsonl
  done
done
cat gpurun_out/${tag}_ab.jsonl
bash scripts/step_breakdown.sh ${tag}_fp8_b4096 --precision fp8 --batch 4096 || exit 1
head -6 gpurun_out/step_${tag}_fp8_b4096.txt; tail -1 gpurun_out/step_${tag}_fp8_b4096.txt
