#!/bin/bash
# gemm_d3 with X pre-split (a_packed 3: h as its three bf16 terms, fragment-packed by the SwiGLU epilogue) vs fp32 X split
# in registers (a_packed 1): FFN down in gemm_bench, the producer's output checked (CPACK=3), the fp32 step tests with
# TONE_D3S=1, then the fp32 headline step A/B, same box, interleaved.  Measured and NOT kept: the a_packed / c_packed 3
# form, PACKX=3 / CPACK=3 and TONE_D3S were removed after this run (profiles/r06_d3s_ab.jsonl, step_r06_d3s_s*_fp32_b256.txt)
set -u
tag=${1:-d3s}
mkdir -p gpurun_out; out=gpurun_out/${tag}_ab.jsonl; : > $out
for M in 2560 1280 3328 1536 640 100; do
  for px in 1 3; do
    PACKX=$px FULLF32=1 timeout -k 10 120 t-one_amd/gemm_bench $M 1536 384 1 -499,-503,-504,-507 1 200 | sed "s/^{/{\"packx\": $px, /" >> $out || { echo "fail M=$M px=$px"; exit 1; }
  done
done
for M in 2560 1280 100; do
  for c in 1 3; do
    CPACK=$c FULLF32=1 timeout -k 10 120 t-one_amd/gemm_bench $M 384 3072 2 -2 1 200 | sed "s/^{/{\"cpack\": $c, /" >> $out || exit 1
  done
done
cut -c1-150 $out
TONE_D3S=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_400ms.py tests/test_gpu_ring.py -m gpu -q -k "not bf16 and not fp8 and not lowprec" --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "d3s tests rc=$rc: $(tail -1 gpurun_out/${tag}_tests.log)"; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for x in 0 1; do
    TONE_D3S=$x timeout -k 10 300 python bench.py --steps 60 --warmup 5 --cpu-baseline-s 0 --alt 0 --config4 0 --config5 0 > gpurun_out/${tag}_b.log 2>&1 || { tail -5 gpurun_out/${tag}_b.log; exit 1; }
    tail -1 gpurun_out/${tag}_b.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(json.dumps({'d3s': $x, 'value': r['value'], 'ms_per_step': r['ms_per_step']}))" >> $out
  done
done
for x in 0 1; do
  TONE_D3S=$x bash scripts/step_breakdown.sh ${tag}_s$x --precision fp32 --batch 256 || exit 1
  echo "d3s=$x: $(grep -E 'gemm_d3_kernel<4, 1, 1, 3, 1' gpurun_out/step_${tag}_s$x.txt | awk '{s+=$1} END {print s}') us FFN down (M 2560), $(tail -1 gpurun_out/step_${tag}_s$x.txt)"
done
grep '"d3s"' $out
