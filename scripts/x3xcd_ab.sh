#!/bin/bash
# TONE_X3_XCD A/B: gemm_x3's tiles dealt to the XCDs as 2 M halves x 4 N quarters (each L2 fills half of X and a quarter
# of W) vs the N-only split (all of X per XCD): fp32 FFN up in gemm_bench, then the fp32 headline step, same box,
# interleaved
set -u
tag=${1:-x3xcd}
mkdir -p gpurun_out; out=gpurun_out/${tag}_ab.jsonl; : > $out
for M in 2560 1280; do
  for x in 0 1; do
    TONE_X3_XCD=$x FULLF32=1 timeout -k 10 120 t-one_amd/gemm_bench $M 384 3072 2 -2 1 200 | sed "s/^{/{\"x3_xcd\": $x, /" >> $out || exit 1
  done
done
for i in 1 2 3; do
  for x in 0 1; do
    TONE_X3_XCD=$x timeout -k 10 300 python bench.py --steps 60 --warmup 5 --cpu-baseline-s 0 --alt 0 --config4 0 --config5 0 > gpurun_out/${tag}_b.log 2>&1 || { tail -5 gpurun_out/${tag}_b.log; exit 1; }
    tail -1 gpurun_out/${tag}_b.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(json.dumps({'x3_xcd': $x, 'value': r['value'], 'ms_per_step': r['ms_per_step']}))" >> $out
  done
done
for x in 0 1; do
  TONE_X3_XCD=$x bash scripts/step_breakdown.sh ${tag}_x$x --precision fp32 --batch 256 || exit 1
  echo "x3_xcd=$x: $(grep -E 'gemm_x3_kernel<tone::XT<128, (256|128), 2, 4, 1, [23]>, 2' gpurun_out/step_${tag}_x$x.txt | awk '{s+=$1} END {print s}') us FFN up, $(tail -1 gpurun_out/step_${tag}_x$x.txt)"
done
cut -c1-160 $out
