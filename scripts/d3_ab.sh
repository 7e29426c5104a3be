#!/bin/bash
# gemm_d3 on / off (TONE_D3) in the fp32 headline step, same box, interleaved; plus the 400 ms fp32 step breakdown
set -u
tag=${1:-d3ab}
mkdir -p gpurun_out; : > gpurun_out/${tag}_ab.jsonl
for i in 1 2; do
  for d in 0 1; do
    TONE_D3=$d timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-s 0 --alt 0 --config4 0 --config5 0 > gpurun_out/${tag}_b.log 2>&1 || { tail -5 gpurun_out/${tag}_b.log; exit 1; }
    tail -1 gpurun_out/${tag}_b.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(json.dumps({'d3': $d, 'value': r['value'], 'ms_per_step': r['ms_per_step']}))" >> gpurun_out/${tag}_ab.jsonl
  done
done
cat gpurun_out/${tag}_ab.jsonl
