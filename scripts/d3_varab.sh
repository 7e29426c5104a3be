#!/bin/bash
# gemm_d3 variant choice in the step itself (TONE_D3_V forces one variant for every shape; "d" = the shape table)
set -u
tag=${1:-d3v}
mkdir -p gpurun_out; : > gpurun_out/${tag}_varab.jsonl
run() {  # label, env var value, bench args...
  local lab=$1 v=$2; shift 2
  if [ "$v" = d ]; then unset TONE_D3_V; else export TONE_D3_V=$v; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-s 0 --alt 0 --config4 0 --config5 0 "$@" > gpurun_out/${tag}_b.log 2>&1 || { tail -5 gpurun_out/${tag}_b.log; exit 1; }
  tail -1 gpurun_out/${tag}_b.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(json.dumps({'leg': '$lab', 'v': '$v', 'value': r['value'], 'ms_per_step': r['ms_per_step']}))" >> gpurun_out/${tag}_varab.jsonl
  unset TONE_D3_V
}
for i in 1 2; do
  for v in d 6 7; do run headline $v; done
done
for v in d 3 6; do run 400ms $v --chunk-samples 3200; done
cat gpurun_out/${tag}_varab.jsonl
