#!/bin/bash
# gemm_x3 tile variants (gemm_bench 70 + v) for the fp32 FFN up (and q|k|v) at the headline's heights, with the 2-D XCD
# deal on: does the routed tile (-2) stay the best?
set -u
out=gpurun_out/${1:-x3rs}_sweep.jsonl
mkdir -p gpurun_out; : > $out
for M in 2560 1280; do
  ROWSCALE=1 FULLF32=1 NOC2=1 timeout -k 10 120 t-one_amd/gemm_bench $M 384 3072 2 -2,70,71,72,73,74,75,76,77,78 1 200 >> $out || exit 1
  ROWSCALE=1 FULLF32=1 NOC2=1 timeout -k 10 120 t-one_amd/gemm_bench $M 384 1152 0 -2,70,71,72,73,74,75,76,77,78,79,80,81 1 200 >> $out || exit 1
done
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l)
    if 'us' in d: print(d['M'], d['N'], d['variant'], d['us'], d.get('max_rel_err'))
"
