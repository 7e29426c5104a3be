#!/bin/bash
# fp32 400 ms shapes still on tile rounds of 1.2: attn-out / pw2 (K = 384, N = 384, RESID) and pw1 (GLU, N = 768) at
# M = 3328 (T = 13) and 1536 (T = 6), every x3 tile variant the epilogue allows
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_x3_400.jsonl
: > $out
for rep in 1 2; do
  for M in 3328 1536; do
    timeout -k 10 120 ./t-one_amd/gemm_bench $M 384 384 1 -2,50,51,52,53,54,55,56,57,58,59,61 1 20 >> $out || exit $?
    timeout -k 10 120 ./t-one_amd/gemm_bench $M 384 768 3 -2,51,53,55,56,57,58 1 20 >> $out || exit $?
  done
done
python3 - <<'PY'
import json, collections
r = collections.defaultdict(list)
for l in open('gpurun_out/r05_x3_400.jsonl'):
    try: d = json.loads(l)
    except ValueError: continue
    if 'us' in d: r[(d['M'], d['N'], d['variant'])].append(d['us'])
for k in sorted(r): print(k, r[k])
PY
