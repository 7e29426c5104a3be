#!/bin/bash
# fp32 RESID shapes of the 400 ms leg (M = 3328 at T = 13, 1536 at T = 6) and the 300 ms leg (2560 / 1280): the x3 tile
# variants with an nsplit-way K split (partials + splitk_epilogue), against the routed gemm() (-2)
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_x3_splitk.jsonl
: > $out
for MK in "3328 1536" "2560 1536" "1536 1536" "1280 1536" "3328 384"; do
  set -- $MK
  timeout -k 10 120 ./t-one_amd/gemm_bench $1 $2 384 1 -2 1 20 >> $out || exit $?
  for ns in 2 3 4; do
    [ $2 -eq 384 ] && [ $ns -gt 2 ] && continue
    timeout -k 10 120 ./t-one_amd/gemm_bench $1 $2 384 1 50,51,52,56,59,60 $ns 20 >> $out || exit $?
  done
done
python3 - <<'PY'
import json
best = {}
for l in open('gpurun_out/r05_x3_splitk.jsonl'):
    try: d = json.loads(l)
    except ValueError: continue
    if 'us' not in d: continue
    k = (d['M'], d['K'])
    print(k, d['variant'], d['nsplit'], d['us'], d.get('max_rel_err'))
PY
