#!/bin/bash
# gemm_xs8 SwiGLU epilogue cost split (XS8_ABLATE DBG bits: 1 no epilogue, 2 no MFMA, 8 no MX quantization,
# 1024 no epilogue stores, 2048 no bias reads), M = 40960, timing only
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_xs8_epi.jsonl
: > $out
for rep in 1 2; do
  for d in 0 1 8 1024 2048 3072 1032 2 1026; do
    NOREF=1 ROWSCALE=1 MXDBG=$d timeout -k 10 60 ./t-one_amd/gemm_bench_ablate 40960 384 3072 2 98 1 20 | sed "s/}\$/, \"dbg\": $d}/" >> $out || exit $?
  done
done
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('$out'):
    d=json.loads(l); r[d['dbg']].append(d['us'])
for k,v in r.items(): print(k, v)"
