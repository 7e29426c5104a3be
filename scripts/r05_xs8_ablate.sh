#!/bin/bash
# gemm_xs8 (fp8 FFN up, M = 40960) skeleton ablations, timing only (XS8_ABLATE DBG bits: 1 no epilogue, 2 no MFMA,
# 4 no DMA after the prologue, 16 no barrier, 256 no W fragment reads, 512 no X loads)
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_xs8_ablate.jsonl
: > $out
for rep in 1 2; do
  for d in 0 1 3 7 19 259 515 771 263; do
    NOREF=1 ROWSCALE=1 MXDBG=$d timeout -k 10 60 ./t-one_amd/gemm_bench_ablate 40960 384 3072 2 98 1 20 | sed "s/}\$/, \"dbg\": $d}/" >> $out || exit $?
  done
done
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('$out'):
    d=json.loads(l); r[d['dbg']].append(d['us'])
for k,v in r.items(): print(k, v)"
