#!/bin/bash
# A/B of two library builds: TONEHIP_LIB=${BASE_LIB:-t-one_amd/libtonehip_base.so} (A, round-5 start by default) vs the tree's
# libtonehip.so (B), alternating, one bench process per leg; LEGS="precision batch [chunk];..."
# -> gpurun_out/r05_ab_<tag>.jsonl
set -u
tag=${1:-ab}
out=gpurun_out/r05_ab_$tag.jsonl
mkdir -p gpurun_out
: > $out
for rep in 1 2; do
  IFS=';' read -ra legs <<< "${LEGS:-fp32 256;bf16 4096;fp8 4096}"
  for leg in "${legs[@]}"; do
    set -- $leg
    for lib in base cur; do
      if [ $lib = base ]; then export TONEHIP_LIB=${BASE_LIB:-t-one_amd/libtonehip_base.so}; else unset TONEHIP_LIB; fi
      timeout -k 10 240 python bench.py --precision $1 --batch $2 --steps ${STEPS:-150} --warmup 3 --alt 0 --config4 0 --config5 0 \
        --chunk-samples ${3:-2400} --cpu-baseline-s 0 --detail gpurun_out/ab_detail.json > gpurun_out/ab_leg.json 2> gpurun_out/ab_leg.err || { tail -5 gpurun_out/ab_leg.err; exit 1; }
      python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_leg.json').read().splitlines()[-1])
print(json.dumps({'lib': '$lib', 'precision': '$1', 'batch': $2, 'chunk': ${3:-2400}, 'rep': $rep, 'ms_per_step': d['ms_per_step'], 'value': d['value']}))" >> $out
      tail -1 $out
    done
  done
done
unset TONEHIP_LIB
