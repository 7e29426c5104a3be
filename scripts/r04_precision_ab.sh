# bf16 / fp8 error against the fp32 oracle (scripts/bf16_measure.py: B = 2048, 10 staggered chunks, 64 sampled streams)
# for two library builds: TONEHIP_LIB=t-one_amd/libtonehip_base.so (fp32 residual stream) vs the tree's (fp16)
# -> gpurun_out/r04_precision_ab.jsonl
set -u
out=gpurun_out/r04_precision_ab.jsonl
mkdir -p gpurun_out
: > $out
for prec in fp8 bf16; do
  for lib in base cur; do
    if [ $lib = base ]; then export TONEHIP_LIB=t-one_amd/libtonehip_base.so; else unset TONEHIP_LIB; fi
    PREC=$prec timeout -k 10 400 python scripts/bf16_measure.py > gpurun_out/pm.json 2> gpurun_out/pm.err || { tail -5 gpurun_out/pm.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/pm.json'))
r=d['stagger']
print(json.dumps({'prec': '$prec', 'lib': '$lib', 'max': max(x['max'] for x in r), 'p99': max(x['p99'] for x in r),
  'argmax_min': min(x['argmax_agree'] for x in r), 'argmax_mean': sum(x['argmax_agree'] for x in r)/len(r),
  'example': d['example_audio']['$prec']['frame_token_agree'], 'phrases_identical': d['example_audio']['$prec']['phrases_identical']}))" >> $out
    tail -1 $out
  done
done
unset TONEHIP_LIB
