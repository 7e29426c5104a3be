# A/B of two library builds on the B = 1 fp32 device step (the drop-in's per-call batch):
# TONEHIP_LIB=t-one_amd/libtonehip_base.so (A) vs the tree's libtonehip.so (B), alternating, one bench process per
# leg -> gpurun_out/r04_b1_ab_<tag>.jsonl; then a one-step kernel breakdown of the tree's build
set -u
tag=${1:-b1}
out=gpurun_out/r04_b1_ab_$tag.jsonl
mkdir -p gpurun_out
: > $out
for rep in 1 2 3; do
  for lib in base cur; do
    if [ $lib = base ]; then export TONEHIP_LIB=t-one_amd/libtonehip_base.so; else unset TONEHIP_LIB; fi
    timeout -k 10 180 python bench.py --precision fp32 --batch 1 --steps 1000 --warmup 20 --alt 0 --config4 0 --config5 0 \
      --cpu-baseline-s 0 > gpurun_out/b1_leg.json 2> gpurun_out/b1_leg.err || { tail -5 gpurun_out/b1_leg.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/b1_leg.json'))
print(json.dumps({'lib': '$lib', 'rep': $rep, 'ms_per_step': d['ms_per_step'], 'median_ms': d.get('median_ms'), 'p99_ms': d.get('p99_ms')}))" >> $out
    tail -1 $out
  done
done
unset TONEHIP_LIB
bash scripts/step_breakdown.sh ${tag}_fp32_b1 --batch 1
