#!/bin/bash
# TONE_RING_NT A/B: dwconv_ring with non-temporal ring accesses, bf16 B = 4096 step breakdown, twice interleaved
set -u
tag=${1:-rnt}
for i in 1 2; do
  for n in 0 1; do
    TONE_RING_NT=$n bash scripts/step_breakdown.sh ${tag}_nt${n}_$i --precision bf16 --batch 4096 || exit 1
    echo "nt=$n run $i: $(grep -E 'dwconv_ring' gpurun_out/step_${tag}_nt${n}_$i.txt | awk '{s+=$1} END {print s}') us dwconv, $(tail -1 gpurun_out/step_${tag}_nt${n}_$i.txt)"
  done
done
