#!/bin/bash
# resident vs flat state: dwconv launch times (kernel_check), one profiled bf16 B = 4096 step per form, and the fp32
# B = 256 headline leg per form (unprofiled, no other legs).  Tag: gpurun_out/<tag>_*
set -u
tag=${1:-ringab}
mkdir -p gpurun_out
for c in dwconv_bf16 dwconv_ring_bf16; do for T in 10 5; do timeout -k 10 120 t-one_amd/kernel_check $c 4096 $T || exit 1; done; done > gpurun_out/${tag}_dw_times.jsonl
for c in dwconv dwconv_ring; do for T in 10 5; do timeout -k 10 120 t-one_amd/kernel_check $c 256 $T || exit 1; done; done >> gpurun_out/${tag}_dw_times.jsonl
cat gpurun_out/${tag}_dw_times.jsonl | cut -c1-160
bash scripts/step_breakdown.sh ${tag}_flat_bf16_b4096 --precision bf16 --batch 4096 --state flat || exit 1
bash scripts/step_breakdown.sh ${tag}_ring_bf16_b4096 --precision bf16 --batch 4096 --state ring || exit 1
for v in flat ring; do echo "== $v"; grep -E "dwconv|kv_assemble|mel_prep" gpurun_out/step_${tag}_${v}_bf16_b4096.txt; tail -1 gpurun_out/step_${tag}_${v}_bf16_b4096.txt; done
for st in flat ring; do
  timeout -k 10 300 python bench.py --steps 200 --cpu-baseline-s 0 --alt 0 --config4 0 --config5 0 --state $st > gpurun_out/${tag}_headline_$st.json 2>gpurun_out/${tag}_headline_$st.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_headline_$st.json').read().splitlines()[-1]); print('$st', d['value'], d['ms_per_step'])"
done
