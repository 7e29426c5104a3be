#!/bin/bash
# TONE_DW_KO A/B: dwconv_ring in its tap-outer form (sliding frame window, 100 vs 166 VGPRs at T = 10) -- the kernel's
# every-element checks and the ring-vs-flat bit-identity tests with it on, then the bf16 B = 4096 step breakdown and the
# fp32 headline, same box, interleaved.  Measured and NOT kept (no faster: 568-569 vs 568-583 us per bf16 B = 4096 step);
# the KO variant and TONE_DW_KO were removed after this run (profiles/r06_dwko_ab.txt)
set -u
tag=${1:-dwko}
mkdir -p gpurun_out; out=gpurun_out/${tag}_ab.txt; : > $out
TONE_DW_KO=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ring.py -m gpu -q -k "dwconv_ring or ring" --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "ko tests rc=$rc: $(tail -1 gpurun_out/${tag}_tests.log)" | tee -a $out; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for k in 0 1; do
    TONE_DW_KO=$k bash scripts/step_breakdown.sh ${tag}_k${k}_$i --precision bf16 --batch 4096 || exit 1
    echo "ko=$k run $i: $(grep -E 'dwconv_ring' gpurun_out/step_${tag}_k${k}_$i.txt | awk '{s+=$1} END {print s}') us dwconv, $(tail -1 gpurun_out/step_${tag}_k${k}_$i.txt)" | tee -a $out
  done
done
for i in 1 2; do
  for k in 0 1; do
    TONE_DW_KO=$k timeout -k 10 300 python bench.py --steps 60 --warmup 5 --cpu-baseline-s 0 --alt 0 --config4 0 --config5 0 > gpurun_out/${tag}_b.log 2>&1 || { tail -5 gpurun_out/${tag}_b.log; exit 1; }
    tail -1 gpurun_out/${tag}_b.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(json.dumps({'dw_ko': $k, 'fp32_b256_value': r['value'], 'ms_per_step': r['ms_per_step']}))" | tee -a $out
  done
done
