#!/bin/bash
# gemm_rp with the next stage's fragment reads pinned before the step's MFMAs (sched_barrier) vs the previous build
# (t-one_amd/gemm_bench_prev), M = 40960 / 20480, K = 1536 / 384, then the GPU suite and a bf16 B = 4096 per-kernel A/B.
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_rp_sb.jsonl
: > $out
for rep in 1 2; do
  for MK in "40960 1536" "40960 384" "20480 1536" "20480 384"; do
    set -- $MK
    for b in prev cur; do
      exe=./t-one_amd/gemm_bench; [ $b = prev ] && exe=./t-one_amd/gemm_bench_prev
      RES16=1 timeout -k 10 120 $exe $1 $2 384 1 90 1 30 | sed "s/}\$/, \"build\": \"$b\", \"rep\": $rep}/" >> $out || exit $?
    done
  done
  for b in prev cur; do
    exe=./t-one_amd/gemm_bench; [ $b = prev ] && exe=./t-one_amd/gemm_bench_prev
    NORMW=1 RES16=1 timeout -k 10 120 $exe 40960 1536 384 1 90 1 30 | sed "s/}\$/, \"build\": \"$b\", \"norm\": 1, \"rep\": $rep}/" >> $out || exit $?
  done
done
cat $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_rp_sb_tests.log 2>&1 || { tail -30 gpurun_out/r05_rp_sb_tests.log; exit 1; }
tail -2 gpurun_out/r05_rp_sb_tests.log
bash scripts/r05_step_ab.sh rpsb_bf16_b4096 --precision bf16 --batch 4096
