#!/bin/bash
# gemm_rp_mx: barrier between the last K-tile and the epilogue's use of stage slot 0 (odd K-tile counts).
# Errors and times vs gemm_bench_head at the step's shapes, 3 reps; GPU suite; fp8 B = 4096 per-kernel A/B.
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_rpmx_race.jsonl
: > $out
for rep in 1 2 3; do
  for MK in "40960 1536" "40960 384" "20480 1536" "20480 384" "10240 384" "16384 384"; do
    set -- $MK
    for b in gemm_bench_head gemm_bench; do
      RPMX=1 RES16=1 timeout -k 10 60 ./t-one_amd/$b $1 $2 384 1 99 1 30 | sed "s/}\$/, \"bin\": \"$b\"}/" >> $out || exit $?
    done
  done
done
cat $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_rpmx_race_tests.log 2>&1 || { tail -30 gpurun_out/r05_rpmx_race_tests.log; exit 1; }
tail -2 gpurun_out/r05_rpmx_race_tests.log
bash scripts/r05_step_ab.sh rpmxr_fp8_b4096 --precision fp8 --batch 4096
