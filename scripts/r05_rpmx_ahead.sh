#!/bin/bash
# gemm_rp_mx (fp8 RESID) with W fragments two column tiles ahead: microbenchmark vs the previous build
# (gemm_bench_head), GPU suite, fp8 B = 4096 per-kernel A/B against libtonehip_prev.so (= HEAD before the change)
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_rpmx_ahead.jsonl
: > $out
for rep in 1 2; do
  for MK in "40960 1536" "40960 384" "20480 1536" "20480 384"; do
    set -- $MK
    for b in gemm_bench_head gemm_bench; do
      RPMX=1 RES16=1 timeout -k 10 60 ./t-one_amd/$b $1 $2 384 1 99 1 30 | sed "s/}\$/, \"bin\": \"$b\"}/" >> $out || exit $?
    done
  done
done
cat $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_rpmx_ahead_tests.log 2>&1 || { tail -30 gpurun_out/r05_rpmx_ahead_tests.log; exit 1; }
tail -2 gpurun_out/r05_rpmx_ahead_tests.log
bash scripts/r05_step_ab.sh rpmxa_fp8_b4096 --precision fp8 --batch 4096
