#!/bin/bash
# gemm_xw row-factor forms, each with counted LDS waits: X pre-scaled (gemm_bench_pre) vs accumulators from bias x RMS
# and the factor in the epilogue (gemm_bench), against gemm_bench_prev; GPU suite; bf16 B = 4096 per-kernel A/B
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_xw_rs.jsonl
: > $out
for rep in 1 2; do
  for bin in gemm_bench_prev gemm_bench_pre gemm_bench; do
    for shape in "40960 384 3072 2" "20480 384 3072 2" "40960 384 768 3"; do
      ROWSCALE=1 timeout -k 10 120 ./t-one_amd/$bin $shape -300 1 20 | sed "s/}\$/, \"bin\": \"$bin\"}/" >> $out || exit $?
    done
  done
done
cat $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_xw_rs_tests.log 2>&1 || { tail -30 gpurun_out/r05_xw_rs_tests.log; exit 1; }
tail -2 gpurun_out/r05_xw_rs_tests.log
bash scripts/r05_step_ab.sh xwrs_bf16_b4096 --precision bf16 --batch 4096
