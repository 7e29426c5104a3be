#!/bin/bash
# gemm_xw epilogue with the row factor on the exp2 scale and on the SwiGLU product (one multiply per output fewer) vs
# gemm_bench_head; kernel tests for gemm_xw; bf16 B = 4096 per-kernel A/B against libtonehip_prev.so (= HEAD)
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_xw_cz.jsonl
: > $out
for rep in 1 2; do
  for bin in gemm_bench_head gemm_bench; do
    for shape in "40960 384 3072 2" "20480 384 3072 2" "40960 384 768 3"; do
      ROWSCALE=1 timeout -k 10 120 ./t-one_amd/$bin $shape -300 1 20 | sed "s/}\$/, \"bin\": \"$bin\"}/" >> $out || exit $?
    done
  done
done
cat $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "xw or bf16_routes" --timeout 300 --timeout-method thread > gpurun_out/r05_xw_cz_tests.log 2>&1 || { tail -20 gpurun_out/r05_xw_cz_tests.log; exit 1; }
tail -1 gpurun_out/r05_xw_cz_tests.log
bash scripts/r05_step_ab.sh xwcz_bf16_b4096 --precision bf16 --batch 4096
