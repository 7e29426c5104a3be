#!/bin/bash
# gemm_rp: the fused norm (NORMW=1) and the bf16 shadow (NOC2=1) priced in the microbenchmark, M = 40960 / 20480.
set -u
mkdir -p gpurun_out
out=gpurun_out/r05_rp_norm.jsonl
: > $out
for MK in "40960 1536" "40960 384" "20480 1536"; do
  set -- $MK
  RES16=1 timeout -k 10 60 ./t-one_amd/gemm_bench $1 $2 384 1 90,90,90 1 50 | sed 's/}$/, "case": "plain"}/' >> $out || exit $?
  NORMW=1 RES16=1 timeout -k 10 60 ./t-one_amd/gemm_bench $1 $2 384 1 90,90,90 1 50 | sed 's/}$/, "case": "norm"}/' >> $out || exit $?
  NOC2=1 RES16=1 timeout -k 10 60 ./t-one_amd/gemm_bench $1 $2 384 1 90,90,90 1 50 | sed 's/}$/, "case": "noc2"}/' >> $out || exit $?
done
cat $out
