#!/bin/bash
# gemm_rp with the read-ahead ring: sweep + ablations + low-precision parity tests + bf16 B = 4096 step sequence.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-ra}
out=gpurun_out/r05_rp_${tag}.jsonl
: > $out
for MK in "40960 1536" "20480 1536" "40960 384" "20480 384" "10240 1536" "10240 384"; do
  set -- $MK
  RES16=1 timeout -k 10 120 ./t-one_amd/gemm_bench $1 $2 384 1 14,90,93,94,95,96 1 30 >> $out || exit $?
done
for MK in ${ABL:-}; do
  set -- $MK
  for dbg in 0 1 4 8 9 24 32; do
    vv=$((dbg * 400 + 90))
    RES16=1 timeout -k 10 120 ./t-one_amd/gemm_bench_ablate $1 $2 384 1 $vv 1 30 | sed "s/}\$/, \"dbg\": $dbg}/" >> $out || exit $?
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "bf16 or fp8 or large or ragged or lowprec or stagewise" > gpurun_out/r05_rp_${tag}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05_rp_${tag}_tests.log; [ $rc -ne 0 ] && exit $rc
SEQ=seq bash scripts/step_breakdown.sh bf16_b4096_${tag} --precision bf16 --batch 4096 || exit $?
head -12 gpurun_out/step_bf16_b4096_${tag}.txt
[ -n "${FP32:-}" ] && { SEQ=seq bash scripts/step_breakdown.sh fp32_b256_${tag} || exit $?; }
echo done
