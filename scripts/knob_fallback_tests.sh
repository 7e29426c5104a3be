#!/bin/bash
# the documented A/B switches still give passing results: fp32 step tests with gemm_d3 / gemm_d3n and the 2-D XCD deal off, ring tests
# with the ring's non-temporal accesses off, bf16 step tests with the blocked hidden off
set -u
tag=${1:-knobs}
mkdir -p gpurun_out
TONE_D3=0 TONE_D3X=0 TONE_X3_XCD=0 TONE_HEAD_MFMA=0 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_400ms.py tests/test_gpu_ring.py -m gpu -q -k "not bf16 and not fp8 and not lowprec" --timeout 300 --timeout-method thread > gpurun_out/${tag}_d3off.log 2>&1
rc=$?; echo "d3 off rc=$rc: $(tail -1 gpurun_out/${tag}_d3off.log)"; [ $rc -ne 0 ] && exit $rc
TONE_RING_NT=0 TONE_H_BLOCKED=0 timeout -k 10 900 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_parity.py -m gpu -q -k "ring or bf16" --timeout 300 --timeout-method thread > gpurun_out/${tag}_ntoff.log 2>&1
rc=$?; echo "nt / blocked-h off rc=$rc: $(tail -1 gpurun_out/${tag}_ntoff.log)"; exit $rc
