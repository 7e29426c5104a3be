#!/bin/bash
# fp32 routing check: fp32 / 400 ms GPU parity tests, then the headline and 400 ms legs (short bench).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-fp32}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_400ms.py -x -v --timeout 300 --timeout-method thread \
  -k "not bf16 and not fp8 and not lowprec and not large" > gpurun_out/r05_${tag}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05_${tag}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 200 --config4 0 --config5 0 --cpu-baseline-s 0 --detail gpurun_out/r05_${tag}_detail.json > gpurun_out/r05_${tag}_bench.json 2> gpurun_out/r05_${tag}_bench.err || exit $?
python3 -c "
import json; d=json.loads(open('gpurun_out/r05_${tag}_bench.json').read().splitlines()[-1])
print('headline', d['value'], d['ms_per_step'], d['roofline']['frac'])
for a in d['alt_workloads']: print(a['workload'], a['value'], a['ms_per_step'])
print(d['latency_b1'])"
