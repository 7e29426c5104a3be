#!/bin/bash
# the drop-in at B = 1: its GPU tests, then bench.dropin_latency_b1 (pinned staging + graph replay)
set -u
mkdir -p gpurun_out
tag=${1:-b1}
timeout -k 10 600 python -u -m pytest tests/test_pipeline_dropin.py tests/test_gpu_parity.py -m gpu -v -k "dropin or forward or model or pipeline" --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${tag}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "
import json, bench
print(json.dumps(bench.dropin_latency_b1(0)))" > gpurun_out/${tag}_latency.json 2>&1 || { tail -5 gpurun_out/${tag}_latency.json; exit 1; }
cat gpurun_out/${tag}_latency.json
