#!/bin/bash
# Closing evidence on the current tree: the GPU suite, smoke(), the unprofiled default bench, rocprofv3 kernel stats
# of the headline leg.  Tag argument: output names gpurun_out/<tag>_*.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-mid}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 gpurun_out/${tag}_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -5 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 600 python -u bench.py --detail gpurun_out/${tag}_bench_detail.json > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit $?
echo bench done
python3 -c "
import json; d=json.loads(open('gpurun_out/${tag}_bench.json').read().splitlines()[-1])
print('headline', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['encoder_gemm_frac'])
for a in d['alt_workloads']: print(a['workload'], a['value'], a['ms_per_step'], (a['roofline'] or {}).get('encoder_gemm_frac'))
print(d['latency_b1']['device_step_median_ms'], d['latency_b1']['dropin_numpy_median_ms'], len(open('gpurun_out/${tag}_bench.json').read()))"
bash scripts/prof_headline.sh || exit $?
echo profiles done
