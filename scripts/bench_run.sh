#!/bin/bash
# the unprofiled default bench, then rocprofv3 kernel stats of the headline leg alone.  Tag: gpurun_out/<tag>_*
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-mid}
timeout -k 10 700 python -u bench.py --detail gpurun_out/${tag}_bench_detail.json > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -5 gpurun_out/${tag}_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${tag}_bench.json').read().splitlines()[-1])
print('headline', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['encoder_gemm_frac'])
for a in d['alt_workloads']: print(a['workload'], a['value'], a['ms_per_step'], (a['roofline'] or {}).get('encoder_gemm_frac'))
print(d['latency_b1']['device_step_median_ms'], d['latency_b1']['dropin_numpy_median_ms'], d['cpu_baseline']['value'], len(open('gpurun_out/${tag}_bench.json').read()))"
bash scripts/prof_headline.sh || exit $?
cp -r gpurun_out/prof_head gpurun_out/${tag}_prof_head
echo profiles done
