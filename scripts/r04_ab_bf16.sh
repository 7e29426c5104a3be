# bf16 A/B of two library builds (base = TONEHIP_LIB=t-one_amd/libtonehip_base.so) at B = 4096 and 2048, then the
# bf16 GPU tests on the tree's library -> gpurun_out/r04_ab_bf16.jsonl
set -u
export TMPDIR=/tmp
out=gpurun_out/r04_ab_bf16.jsonl
mkdir -p gpurun_out
: > $out
for rep in 1 2; do
  for b in 4096 2048; do
    for lib in base cur; do
      if [ $lib = base ]; then export TONEHIP_LIB=t-one_amd/libtonehip_base.so; else unset TONEHIP_LIB; fi
      timeout -k 10 240 python bench.py --precision bf16 --batch $b --steps 100 --warmup 3 --alt 0 --config4 0 --config5 0 \
        --cpu-baseline-s 0 > gpurun_out/ab_leg.json 2> gpurun_out/ab_leg.err || { tail -5 gpurun_out/ab_leg.err; exit 1; }
      python3 -c "
import json; d=json.load(open('gpurun_out/ab_leg.json'))
print(json.dumps({'lib': '$lib', 'batch': $b, 'rep': $rep, 'ms_per_step': d['ms_per_step'], 'qkv_us': d['roofline']['families_us_per_step']['gemm_qkv']}))" >> $out
      tail -1 $out
    done
  done
done
unset TONEHIP_LIB
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "bf16 or 400ms or large_batch" --timeout 300 --timeout-method thread > gpurun_out/r04_bf16_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_bf16_tests.log; exit $rc
