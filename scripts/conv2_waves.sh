# conv2_x3 waves per workgroup (TONE_CONV2_WAVES 8 / 4): parity of the pre-encode stage and fp32 B=256 bench
set -u
mkdir -p gpurun_out
for w in 4 8; do
  TONE_CONV2_WAVES=$w timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -k "pre_encode_split or b256" --timeout 120 --timeout-method thread > gpurun_out/c2w_test_$w.log 2>&1 || { tail -5 gpurun_out/c2w_test_$w.log; exit 1; }
  echo "waves=$w $(tail -1 gpurun_out/c2w_test_$w.log)"
  TONE_CONV2_WAVES=$w timeout -k 10 200 python bench.py --cpu-baseline-s 0 --alt 0 > gpurun_out/c2w_bench_$w.log 2>&1 || exit $?
  echo "waves=$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c2w_bench_$w.log)"
done
rm -rf gpurun_out/c2w_trace
TONE_CONV2_WAVES=4 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c2w_trace -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-baseline-s 0 --alt 0 > gpurun_out/c2w_trace.log 2>&1 || exit $?
grep conv2_x3 gpurun_out/c2w_trace/run_kernel_stats.csv
