# Round-3 final evidence on the final tree: fp8 FFN-up PMC traffic (the kernel changed), step breakdowns at B = 4096,
# rocprofv3 kernel stats of the headline leg and the default command, the unprofiled default bench, the GPU suite.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/pmc_traffic.sh fp8 4096 || exit $?
python scripts/traffic_summary.py gpurun_out/pmc_fp8 fp8 4096 > gpurun_out/r03_traffic_fp8_b4096.json || exit $?
rm -rf gpurun_out/pmc_fp8
bash scripts/step_breakdown.sh bf16_b4096 --precision bf16 --batch 4096 || exit $?
bash scripts/step_breakdown.sh fp8_b4096 --precision fp8 --batch 4096 || exit $?
echo breakdowns done
bash scripts/prof_headline.sh || exit $?
rm -rf /tmp/prof_def
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_def -o run --output-format csv -- python bench.py > gpurun_out/prof_def.log 2>&1 || exit $?
mkdir -p gpurun_out/prof_def
find /tmp/prof_def -name '*kernel_stats.csv' -exec cp {} gpurun_out/prof_def/ \;
echo profiles done
timeout -k 10 600 python -u bench.py > gpurun_out/r03_final_bench.log 2>&1 || exit $?
echo bench done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_final_gpu.log 2>&1
echo "suite rc=$?"
