# Round-4 evidence on the current tree: the GPU suite, smoke(), the unprofiled default bench, rocprofv3 kernel stats
# of the headline leg and of the default command, one-step breakdowns at B = 4096 (bf16 / fp8) and B = 1 (fp32).
# Tag argument: output names gpurun_out/r04_<tag>_*.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-final}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04_${tag}_gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 gpurun_out/r04_${tag}_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_${tag}_smoke.log 2>&1 || { tail -5 gpurun_out/r04_${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/r04_${tag}_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r04_${tag}_bench.json 2> gpurun_out/r04_${tag}_bench.err || exit $?
echo bench done
bash scripts/prof_headline.sh || exit $?
rm -rf /tmp/prof_def
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_def -o run --output-format csv -- python bench.py > gpurun_out/prof_def.log 2>&1 || exit $?
mkdir -p gpurun_out/prof_def
find /tmp/prof_def -name '*kernel_stats.csv' -exec cp {} gpurun_out/prof_def/ \;
echo profiles done
bash scripts/step_breakdown.sh bf16_b4096 --precision bf16 --batch 4096 || exit $?
bash scripts/step_breakdown.sh fp8_b4096 --precision fp8 --batch 4096 || exit $?
bash scripts/step_breakdown.sh fp32_b1 --batch 1 || exit $?
bash scripts/step_breakdown.sh fp32_b256 || exit $?
echo breakdowns done
