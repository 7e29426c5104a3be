set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --precision bf16 --batch 2048 --cpu-baseline-s 0 --alt 0 > gpurun_out/bench_bf16.log 2>&1 || exit 1
tail -1 gpurun_out/bench_bf16.log | cut -c1-400
