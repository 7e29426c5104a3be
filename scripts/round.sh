# GPU iteration: parity tests, fp32 B=256 and bf16 B=2048 bench lines, a bf16 kernel trace.
# Each GPU step has its own time limit; any failure ends the script.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
if [ "${TESTS:-1}" = 1 ]; then
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
fi
step bench_fp32 300 python bench.py --cpu-baseline-s 0 --alt 0
step bench_bf16 300 python bench.py --precision bf16 --batch 2048 --cpu-baseline-s 0 --alt 0
if [ "${TRACE32:-0}" = 1 ]; then
  rm -rf gpurun_out/trace_fp32
  step trace_fp32 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_fp32 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-baseline-s 0 --alt 0
fi
if [ "${TRACE:-1}" = 1 ]; then
  rm -rf gpurun_out/trace_bf16
  step trace_bf16 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_bf16 -o run --output-format csv -- python bench.py --precision bf16 --batch 2048 --steps 3 --warmup 1 --cpu-baseline-s 0 --alt 0
fi
