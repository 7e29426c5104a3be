# GPU round check: smoke, GPU parity tests, a short bench, a rocprofv3 kernel-trace profile.
# Every GPU step has its own time limit; a crash/timeout (rc > 1) ends the script.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"
  if [ $rc -gt 1 ]; then exit $rc; fi
}
run smoke 300 python __graft_entry__.py smoke
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rA
run bench 300 python bench.py --steps 20 --warmup 3 --cpu-baseline-s 10
if [ "${PROFILE:-1}" = 1 ]; then
  run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --cpu-baseline-s 0
fi
