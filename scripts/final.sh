# Round-end validation: smoke, GPU parity suite, the default bench line (fp32 B=256 + bf16 B=2048 alt,
# CPU baseline) and a rocprofv3 kernel-stats summary of the same default command.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -ne 0 ] && exit $rc; return 0; }
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_default 400 python bench.py
rm -rf gpurun_out/prof_default
step prof_default 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run --output-format csv -- python bench.py --cpu-baseline-s 0
