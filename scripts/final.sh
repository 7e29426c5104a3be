# Round-end validation: smoke, GPU parity suite, the default bench line (fp32 B=256 + alt legs, CPU
# baseline) and a rocprofv3 kernel-stats summary of the same default command.  The kernel trace stays in /tmp
# (it exceeds gpurun's 64 MiB copy-back); only the stats CSVs come back under gpurun_out/.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -ne 0 ] && exit $rc; return 0; }
if [ "${TESTS:-1}" = 1 ]; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
fi
step bench_default 600 python bench.py
rm -rf /tmp/prof_default
step prof_default 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_default -o run --output-format csv -- python bench.py --cpu-baseline-s 0
mkdir -p gpurun_out/prof_default
find /tmp/prof_default -name '*stats*.csv' -exec cp {} gpurun_out/prof_default/ \;
ls gpurun_out/prof_default
