# Profiling pass: rocprofv3 kernel-trace stats (and, with PMC=1, separate FETCH_SIZE / WRITE_SIZE passes)
# for one bench configuration.  Usage: bash scripts/profile.sh <tag> [bench args...]
set -u
tag=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"
  if [ $rc -gt 1 ]; then exit $rc; fi
}
run "bench_$tag" 300 python bench.py --cpu-baseline-s 0 --alt 0 "$@"
run "stats_$tag" 400 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_$tag" -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --cpu-baseline-s 0 --alt 0 "$@"
if [ "${PMC:-0}" = 1 ]; then
  run "pmcf_$tag" 400 rocprofv3 --pmc FETCH_SIZE -d "gpurun_out/pmcf_$tag" -o run --output-format csv -- python bench.py --steps 2 --warmup 2 --no-graph --cpu-baseline-s 0 --alt 0 "$@"
  run "pmcw_$tag" 400 rocprofv3 --pmc WRITE_SIZE -d "gpurun_out/pmcw_$tag" -o run --output-format csv -- python bench.py --steps 2 --warmup 2 --no-graph --cpu-baseline-s 0 --alt 0 "$@"
fi
