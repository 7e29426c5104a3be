# Round-3 GPU check: the bf16 K = 384 GEMM sweep (gemm_t vs gemm_t4 vs gemm_xs), then smoke and the GPU suite.
# Every GPU step has its own time limit; a crash / timeout (rc > 1) ends the script.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"
  if [ $rc -gt 1 ]; then exit $rc; fi
}
if [ "${SWEEP:-1}" = 1 ]; then
  B=t-one_amd/gemm_bench
  sw() { timeout -k 5 90 "$@" >> gpurun_out/r03_sweep.jsonl 2>&1; local rc=$?; if [ $rc -gt 1 ]; then echo "sweep rc=$rc: $*"; exit $rc; fi; }
  : > gpurun_out/r03_sweep.jsonl
  sw env ROWSCALE=1 $B 40960 384 3072 2 20,26,27,-10,-18,-22,-26 1 20
  sw env ROWSCALE=1 $B 20480 384 3072 2 20,22,26,-10,-18,-26 1 20
  sw env ROWSCALE=1 $B 40960 384 768 3 25,-10,-14,-16 1 20
  sw env ROWSCALE=1 $B 20480 384 1152 0 14,-10 1 20
  sw $B 40960 1536 384 1 14,28,29 1 20
  echo "sweep done"
fi
if [ "${BENCH:-0}" = 1 ]; then
  run r03_bench 600 python -u bench.py --cpu-baseline-s 2
fi
if [ "${SUITE:-1}" = 1 ]; then
  run r03_smoke 300 python __graft_entry__.py smoke
  run r03_gpu_all 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread
fi
