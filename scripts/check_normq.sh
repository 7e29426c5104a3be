# fp8 norm-fused MXFP8 quantization: GPU tests (fp8 + the fused-vs-separate check), fp8 bench A/B
# (TONE_FP8_NORMQ=1 default vs 0) at B = 512 / 2048 / 4096, then the final-tree PMC traffic summaries
set -u
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-200
  [ $rc -ne 0 ] && exit $rc; return 0; }
TONE_FP8_NORMQ=1 step pytest_fp8 600 python -u -m pytest tests -m gpu -x -q -k "fp8 or ragged or low_precision" --timeout 300 --timeout-method thread
for B in 512 2048 4096; do for Q in 1 0; do
  TONE_FP8_NORMQ=$Q step bench_fp8_${B}_q$Q 200 python bench.py --precision fp8 --batch $B --cpu-baseline-s 0 --alt 0 --steps 100
done; done
for B in 512 2048 4096; do for Q in 1 0; do grep '^{' gpurun_out/bench_fp8_${B}_q$Q.log | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print('fp8 B=$B normq=$Q', d['value'], d['ms_per_step'])"; done; done
bash scripts/pmc_final.sh
