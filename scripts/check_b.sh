# GPU parity suite + bench lines at the batches the routing touches (fp32 256, bf16 2048 / 512)
set -u
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-200
  [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_fp32 200 python bench.py --cpu-baseline-s 0 --alt 0
step bench_bf16 200 python bench.py --precision bf16 --batch 2048 --cpu-baseline-s 0 --alt 0
step bench_bf16_512 200 python bench.py --precision bf16 --batch 512 --cpu-baseline-s 0 --alt 0
for f in bench_fp32 bench_bf16 bench_bf16_512; do grep '^{' gpurun_out/$f.log | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f', d['value'], d['ms_per_step'])"; done
