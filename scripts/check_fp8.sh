# fp8 / bf16 parity + bench lines at B = 512 / 2048 / 4096 after the MX tile and GLU routing changes
set -u
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-200
  [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for P in fp8 bf16; do for B in 512 2048 4096; do
  step bench_${P}_$B 200 python bench.py --precision $P --batch $B --cpu-baseline-s 0 --alt 0 --steps 100
done; done
for P in fp8 bf16; do for B in 512 2048 4096; do grep '^{' gpurun_out/bench_${P}_$B.log | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$P $B', d['value'], d['ms_per_step'])"; done; done
