# in-step A/B of the FFN up-projection on gemm_pp (TONE_PP=1 + variant) vs gemm_x3, fp32 B=256, plus fp32 parity with pp
set -u
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; grep '^{' "gpurun_out/$name.log" | python3 -c "import sys,json; [print(json.loads(l)['value'], json.loads(l)['ms_per_step']) for l in sys.stdin]"
  [ $rc -ne 0 ] && exit $rc; return 0; }
step x3 200 python bench.py --cpu-baseline-s 0 --alt 0
TONE_PP=1 step pp0 200 python bench.py --cpu-baseline-s 0 --alt 0
TONE_PP=2 step pp1 200 python bench.py --cpu-baseline-s 0 --alt 0
step x3b 200 python bench.py --cpu-baseline-s 0 --alt 0
TONE_PP=1 step parity_pp 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "golden_stream_parity or hip_vs_forward" --timeout 200 --timeout-method thread
