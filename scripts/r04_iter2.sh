# GPU suite, fp8 B = 4096 step breakdown, and the default bench on the current tree
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_it2_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r04_it2_gpu.log; [ $rc -ne 0 ] && exit $rc
bash scripts/step_breakdown.sh fp8_b4096 --precision fp8 --batch 4096 || exit $?
head -12 gpurun_out/step_fp8_b4096.txt
bash scripts/r04_bench.sh it2
