# Round-3 step breakdowns (rocprofv3 kernel trace) at B = 4096: bf16 and fp8; then the GPU suite.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/step_breakdown.sh bf16_b4096 --precision bf16 --batch 4096 || exit $?
bash scripts/step_breakdown.sh fp8_b4096 --precision fp8 --batch 4096 || exit $?
echo breakdowns done
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_all.log 2>&1
  echo "suite rc=$?"
fi
