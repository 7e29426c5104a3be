# gemm_xw / gemm_sm microbenchmarks, the GPU suite, and a B = 1 fp32 step breakdown
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/r04_xw_sweep.sh > /dev/null || exit $?
bash scripts/r04_sm_check.sh > /dev/null || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_it1_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r04_it1_gpu.log; [ $rc -ne 0 ] && exit $rc
bash scripts/step_breakdown.sh fp32_b1 --batch 1 || exit $?
cat gpurun_out/r04_xw_sweep.jsonl gpurun_out/r04_sm_check.jsonl | cut -c1-200; cat gpurun_out/step_fp32_b1.txt
