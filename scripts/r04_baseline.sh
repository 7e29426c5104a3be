# Round-4 start: GPU suite + the driver's default bench command on the unchanged round-3 tree.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_base_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r04_base_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r04_base_bench.json 2> gpurun_out/r04_base_bench.err
rc=$?; echo "bench rc=$rc"; exit $rc
