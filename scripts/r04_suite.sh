# GPU test suite, then the driver's default bench on the current tree (tag arg)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-cur}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_gpu_$tag.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -5 gpurun_out/r04_gpu_$tag.log; [ $rc -ne 0 ] && exit $rc
bash scripts/r04_bench.sh $tag
