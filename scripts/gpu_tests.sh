#!/bin/bash
# the GPU suite and smoke() on the current tree.  Tag: gpurun_out/<tag>_*
set -u
mkdir -p gpurun_out
tag=${1:-mid}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 gpurun_out/${tag}_gpu_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/${tag}_gpu_tests.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -5 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
