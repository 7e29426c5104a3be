#!/bin/bash
# one profiled step of the same workload with the previous build (t-one_amd/libtonehip_prev.so) and the tree's build,
# on one box: per-kernel A/B.  Args: tag, bench args...
set -u
tag=$1; shift
TONEHIP_LIB=t-one_amd/libtonehip_prev.so bash scripts/step_breakdown.sh ${tag}_prev "$@" || exit 1
bash scripts/step_breakdown.sh ${tag}_cur "$@" || exit 1
for v in prev cur; do echo "== $v"; head -14 gpurun_out/step_${tag}_$v.txt; tail -1 gpurun_out/step_${tag}_$v.txt; done
