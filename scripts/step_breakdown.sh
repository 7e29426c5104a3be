#!/bin/bash
# One-step kernel breakdown (rocprofv3 kernel trace, last full step of a short graph-replayed run) for
# the fp32 B = 256 headline and the bf16 B = 2048 config.  Output: gpurun_out/step_<tag>.txt
set -eu
export TMPDIR=/tmp
mkdir -p gpurun_out
prof() {  # tag, bench args...
  local tag=$1; shift
  rm -rf /tmp/st_$tag
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/st_$tag -o run -- \
    python bench.py --steps 5 --warmup 2 --cpu-baseline-s 0 --alt 0 --config4 0 --config5 0 "$@" > gpurun_out/st_$tag.log 2>&1
  python scripts/step_trace.py "$(find /tmp/st_$tag -name '*kernel_trace.csv' | head -1)" ${SEQ:-} > gpurun_out/step_$tag.txt
}
if [ $# -gt 0 ]; then prof "$@"; exit 0; fi   # one custom leg: tag, bench args...
prof fp32_b256
prof bf16_b2048 --precision bf16 --batch 2048
