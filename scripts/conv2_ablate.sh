#!/bin/bash
# conv2_x3 ablations at B = 256 (TONE_CONV2_DBG: 1 taps not re-staged, 2 no split, 4 no MFMA), one
# graph-replayed bench run each under a rocprofv3 kernel trace; prints the conv2 kernel's mean duration
set -eu
export TMPDIR=/tmp
mkdir -p gpurun_out
for D in 0 1 2 3 4 5 7; do
  rm -rf /tmp/c2_$D
  TONE_CONV2_DBG=$D timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d /tmp/c2_$D -o run -- \
    python bench.py --steps 5 --warmup 2 --cpu-baseline-s 0 --alt 0 --config4 0 --config5 0 > gpurun_out/c2_$D.log 2>&1
  python - "$D" "$(find /tmp/c2_$D -name '*kernel_trace.csv' | head -1)" <<'PY'
import csv, sys
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in csv.DictReader(open(sys.argv[2])) if "conv2_x3" in r["Kernel_Name"]]
print(f"dbg {sys.argv[1]}: conv2_x3 {sum(d) / len(d):.1f} us over {len(d)} launches")
PY
done
