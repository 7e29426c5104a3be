#!/bin/bash
# L2 hit rate (TCC_HIT / (TCC_HIT + TCC_MISS)) and fabric fetch per dispatch for gemm_bench runs.
# Usage: scripts/pmc_hit.sh <tag> <env assignments...> -- <gemm_bench args>
set -eu
export TMPDIR=/tmp
tag=$1; shift
envs=()
while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
for pass in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
  d=/tmp/pmc_${tag}_${pass%% *}
  rm -rf "$d"
  env "${envs[@]}" timeout -s KILL 60 rocprofv3 --pmc $pass --output-format csv -d "$d" -o run -- t-one_amd/gemm_bench "$@" > /dev/null 2>&1
  python3 - "$tag" "$(find "$d" -name '*counter_collection.csv' | head -1)" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[2])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, v in agg.items():
    if "gemm" not in k:
        continue
    n = max(c for (kk, _), c in cnt.items() if kk == k)
    per = {c: x / n for c, x in v.items()}
    s = " ".join(f"{c}={x:.4g}" for c, x in per.items())
    if "TCC_HIT_sum" in per:
        s += f" hit_rate={per['TCC_HIT_sum'] / (per['TCC_HIT_sum'] + per['TCC_MISS_sum']):.3f}"
    print(sys.argv[1], k, "dispatches", n, s)
PY
done
