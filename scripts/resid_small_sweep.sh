#!/bin/bash
# bf16 RESID (N = 384, fp16 residual) at the per-GPU batches of config 4 at N = 8 / 4 (B = 512 / 1024): every tile
# family through gemm_bench -- the routed kernel (-1), LDS-DMA tiles (0-9, 14), gemm_f32t on bf16 (32), gemm_rp panels
# (90 auto, 91-98: 16 .. 160 rows)
set -u
mkdir -p gpurun_out
out=gpurun_out/${1:-rs}_resid_small.jsonl
: > $out
for M in 5120 2560 10240; do
  for K in 1536 384; do
    RES16=1 timeout -k 10 120 t-one_amd/gemm_bench $M $K 384 1 -1,0,1,7,8,14,90,91,92,93,94,95 1 30 >> $out || exit 1
  done
done
python3 - $out <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
from collections import defaultdict
best = defaultdict(list)
for r in rows:
    if "us" in r: best[(r["M"], r["K"])].append((r["us"], r["variant"], r["max_rel_err"]))
for k, v in sorted(best.items()):
    v.sort(); routed = [x for x in v if x[1] == -1]
    print(k, "routed", routed[0][:2] if routed else None, "best", v[:3])
PY
