#!/bin/bash
# gemm_d3n (wide direct-load fp32 split with the folded-norm row factor) on the rowscale projections of the fp32 step
# (FFN up SwiGLU, pw1 GLU, q|k|v STORE), A fragment-packed (PACKX=1), against gemm_x3
set -u
out=gpurun_out/${1:-d3n}_sweep.jsonl
mkdir -p gpurun_out; : > $out
V=-2,-602,-603
for M in 2560 1280; do
  for NE in "3072 2" "768 3" "1152 0"; do
    set -- $NE
    PACKX=1 FULLF32=1 NOC2=1 ROWSCALE=1 timeout -k 10 120 t-one_amd/gemm_bench $M 384 $1 $2 $V 1 100 >> $out || { echo "fail M=$M N=$1"; exit 1; }
  done
done
python3 - $out <<'PY'
import json,sys
from collections import defaultdict
g=defaultdict(dict)
for l in open(sys.argv[1]):
    if not l.startswith('{'): continue
    r=json.loads(l)
    if 'error' in r: continue
    g[(r['M'],r['N'],r['epi'])][r['variant']]=(r['us'],r['max_rel_err'])
for k in g: print(k, ' '.join(f"{v}:{u[0]:.1f}/{u[1]:.1e}" for v,u in sorted(g[k].items(), reverse=True)))
PY
