# fp32 (x3 split) tile / split-K choices at the B = 1 shapes (M = 10 and 5 rows): the drop-in's per-call latency
set -u
mkdir -p gpurun_out
B=t-one_amd/gemm_bench
O=gpurun_out/r03_b1_sweep.jsonl
: > $O
sw() { timeout -k 5 90 "$@" >> $O 2>&1; local rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: $*"; exit $rc; fi; }
for M in 10 5; do
  sw env ROWSCALE=1 NOC2=1 $B $M 384 3072 2 -2,50,53,54,55,56,57 1 50
  sw env ROWSCALE=1 NOC2=1 $B $M 384 768 3 -2,50,51,53,54,55,56 1 50
  for K in 1536 384; do
    sw env NOC2=1 $B $M $K 384 1 -2,50,54,59,60,61 1 50
    for s in 2 4 8; do sw env NOC2=1 $B $M $K 384 1 50,54,59,60 $s 50; done
  done
  sw env NOC2=1 $B $M 384 1152 0 -2,50,54,56,59,60 1 50
  for s in 2 4; do sw env NOC2=1 $B $M 384 1152 0 50,54,60 $s 50; done
done
sw env NOC2=1 $B 10 2176 384 0 -2,50,54,59,60 1 50
for s in 2 4 8; do sw env NOC2=1 $B 10 2176 384 0 50,54,60 $s 50; done
echo done
