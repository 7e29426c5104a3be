# gemm_rows (full-row RESID, N = 384) vs the routed RESID kernels: FFN down (K = 1536) and attn-out / pw2 (K = 384).
set -u
mkdir -p gpurun_out
B=t-one_amd/gemm_bench
out=gpurun_out/r03_rows_sweep.jsonl
: > $out
sw() { timeout -k 5 90 "$@" >> $out 2>&1; local rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: $*"; exit $rc; fi; }
for M in 40960 20480 10240 5120 2560; do
  for K in 1536 384; do
    sw $B $M $K 384 1 -1 1 20
    for mb in 0 2 3 4 5 6 8; do echo "mb=$mb" >> $out; sw env RWMB=$mb $B $M $K 384 1 -5 1 20; done
  done
done
echo done
