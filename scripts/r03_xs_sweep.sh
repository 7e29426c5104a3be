# gemm_xs (bf16) / gemm_xs8 (MXFP8) X-stationary kernels vs the routed kernels at the K = 384 shapes.
set -u
mkdir -p gpurun_out
B=t-one_amd/gemm_bench
out=gpurun_out/r03_xs_sweep.jsonl
: > $out
sw() { timeout -k 5 90 "$@" >> $out 2>&1; local rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: $*"; exit $rc; fi; }
sw env ROWSCALE=1 $B 40960 384 3072 2 20,-18,-26,-42 1 20
sw env ROWSCALE=1 $B 20480 384 3072 2 20,-18,-26 1 20
sw env ROWSCALE=1 $B 40960 384 768 3 25,-14 1 20
for nc in 8 16; do
  sw env ROWSCALE=1 XSNC=$nc $B 40960 384 3072 2 98 1 20
  sw env ROWSCALE=1 XSNC=$nc $B 20480 384 3072 2 98 1 20
done
echo done
