# gemm_xs / gemm_xs8 vs the current routes over the encoder's M range (B = 256 .. 4096 at 10 and 5 frames).
set -u
mkdir -p gpurun_out
B=t-one_amd/gemm_bench
out=gpurun_out/r03_xs_route_sweep.jsonl
: > $out
sw() { timeout -k 5 90 "$@" >> $out 2>&1; local rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: $*"; exit $rc; fi; }
for M in 2560 5120 10240 20480 40960; do
  sw env ROWSCALE=1 $B $M 384 3072 2 -1,-10,-14,-18,-22,-26,-34 1 20
  sw env ROWSCALE=1 $B $M 384 768 3 -1,-10,-12,-14,-16,-22 1 20
  for nc in 0 8 12 16; do sw env ROWSCALE=1 XSNC=$nc $B $M 384 3072 2 98 1 20; done
  sw env ROWSCALE=1 $B $M 384 3072 2 99 1 20
done
echo done
