# gemm_xs ablations at FFN-up M=40960 nc=16: 0 full, 1 no epilogue, 2 no MFMA, 4 no DMA, 5, 7.
set -u
mkdir -p gpurun_out
B=t-one_amd/gemm_bench
out=gpurun_out/r03_xs_ablate.jsonl
: > $out
sw() { timeout -k 5 90 "$@" >> $out 2>&1; local rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: $*"; exit $rc; fi; }
for d in ${DBGS:-0 8 1 9 2 7}; do
  echo "dbg=$d" >> $out
  sw env ROWSCALE=1 XSDBG=$d ${B}_ablate 40960 384 3072 2 -26 1 20
done
echo done
