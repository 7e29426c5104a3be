# gemm_ws (W-stationary K = 384) vs the routed kernels at the encoder's large-batch shapes, plus its ablations.
set -u
mkdir -p gpurun_out
B=t-one_amd/gemm_bench
A=t-one_amd/gemm_bench_ablate
O=gpurun_out/r03_ws_sweep.jsonl
: > $O
sw() { timeout -k 5 90 "$@" >> $O 2>&1; local rc=$?; if [ $rc -gt 1 ]; then echo "rc=$rc: $*"; exit $rc; fi; }
sw env ROWSCALE=1 $B 40960 384 3072 2 -10,-26,-200,-201 1 20
sw env ROWSCALE=1 $B 20480 384 3072 2 -10,-200,-201 1 20
sw env ROWSCALE=1 $B 10240 384 3072 2 -1,-200,-201 1 20
sw env ROWSCALE=1 $B 5120 384 3072 2 -1,-200,-201 1 20
sw env ROWSCALE=1 $B 40960 384 768 3 -1,-200,-201 1 20
sw env ROWSCALE=1 $B 20480 384 768 3 -1,-200,-201 1 20
sw env ROWSCALE=1 NOC2=1 $B 40960 384 1152 0 -1,-200,-201 1 20
sw env ROWSCALE=1 NOC2=1 $B 20480 384 1152 0 -1,-200 1 20
for d in 1 2 4 3; do echo "dbg=$d" >> $O; sw env ROWSCALE=1 XSDBG=$d $A 40960 384 3072 2 -200,-201 1 20; done
echo done
