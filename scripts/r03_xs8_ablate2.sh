# gemm_xs8 at M = 40960: per-tile barrier removed (timing only), static priority, and their combinations
set -u
mkdir -p gpurun_out
O=gpurun_out/r03_xs8_ablate2.jsonl
: > $O
A=t-one_amd/gemm_bench_ablate
for d in 0 256 1; do echo "xs8 dbg=$d" >> $O; timeout -k 5 90 env ROWSCALE=1 MXDBG=$d $A 40960 384 3072 2 98 1 20 >> $O 2>&1 || exit $?; done
echo done
