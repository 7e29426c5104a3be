# Ablations of the routed K = 384 FFN-up kernels at M = 40960 (B = 4096): gemm_xs (bf16) and gemm_xs8 (MXFP8)
set -u
mkdir -p gpurun_out
O=gpurun_out/r03_k384_ablate.jsonl
: > $O
A=t-one_amd/gemm_bench_ablate
for d in 0 1 2 4 5 3; do echo "xs dbg=$d" >> $O; timeout -k 5 90 env ROWSCALE=1 XSDBG=$d $A 40960 384 3072 2 -10 1 20 >> $O 2>&1 || exit $?; done
for d in 0 1 2 4 8 5 3; do echo "xs8 dbg=$d" >> $O; timeout -k 5 90 env ROWSCALE=1 MXDBG=$d $A 40960 384 3072 2 98 1 20 >> $O 2>&1 || exit $?; done
echo done
