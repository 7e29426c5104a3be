# quick A/B of the routed K = 384 FFN-up kernels at M = 40960 / 20480 (gemm_xs bf16, gemm_xs8 MXFP8)
set -u
mkdir -p gpurun_out
O=gpurun_out/r03_k384_quick.jsonl
: > $O
A=t-one_amd/gemm_bench_ablate
for M in 40960 20480; do
  echo "xs M=$M" >> $O; timeout -k 5 90 env ROWSCALE=1 $A $M 384 3072 2 -10 1 20 >> $O 2>&1 || exit $?
  for d in 0 1; do echo "xs8 M=$M dbg=$d" >> $O; timeout -k 5 90 env ROWSCALE=1 MXDBG=$d $A $M 384 3072 2 98 1 20 >> $O 2>&1 || exit $?; done
done
echo "xs GLU M=40960" >> $O; timeout -k 5 90 env ROWSCALE=1 $A 40960 384 768 3 -10 1 20 >> $O 2>&1 || exit $?
echo done
