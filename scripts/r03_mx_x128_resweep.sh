# gemm_mx 256- vs 128-row X tiles (MXDBG 16 / 32) after the side-data fix, FFN down (RESID) and q|k|v (STORE)
set -u
mkdir -p gpurun_out
O=gpurun_out/r03_mx_x128_resweep.jsonl
: > $O
for r in 1 2; do
  for M in 40960 20480 10240 5120; do
    for d in 16 32; do
      echo "down M=$M MXDBG=$d" >> $O; MXDBG=$d timeout -k 5 90 t-one_amd/gemm_bench $M 1536 384 1 99 1 50 >> $O 2>&1 || exit $?
      echo "qkv384 M=$M MXDBG=$d" >> $O; MXDBG=$d ROWSCALE=1 timeout -k 5 90 t-one_amd/gemm_bench $M 384 384 0 99 1 50 >> $O 2>&1 || exit $?
      echo "qkv1152 M=$M MXDBG=$d" >> $O; MXDBG=$d ROWSCALE=1 timeout -k 5 90 t-one_amd/gemm_bench $M 384 1152 0 99 1 50 >> $O 2>&1 || exit $?
    done
  done
done
echo done
