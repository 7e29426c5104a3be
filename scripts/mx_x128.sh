# MXFP8 STORE / RESID GEMMs with 256- vs 128-row X tiles (MXDBG 16 / 32; 0 = the launcher's choice)
set -u
mkdir -p gpurun_out
out=gpurun_out/mx_x128.jsonl
: > $out
B=./t-one_amd/gemm_bench
for pass in 1 2; do
for M in 2560 5120 10240 20480 40960; do
  for D in 16 32; do
    echo "# M=$M K=1536 RESID MXDBG=$D" >> $out
    MXDBG=$D timeout -k 10 60 $B $M 1536 384 1 99 1 20 >> $out 2>&1 || echo "fail $M $D"
    echo "# M=$M K=384 N=1152 STORE rowscale MXDBG=$D" >> $out
    MXDBG=$D ROWSCALE=1 timeout -k 10 60 $B $M 384 1152 0 99 1 20 >> $out 2>&1 || echo "fail $M $D"
  done
done
done
cat $out
