# fp8 FFN down (gemm_mx RESID, K = 1536): X row pitch K + LDAPAD bytes (1536 B = 12 x 128 B lines puts a
# K-tile's 256 rows on few L2 channels if they interleave at 128 B); full kernel and K loop only (MXDBG 5)
set -u
mkdir -p gpurun_out
O=gpurun_out/r03_mx_ldapad.jsonl
: > $O
for r in 1 2; do
for M in 40960 20480; do
  for p in 0 128 256 64; do
    for d in 0 5; do
      echo "M=$M LDAPAD=$p MXDBG=$d" >> $O
      LDAPAD=$p MXDBG=$d timeout -k 5 90 t-one_amd/gemm_bench_ablate $M 1536 384 1 99 1 50 >> $O 2>&1 || exit $?
    done
  done
done
done
echo done
# E = QPT default vs the previous commit on the other gemm_mx routes (q|k|v STORE, small-M FFN up)
O2=gpurun_out/r03_mx_e_other.jsonl
: > $O2
for r in 1 2; do
  for b in gemm_bench_old gemm_bench; do
    echo "$b qkv M=40960" >> $O2; timeout -k 5 90 env ROWSCALE=1 t-one_amd/$b 40960 384 1152 0 99 1 50 >> $O2 2>&1 || exit $?
    echo "$b qkv M=10240" >> $O2; timeout -k 5 90 env ROWSCALE=1 t-one_amd/$b 10240 384 1152 0 99 1 50 >> $O2 2>&1 || exit $?
    echo "$b up M=2560" >> $O2; timeout -k 5 90 env ROWSCALE=1 t-one_amd/$b 2560 384 3072 2 99 1 50 >> $O2 2>&1 || exit $?
    echo "$b down M=40960" >> $O2; timeout -k 5 90 t-one_amd/$b 40960 1536 384 1 99 1 50 >> $O2 2>&1 || exit $?
    echo "$b down M=5120" >> $O2; timeout -k 5 90 t-one_amd/$b 5120 1536 384 1 99 1 50 >> $O2 2>&1 || exit $?
  done
done
echo done2
