# gemm_xw STORE (bf16 out, folded-RMSNorm row factor: the q|k|v shape) vs the LDS-DMA 128x128 kernel (variant 14)
# -> gpurun_out/r04_xw_store.jsonl
set -u
mkdir -p gpurun_out
out=gpurun_out/r04_xw_store.jsonl
: > $out
for MN in "40960 384" "40960 1152" "20480 384" "20480 1152" "10240 384" "10240 1152"; do
  set -- $MN
  CBF=1 NOC2=1 ROWSCALE=1 timeout -k 10 120 ./t-one_amd/gemm_bench $1 384 $2 0 14,-300,14,-300 1 20 >> $out || exit $?
done
cat $out
