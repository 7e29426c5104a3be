# Output-byte sensitivity of the bf16 RESID shapes (routed kernel, gemm() bf16): RESID (fp32 R + fp32 C + bf16
# shadow, 10 B per output), STORE fp32 + shadow (6), STORE fp32 (4), STORE bf16 (2) -> gpurun_out/r04_resid_bytes.jsonl
set -u
mkdir -p gpurun_out
out=gpurun_out/r04_resid_bytes.jsonl
: > $out
for MK in "40960 1536" "20480 1536" "40960 384" "20480 384"; do
  set -- $MK
  timeout -k 10 120 ./t-one_amd/gemm_bench $1 $2 384 1 -1 1 20 | sed 's/}$/, "case": "resid_f32_c2"}/' >> $out || exit $?
  timeout -k 10 120 ./t-one_amd/gemm_bench $1 $2 384 0 -1 1 20 | sed 's/}$/, "case": "store_f32_c2"}/' >> $out || exit $?
  NOC2=1 timeout -k 10 120 ./t-one_amd/gemm_bench $1 $2 384 0 -1 1 20 | sed 's/}$/, "case": "store_f32"}/' >> $out || exit $?
  CBF=1 NOC2=1 timeout -k 10 120 ./t-one_amd/gemm_bench $1 $2 384 0 -1 1 20 | sed 's/}$/, "case": "store_bf16"}/' >> $out || exit $?
done
cat $out
