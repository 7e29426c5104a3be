# bf16 RESID tile sweep (tools/gemm_bench variants 14 = routed 128x128, 15 = 128x384, 16 = 64x384, 17 = 128x192)
# at the FFN-down / attn-out shapes -> gpurun_out/r04_resid_tiles.jsonl
set -u
mkdir -p gpurun_out
out=gpurun_out/r04_resid_tiles.jsonl
: > $out
for MK in "40960 1536" "20480 1536" "40960 384" "20480 384" "5120 1536"; do
  set -- $MK
  timeout -k 10 120 ./t-one_amd/gemm_bench $1 $2 384 1 -1,14,15,16,17 1 20 >> $out || exit $?
done
cat $out
