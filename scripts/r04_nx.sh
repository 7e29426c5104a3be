# gemm_nx (W-stationary, N split over the XCDs) against the routed bf16 RESID kernel, fp16 residual (RES16=1)
# -> gpurun_out/r04_nx.jsonl
set -u
mkdir -p gpurun_out
out=gpurun_out/r04_nx.jsonl
: > $out
for MK in "40960 1536" "20480 1536" "40960 384" "20480 384" "10240 1536" "5120 1536"; do
  set -- $MK
  RES16=1 timeout -k 10 120 ./t-one_amd/gemm_bench $1 $2 384 1 -1,-400,-1,-400 1 20 >> $out || exit $?
done
cat $out
