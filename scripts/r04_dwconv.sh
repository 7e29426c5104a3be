# dwconv state-stream microbenchmark (tools/dwconv_bench.hip) -> gpurun_out/r04_dwconv.jsonl
set -u
mkdir -p gpurun_out
out=gpurun_out/r04_dwconv.jsonl
: > $out
for cfg in "4096 10 1" "4096 5 1" "256 10 0" "256 5 0" "2048 10 1" "1 10 0" "1 10 1"; do
  timeout -k 10 120 ./t-one_amd/dwconv_bench $cfg 50 >> $out || exit $?
done
cat $out
