# dwconv ablations (tools/dwconv_bench.hip dw_ablate_kernel) -> gpurun_out/r04_dwconv_ablate.jsonl
set -u
mkdir -p gpurun_out
out=gpurun_out/r04_dwconv_ablate.jsonl
: > $out
for cfg in "4096 10 1" "4096 5 1" "256 10 0"; do
  timeout -k 10 120 ./t-one_amd/dwconv_bench $cfg 50 >> $out || exit $?
done
grep -v check $out
