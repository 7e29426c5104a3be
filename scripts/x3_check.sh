# split-fp32 FFN up-projection after a change: microbench (fp64 reference) + PMC traffic + fp32 bench
set -u
mkdir -p gpurun_out
for M in 2560 1280; do
  ROWSCALE=1 FULLF32=1 timeout -k 10 60 ./t-one_amd/gemm_bench $M 384 3072 2 -3,53,51 1 20 >> gpurun_out/x3_check.jsonl 2>&1 || exit 1
done
cat gpurun_out/x3_check.jsonl
bash scripts/pmc_traffic.sh fp32 256 && python3 scripts/traffic_summary.py gpurun_out/pmc_fp32 fp32 256 > gpurun_out/traffic_fp32.json && cat gpurun_out/traffic_fp32.json
