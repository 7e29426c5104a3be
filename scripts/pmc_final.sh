# Final-tree PMC traffic of the dominant kernel (FFN up) for the bench's roofline: fp32 B=256, bf16 B=2048 / 4096
set -u
for pb in "fp32 256" "bf16 2048" "bf16 4096"; do
  set -- $pb
  bash scripts/pmc_traffic.sh $1 $2 || exit $?
  python scripts/traffic_summary.py gpurun_out/pmc_$1 $1 $2 > gpurun_out/r02_traffic_$1_b$2.json || exit 1
  rm -rf gpurun_out/pmc_$1
  cat gpurun_out/r02_traffic_$1_b$2.json
done
