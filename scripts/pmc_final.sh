# Final-tree PMC traffic of the dominant kernel (FFN up) for the bench's roofline (default: bf16 B=2048 / 4096;
# args: "prec batch" pairs)
set -u
pairs=("$@"); [ ${#pairs[@]} -eq 0 ] && pairs=("bf16 2048" "bf16 4096")
for pb in "${pairs[@]}"; do
  set -- $pb
  bash scripts/pmc_traffic.sh $1 $2 || exit $?
  python scripts/traffic_summary.py gpurun_out/pmc_$1 $1 $2 > gpurun_out/r02_traffic_$1_b$2.json || exit 1
  rm -rf gpurun_out/pmc_$1
  cat gpurun_out/r02_traffic_$1_b$2.json
done
