# PMC traffic (FETCH_SIZE / WRITE_SIZE passes) of the FFN-up and RESID families for every bench precision / batch
# -> profiles-ready JSON in gpurun_out/r04_traffic_<prec>_b<B>.json (copied to profiles/ by hand)
set -u
export TMPDIR=/tmp
for pb in "fp32 256" "bf16 2048" "bf16 4096" "fp8 4096"; do
  set -- $pb
  bash scripts/pmc_traffic.sh $1 $2 || exit $?
  rm -rf gpurun_out/pmc_$1_b$2 && cp -r gpurun_out/pmc_$1 gpurun_out/pmc_$1_b$2
  python3 scripts/traffic_summary.py gpurun_out/pmc_$1 $1 $2 > gpurun_out/r04_traffic_$1_b$2.json || exit $?
  cat gpurun_out/r04_traffic_$1_b$2.json
done
