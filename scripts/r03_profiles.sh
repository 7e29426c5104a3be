# Round-3 evidence: PMC traffic of the FFN up-projection (fp32 B = 256, bf16 B = 2048 / 4096, fp8 B = 4096),
# rocprofv3 kernel stats of the headline leg and of the default bench command.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "fp32 256" "bf16 2048" "bf16 4096" "fp8 4096"; do
  set -- $cfg
  bash scripts/pmc_traffic.sh $1 $2 || exit $?
  python scripts/traffic_summary.py gpurun_out/pmc_$1 $1 $2 > gpurun_out/r03_traffic_$1_b$2.json || exit $?
  rm -rf gpurun_out/pmc_$1
done
echo traffic done
bash scripts/prof_headline.sh || exit $?
rm -rf /tmp/prof_def
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_def -o run --output-format csv -- python bench.py > gpurun_out/prof_def.log 2>&1 || exit $?
mkdir -p gpurun_out/prof_def
find /tmp/prof_def -name '*kernel_stats.csv' -exec cp {} gpurun_out/prof_def/ \;
echo profiles done
