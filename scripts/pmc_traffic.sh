# HBM traffic of the dominant kernel family (FFN up-projection, the only SWIGLU GEMM) from separate
# rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md HBM section), eager launches.
# Usage: bash scripts/pmc_traffic.sh <fp32|bf16> <batch>   -> gpurun_out/pmc_<prec>/{fetch,write}/
set -u
prec=$1; B=$2
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  d=gpurun_out/pmc_${prec}/$(echo $c | tr A-Z a-z | cut -d_ -f1)
  rm -rf $d
  timeout -s KILL 240 rocprofv3 --pmc $c -d $d -o run --output-format csv -- python bench.py --precision $prec --batch $B --steps 2 --warmup 1 --no-graph --cpu-baseline-s 0 --alt 0 --config4 0 --config5 0 > gpurun_out/pmc_${prec}_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
