# PMC passes on the standalone GEMM microbenchmark (no torch in the process).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=${ARGS:-"20480 384 3072 2 0,14 1 3"}
i=0
for pmc in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_LDS"; do
  i=$((i + 1))
  timeout -k 10 180 rocprofv3 --pmc $pmc -d gpurun_out/pmc$i -o run --output-format csv -- ./t-one_amd/gemm_bench $ARGS > gpurun_out/pmc$i.log 2>&1
  rc=$?
  echo "pass $i ($pmc) rc=$rc"
  if [ $rc -gt 1 ]; then exit $rc; fi
done
