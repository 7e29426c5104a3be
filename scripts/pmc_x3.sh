# SQ counters of the split-fp32 FFN up-projection (gemm_bench variant 53) and the exact-fp32 kernel (-3)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 53 -3; do
  rm -rf gpurun_out/pmc_x3_$v
  ROWSCALE=1 timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_x3_$v -o run --output-format csv -- ./t-one_amd/gemm_bench 2560 384 3072 2 $v 1 5 > gpurun_out/pmc_x3_$v.log 2>&1
  rc=$?; echo "pmc $v rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
