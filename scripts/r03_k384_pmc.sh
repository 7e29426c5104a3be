# SQ counters of the routed K = 384 FFN-up kernels at M = 40960: gemm_xs (bf16), gemm_xs8 (MXFP8), each full and
# without MFMAs (DBG 2)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
A=t-one_amd/gemm_bench_ablate
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
for v in "xs 0" "xs 2" "xs8 0" "xs8 2"; do
  set -- $v
  d=gpurun_out/k384_pmc_$1_$2
  rm -rf $d
  if [ $1 = xs ]; then
    ROWSCALE=1 XSDBG=$2 timeout -s KILL 60 rocprofv3 --pmc $C -d $d -o run --output-format csv -- $A 40960 384 3072 2 -10 1 5 > $d.log 2>&1 || exit $?
  else
    ROWSCALE=1 MXDBG=$2 timeout -s KILL 60 rocprofv3 --pmc $C -d $d -o run --output-format csv -- $A 40960 384 3072 2 98 1 5 > $d.log 2>&1 || exit $?
  fi
  echo "$v ok"
done
