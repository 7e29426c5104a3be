# SQ + GRBM counters of gemm_xw variants at M = 40960 (FFN up): interleaved (64), ping-pong (0), no MFMA (66),
# and gemm_xs (-10); one rocprofv3 --pmc pass per variant.  Output: gpurun_out/xw_pmc_<tag>/
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
A=t-one_amd/gemm_bench_ablate
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
for v in "xw 64" "xw 0" "xw 66" "xs 0"; do
  set -- $v
  d=gpurun_out/xw_pmc_$1_$2
  rm -rf $d
  if [ $1 = xw ]; then V=-300; else V=-10; fi
  ROWSCALE=1 XSDBG=$2 timeout -s KILL 60 rocprofv3 --pmc $C -d $d -o run --output-format csv -- $A 40960 384 3072 2 $V 1 5 > $d.log 2>&1 || exit $?
  echo "$v ok"
done
