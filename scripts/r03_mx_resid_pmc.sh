# fp8 FFN down (gemm_mx RESID, M = 40960, K = 1536, N = 384): HBM fetch / write and L2 hit / miss per launch,
# full kernel (MXDBG 0) and K loop only (MXDBG 5); one counter group per rocprofv3 pass
set -u
mkdir -p gpurun_out/mxpmc
export TMPDIR=/tmp
for d in 0 5; do
  for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    n=$(echo $c | cut -d' ' -f1 | tr A-Z a-z)
    export MXDBG=$d
    timeout -s KILL 60 rocprofv3 --pmc $c -d gpurun_out/mxpmc/d${d}_$n -o run --output-format csv -- t-one_amd/gemm_bench_ablate 40960 1536 384 1 99 1 5 > gpurun_out/mxpmc/d${d}_$n.log 2>&1
    rc=$?; echo "pmc d=$d $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
