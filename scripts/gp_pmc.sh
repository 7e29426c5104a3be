# L2 hit rate / fabric traffic of one gemm_p variant vs gemm_t at the FFN-up shape (M = 20480),
# one rocprofv3 --pmc pass per counter group (MI355X_MICROARCH.md PMC slot limits)
set -u
mkdir -p gpurun_out/gp_pmc
export TMPDIR=/tmp ROWSCALE=1
V=${V:-92}
for grp in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  tag=$(echo $grp | cut -d' ' -f1)
  for v in 20 $V; do
    timeout -s KILL 60 rocprofv3 --pmc $grp -d gpurun_out/gp_pmc/${tag}_$v -o run --output-format csv -- ./t-one_amd/gemm_bench 20480 384 3072 2 $v 1 5 > gpurun_out/gp_pmc/${tag}_$v.log 2>&1
    rc=$?; echo "pmc $tag v$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
