# gemm_p variants vs the current bf16 routes at the FFN-up / pw1 shapes, B = 2048 (V: variant list)
set -u
mkdir -p gpurun_out
out=gpurun_out/gp_sweep.log
: > $out
V=${V:-20,24,90,92,94,95}
run() { timeout -k 10 120 ./t-one_amd/gemm_bench "$@" >> $out 2>&1 || { echo "rc=$? on $*"; cat $out; exit 1; }; }
export ROWSCALE=1
for r in 1 2; do
run 20480 384 3072 2 $V 1 50
run 10240 384 3072 2 $V 1 50
run 20480 384 768 3 $V 1 50
done
cat $out
