# gemm_xs (bf16 FFN up, M = 40960) after the ring-wait change: full, no epilogue, no W reads, no MFMA
set -u
mkdir -p gpurun_out
O=gpurun_out/r03_xs_ablate2.jsonl
: > $O
A=t-one_amd/gemm_bench_ablate
for d in 0 1 16 2 17 3; do echo "xs dbg=$d" >> $O; timeout -k 5 90 env ROWSCALE=1 XSDBG=$d $A 40960 384 3072 2 -10 1 20 >> $O 2>&1 || exit $?; done
echo done
