# rocprofv3 kernel durations of the gemm_mx FFN-down launch: full kernel and the DBG 31 ablation (no DMA after the
# prologue, no fragment reads, no MFMA, no epilogue), against the HIP-event times of the back-to-back launch loop
set -u
mkdir -p gpurun_out/mxfloor
export TMPDIR=/tmp
for c in 0 31; do
  export MXDBG=$((256 * c))
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/mxfloor_$c -o run --output-format csv -- t-one_amd/gemm_bench_ablate 40960 1536 384 1 99 1 50 > gpurun_out/mxfloor/d$c.log 2>&1 || exit $?
  find /tmp/mxfloor_$c -name '*kernel_stats.csv' -exec cp {} gpurun_out/mxfloor/d${c}_kernel_stats.csv \;
done
echo done
