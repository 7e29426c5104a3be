# gemm_mx persistent grid size (ablation build, MXGRID caps the 256 workgroups): FFN down and q|k|v at M = 40960
set -u
mkdir -p gpurun_out
O=gpurun_out/r03_mx_grid.jsonl
: > $O
python3 -c "import torch; p=torch.cuda.get_device_properties(0); print('cus', p.multi_processor_count)" >> $O 2>&1
for r in 1 2; do
  for g in 256 248 240 224 192 128; do
    echo "down g=$g" >> $O; MXGRID=$g timeout -k 5 90 t-one_amd/gemm_bench_ablate 40960 1536 384 1 99 1 50 >> $O 2>&1 || exit $?
    echo "qkv1152 g=$g" >> $O; MXGRID=$g ROWSCALE=1 timeout -k 5 90 t-one_amd/gemm_bench_ablate 40960 384 1152 0 99 1 50 >> $O 2>&1 || exit $?
  done
done
echo done
# one barrier per K-step instead of two (DBG 128 drops the mid-step one; races, so timing only)
O2=gpurun_out/r03_mx_barrier.jsonl
: > $O2
for r in 1 2; do
  for c in 1 129 31 159; do
    echo "down DBG=$c" >> $O2; MXDBG=$((256 * c)) timeout -k 5 90 t-one_amd/gemm_bench_ablate 40960 1536 384 1 99 1 50 >> $O2 2>&1 || exit $?
  done
done
echo done2
