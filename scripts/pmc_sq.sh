# SQ counter pass over one eager bf16 step (all kernels): where do the waves wait?
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-bf16}; B=${B:-2048}
rm -rf gpurun_out/pmc_sq
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU -d gpurun_out/pmc_sq -o run --output-format csv -- python bench.py --precision $P --batch $B --steps 1 --warmup 1 --no-graph --cpu-baseline-s 0 --alt 0 > gpurun_out/pmc_sq.log 2>&1
echo "pmc rc=$?"
