# SQ counters over one eager bf16 step at B = 4096 (every kernel), two rocprofv3 --pmc passes, summarised per
# kernel by scripts/sq_step_summary.py -> gpurun_out/r04_sq_step.txt
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-bf16}; B=${B:-4096}
run() {  # pass name, counters...
  local n=$1; shift
  rm -rf gpurun_out/sq_$n
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d gpurun_out/sq_$n -o run --output-format csv -- python bench.py --precision $P \
    --batch $B --steps 1 --warmup 1 --no-graph --cpu-baseline-s 0 --alt 0 --config4 0 --config5 0 > gpurun_out/sq_$n.log 2>&1
}
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
run b SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_WAVES || exit $?
python scripts/sq_step_summary.py gpurun_out/sq_a gpurun_out/sq_b > gpurun_out/r04_sq_step.txt
