#!/bin/bash
# LDS bank conflicts and matrix-pipe busy per kernel over one eager step (bf16 B = 4096 by default):
# SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE = the share of LDS cycles lost to conflicts
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-bf16}; B=${B:-4096}
rm -rf gpurun_out/pmc_lds_$P
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU -d gpurun_out/pmc_lds_$P -o run --output-format csv -- python bench.py --precision $P --batch $B --steps 1 --warmup 1 --no-graph --cpu-baseline-s 0 --alt 0 --config4 0 --config5 0 > gpurun_out/pmc_lds_$P.log 2>&1
echo "pmc rc=$?"
python3 scripts/pmc_lds_summary.py gpurun_out/pmc_lds_$P > gpurun_out/pmc_lds_$P.txt && cat gpurun_out/pmc_lds_$P.txt
