set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python scripts/mm_probe.py 2048 bf16 > gpurun_out/mm_bf16.log 2>&1 || exit 1
timeout -k 10 120 python scripts/mm_probe.py 256 fp32 > gpurun_out/mm_fp32.log 2>&1 || exit 1
ARGS="20480 384 3072 2 14 1 3" bash scripts/gemm_pmc.sh
