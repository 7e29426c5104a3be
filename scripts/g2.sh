set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/profile.sh bf16 --precision bf16 --batch 2048 || exit 1
V=0,1,3,5,6,10,13,14 F=0 timeout -k 10 300 bash scripts/gemm_sweep.sh || exit 1
