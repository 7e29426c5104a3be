set -u
mkdir -p gpurun_out
for ns in 1 2 4; do FULLF32=1 timeout -k 10 60 ./t-one_amd/gemm_bench 1280 1536 384 1 50,54 $ns 20 || exit 1; done
FULLF32=1 timeout -k 10 60 ./t-one_amd/gemm_bench 2560 1536 384 1 56 4 20 || exit 1
FULLF32=1 timeout -k 10 60 ./t-one_amd/gemm_bench 1280 1536 384 1 -2 1 20 || exit 1
