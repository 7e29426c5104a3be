# effective clock of the fp32 split GEMMs: GRBM_GUI_ACTIVE / 8 / kernel duration (rocprofv3 PMC pass)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/clk
FULLF32=1 NOC2=1 PP=1 ROWSCALE=1 timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE -d gpurun_out/clk -o run --output-format csv -- ./t-one_amd/gemm_bench 20480 384 3072 2 77,50,1650 1 30 > gpurun_out/clk.log 2>&1
echo rc=$?
find gpurun_out/clk -name '*.csv' | head
