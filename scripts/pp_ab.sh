# gemm_pp schedule A/B at the FFN-up shape: ping-pong (v), no DMA (+1600), X-only DMA (+51200),
# lockstep (+25600), lockstep X-only (+76800)
set -u
mkdir -p gpurun_out
out=gpurun_out/pp_ab.jsonl
: > $out
B=./t-one_amd/gemm_bench
FULLF32=1 NOC2=1 PP=1 ROWSCALE=1 timeout -k 10 60 $B 2560 384 3072 2 50,102450,1650,25650,128050,50,102450 1 50 >> $out 2>&1
cat $out
