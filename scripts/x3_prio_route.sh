# fp32 split GEMM tile choice with the static priority on (default): FFN up 256x128 (77) vs 128x128 (76),
# FFN down / attn-out 64x64 (70) vs 32x64 (80), q|k|v 128x128 (76), pw1 128x64 (71); alternating passes
set -u
mkdir -p gpurun_out
out=gpurun_out/x3_prio_route.jsonl
: > $out
B=./t-one_amd/gemm_bench
for pass in 1 2; do
  FULLF32=1 NOC2=1 ROWSCALE=1 timeout -k 10 60 $B 2560 384 3072 2 77,76 1 50 >> $out 2>&1 || echo fail
  FULLF32=1 NOC2=1 ROWSCALE=1 timeout -k 10 60 $B 1280 384 3072 2 77,76 1 50 >> $out 2>&1 || echo fail
  FULLF32=1 NOC2=1 timeout -k 10 60 $B 2560 1536 384 1 70,80 1 50 >> $out 2>&1 || echo fail
  FULLF32=1 NOC2=1 timeout -k 10 60 $B 1280 1536 384 1 70,80 1 50 >> $out 2>&1 || echo fail
  FULLF32=1 NOC2=1 timeout -k 10 60 $B 2560 384 384 1 70,80 1 50 >> $out 2>&1 || echo fail
  FULLF32=1 NOC2=1 ROWSCALE=1 timeout -k 10 60 $B 2560 384 768 3 71,76 1 50 >> $out 2>&1 || echo fail
done
cat $out
