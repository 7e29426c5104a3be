# in-step A/B of static wave priority in the bf16 (TONE_PRIO_BF16) and MXFP8 (TONE_PRIO_MX) GEMM kernels
set -u
mkdir -p gpurun_out
out=gpurun_out/ab_prio_lp.jsonl
: > $out
AB_BATCH=2048 AB_PREC=bf16 timeout -k 10 300 python scripts/ab_env.py "" "TONE_PRIO_BF16=1" >> $out 2>&1 || { cat $out; exit 1; }
AB_BATCH=512 AB_PREC=bf16 timeout -k 10 200 python scripts/ab_env.py "" "TONE_PRIO_BF16=1" >> $out 2>&1 || { cat $out; exit 1; }
AB_BATCH=2048 AB_PREC=fp8 timeout -k 10 300 python scripts/ab_env.py "" "TONE_PRIO_MX=1" "TONE_PRIO_BF16=1,TONE_PRIO_MX=1" >> $out 2>&1 || { cat $out; exit 1; }
grep '^{' $out
