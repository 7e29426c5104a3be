# in-step A/B of the bf16 FFN up kernel: gemm_p (default) vs gemm_t 256x256 / 256x128 / 128x256, B = 2048 and 512
set -u
mkdir -p gpurun_out
out=gpurun_out/ab_ffnup.jsonl
: > $out
AB_BATCH=2048 timeout -k 10 300 python scripts/ab_env.py "" "TONE_SWIGLU_T=1" "TONE_SWIGLU_T=3" >> $out 2>&1 || { cat $out; exit 1; }
AB_BATCH=512 timeout -k 10 200 python scripts/ab_env.py "" "TONE_SWIGLU_T=1" "TONE_SWIGLU_T=3" "TONE_SWIGLU_T=2" >> $out 2>&1 || { cat $out; exit 1; }
cat $out
