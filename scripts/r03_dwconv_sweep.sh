# dwconv block shapes at the fp32 headline (B = 256) and bf16 B = 2048: whole-step A/B per TONE_DWCONV_VARIANT
set -u
mkdir -p gpurun_out
O=gpurun_out/r03_dwconv_sweep.txt
: > $O
for v in -1 1 4 5 3; do
  for cfg in "fp32 256" "bf16 2048"; do
    set -- $cfg
    r=$(TONE_DWCONV_VARIANT=$v timeout -k 10 200 python bench.py --precision $1 --batch $2 --steps 200 --warmup 5 --alt 0 --cpu-baseline-s 0 --config4 0 --config5 0 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['median_ms'])") || exit 1
    echo "variant $v $1 B=$2: $r" >> $O
  done
done
echo done
