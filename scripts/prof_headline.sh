# rocprofv3 kernel stats of the headline leg alone (fp32 B = 256; no alt legs, no CPU baseline), so the dominant
# kernel's average launch time can be compared with the bench line's roofline.avg_us from the same command
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf /tmp/prof_head
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_head -o run --output-format csv -- python bench.py --cpu-baseline-s 0 --alt 0 --config4 0 --config5 0 > gpurun_out/prof_head.log 2>&1 || exit $?
mkdir -p gpurun_out/prof_head
find /tmp/prof_head -name '*kernel_stats.csv' -exec cp {} gpurun_out/prof_head/ \;
grep '^{' gpurun_out/prof_head.log | head -1 | cut -c1-200
