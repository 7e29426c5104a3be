set -u
bash scripts/r04_xw_sweep.sh > /dev/null && bash scripts/r04_sm_check.sh > /dev/null; rc=$?
cat gpurun_out/r04_xw_sweep.jsonl gpurun_out/r04_sm_check.jsonl | cut -c1-220; exit $rc
