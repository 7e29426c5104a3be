#!/bin/bash
# SQ counters of the fp8 FFN up (gemm_xs8, M = 40960, SwiGLU + MXFP8 epilogue), one PMC pass over
# gemm_bench, per-launch means of the gemm_xs8 launches.  Args: binary (default t-one_amd/gemm_bench; a build of an
# earlier commit for a before / after pair) and tag.
set -u
bin=${1:-t-one_amd/gemm_bench}; tag=${2:-cur}
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_xs8_$tag
NOREF=1 ROWSCALE=1 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc_xs8_$tag -o run --output-format csv -- $bin 40960 384 3072 2 98 1 20 > gpurun_out/pmc_xs8_$tag.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_xs8_$tag.log; exit $rc; }
NOREF=1 ROWSCALE=1 timeout -k 10 60 $bin 40960 384 3072 2 98 1 200 | grep '^{' | tail -1 > gpurun_out/xs8_time_$tag.json || exit 1
TAG=$tag python3 - <<'PY'
import csv, glob, json, collections, os
tag = os.environ["TAG"]
f = glob.glob(f"gpurun_out/pmc_xs8_{tag}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    if "gemm_xs8" in r["Kernel_Name"]:
        acc[r["Counter_Name"]][r.get("Dispatch_Id", r.get("Correlation_Id", ""))].append(float(r["Counter_Value"]))
out = {k: sum(sum(v) for v in d.values()) / len(d) for k, d in acc.items()}
out["launches"] = len(next(iter(acc.values()))) if acc else 0
if out.get("GRBM_GUI_ACTIVE"):
    out["valu_issue_over_mfma_busy"] = round(out["SQ_ACTIVE_INST_VALU"] / max(out["SQ_VALU_MFMA_BUSY_CYCLES"], 1), 3)
    out["mfma_busy_frac_of_launch"] = round(out["SQ_VALU_MFMA_BUSY_CYCLES"] / (out["GRBM_GUI_ACTIVE"] * 128), 3)
out["us"] = json.loads(open(f"gpurun_out/xs8_time_{tag}.json").read()).get("us")
print(tag, json.dumps(out))
json.dump(out, open(f"gpurun_out/xs8_sq_{tag}.json", "w"))
PY
