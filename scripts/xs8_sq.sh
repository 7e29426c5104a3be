#!/bin/bash
# SQ counters of the fp8 FFN up (gemm_xs8, M = 40960, SwiGLU + MXFP8 epilogue) on the current tree, one PMC pass over
# gemm_bench (the round-5 pass: profiles/r05_xs8_sq_counters.json "dbg0"), per-launch means of the gemm_xs8 launches
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_xs8
NOREF=1 ROWSCALE=1 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc_xs8 -o run --output-format csv -- t-one_amd/gemm_bench 40960 384 3072 2 98 1 20 > gpurun_out/pmc_xs8.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_xs8.log; exit $rc; }
python3 - <<'PY'
import csv, glob, json, collections
f = glob.glob("gpurun_out/pmc_xs8/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    if "gemm_xs8" in r["Kernel_Name"]:
        acc[r["Counter_Name"]][r.get("Dispatch_Id", r.get("Correlation_Id", ""))].append(float(r["Counter_Value"]))
out = {k: sum(sum(v) for v in d.values()) / len(d) for k, d in acc.items()}
out["launches"] = len(next(iter(acc.values()))) if acc else 0
if out.get("GRBM_GUI_ACTIVE"):
    out["valu_issue_over_mfma_busy"] = round(out["SQ_ACTIVE_INST_VALU"] / max(out["SQ_VALU_MFMA_BUSY_CYCLES"], 1), 3)
print(json.dumps(out))
json.dump(out, open("gpurun_out/r06_xs8_sq_counters.json", "w"))
PY
