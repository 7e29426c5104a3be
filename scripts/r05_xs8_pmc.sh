#!/bin/bash
# SQ + GRBM counters of the fp8 FFN up (gemm_xs8, gemm_bench variant 98, M = 40960, rowscale) and its ablations
# (MXDBG: 0 full, 1 no epilogue, 2 no MFMA, 3 neither), one rocprofv3 --pmc pass each -> gpurun_out/xs8_pmc_<d>/
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
A=t-one_amd/gemm_bench_ablate
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
for d in 0 1 2 3; do
  o=gpurun_out/xs8_pmc_$d
  rm -rf $o
  NOREF=1 ROWSCALE=1 MXDBG=$d timeout -s KILL 60 rocprofv3 --pmc $C -d $o -o run --output-format csv -- $A 40960 384 3072 2 98 1 5 > $o.log 2>&1 || exit $?
  echo "dbg $d ok"; grep variant $o.log | tail -1
done
python3 - <<'PY'
import csv, glob, collections, json
out = {}
for d in (0, 1, 2, 3):
    f = glob.glob(f"gpurun_out/xs8_pmc_{d}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        if "xs8" not in r["Kernel_Name"]: continue
        per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    c = {k: sum(v.values()) / len(v) for k, v in per.items()}
    c["mfma_busy_frac_of_launch"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] * 4 * 32), 3)
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        c[k + "_frac"] = round(c[k] / c["SQ_WAVE_CYCLES"], 3)
    out[f"dbg{d}"] = c
json.dump(out, open("gpurun_out/r05_xs8_sq_counters.json", "w"), indent=1)
for k, c in out.items(): print(k, {x: c[x] for x in c if x.endswith("frac") or x.startswith("mfma")})
PY
