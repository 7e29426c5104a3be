# The driver's default bench command on the current tree; the JSON line -> gpurun_out/r04_bench_<tag>.json
set -u
mkdir -p gpurun_out
tag=${1:-cur}
timeout -k 10 900 python bench.py > gpurun_out/r04_bench_$tag.json 2> gpurun_out/r04_bench_$tag.err
rc=$?; echo "bench rc=$rc"
python3 - "$tag" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/r04_bench_{sys.argv[1]}.json"))
print("headline", d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["encoder_gemm_frac"])
for a in d["alt_workloads"]:
    r = a["roofline"] or {}
    print(a["workload"][:40], a["value"], a["ms_per_step"], r.get("frac"), r.get("encoder_gemm_frac"))
print(d["latency_b1"])
PY
exit $rc
