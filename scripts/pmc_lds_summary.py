"""Per-kernel sums of the r05_pmc_lds.sh counters: LDS conflict share and counts, from rocprofv3 --pmc CSV output."""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1]
files = glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.Counter()
seen = set()
for f in files:
    for row in csv.DictReader(open(f)):
        name = re.sub(r"\(.*", "", row.get("Kernel_Name", "").replace("(anonymous namespace)::", ""))[:70]
        acc[name][row["Counter_Name"]] += float(row["Counter_Value"])
        key = (f, row.get("Dispatch_Id"), name)
        if key not in seen:
            seen.add(key)
            calls[name] += 1
rows = sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", 0))
print(f"{'kernel':70s} {'calls':>5s} {'conf/idx':>8s} {'lds_inst':>10s} {'valu_inst':>11s} {'mfma_busy':>12s} {'sq_busy':>12s}")
for name, c in rows[:30]:
    idx = c.get("SQ_LDS_IDX_ACTIVE", 0)
    conf = c.get("SQ_LDS_BANK_CONFLICT", 0)
    print(f"{name:70s} {calls[name]:5d} {conf / idx if idx else 0:8.3f} {c.get('SQ_INSTS_LDS', 0):10.3g} "
          f"{c.get('SQ_INSTS_VALU', 0):11.3g} {c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0):12.4g} {c.get('SQ_BUSY_CYCLES', 0):12.4g}")
