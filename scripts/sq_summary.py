"""Summarise an SQ PMC pass per kernel name (mean per dispatch)."""
import collections, csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    agg[r["Kernel_Name"].split("(")[0][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for k, d in agg.items():
    if pat not in k:
        continue
    m = {c: sum(v) / len(v) for c, v in d.items()}
    wc = m.get("SQ_WAVE_CYCLES", 1)
    print(f"{k}: waits any {m.get('SQ_WAIT_ANY',0)/wc:.2f} inst {m.get('SQ_WAIT_INST_ANY',0)/wc:.2f} active {m.get('SQ_ACTIVE_INST_ANY',0)/wc:.2f} "
          f"| vmem {m.get('SQ_INSTS_VMEM',0):.0f} lds {m.get('SQ_INSTS_LDS',0):.0f} valu {m.get('SQ_INSTS_VALU',0):.0f} bankconf {m.get('SQ_LDS_BANK_CONFLICT',0):.0f} wavecyc {wc:.0f}")
