"""Per-kernel sums of the SQ / GRBM counters collected by scripts/r04_sq_step.sh (one eager step, every kernel):
one row per kernel name with its launch count and each counter summed over its launches, plus the ratios that
say where the waves wait (MFMA busy / GRBM active cycles x 4 SIMDs x CUs is not formed: the counters are
per-SE sums, so only ratios within a kernel are printed)."""
import collections, csv, glob, sys


def load(root):
    f = glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", ""))
    return per, disp


def main():
    tot = collections.defaultdict(dict)
    n = {}
    for root in sys.argv[1:]:
        per, disp = load(root)
        for k, v in per.items():
            tot[k].update(v)
            n[k] = max(n.get(k, 0), len(disp[k]))
    rows = sorted(tot.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0))
    for k, c in rows:
        g = lambda x: c.get(x, 0.0)
        wave = g("SQ_WAVE_CYCLES") or 1.0
        out = {
            "launches": n[k],
            "gui_active": g("GRBM_GUI_ACTIVE"),
            "mfma_busy/busy": round(g("SQ_VALU_MFMA_BUSY_CYCLES") / max(g("SQ_BUSY_CYCLES"), 1), 3),
            "wait_any/wave": round(g("SQ_WAIT_ANY") / wave, 3),
            "wait_inst_any/wave": round(g("SQ_WAIT_INST_ANY") / wave, 3),
            "wait_inst_lds/wave": round(g("SQ_WAIT_INST_LDS") / wave, 3),
            "active_inst_any/wave": round(g("SQ_ACTIVE_INST_ANY") / wave, 3),
            "active_valu/wave": round(g("SQ_ACTIVE_INST_VALU") / wave, 3),
            "lds_conflict/lds_active": round(g("SQ_LDS_BANK_CONFLICT") / max(g("SQ_LDS_IDX_ACTIVE"), 1), 3),
            "insts": {x: g(x) for x in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_SALU", "SQ_WAVES")},
        }
        print(k[:90], out)


if __name__ == "__main__":
    main()
