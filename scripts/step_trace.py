"""Per-dispatch durations of the last full step in a rocprofv3 kernel trace (grouped by kernel); with a second
argument "seq", also every dispatch of that step in launch order (name, grid, duration)."""
import collections, csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
seq = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000) for r in rows]
grids = [r.get("Grid_Size", r.get("Grid_Size_X", "")) for r in rows]
idx = [i for i, (n, _) in enumerate(seq) if "mel_prep" in n]
st, en = idx[-2], idx[-1]
agg = collections.defaultdict(lambda: [0, 0.0])
for n, d in seq[st:en]:
    k = re.sub(r"\([^()]*\)$", "", n).replace("(anonymous namespace)::", "")[:110]
    agg[k][0] += 1
    agg[k][1] += d
tot = sum(v[1] for v in agg.values())
for k, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{d:9.1f} us {c:4d}x {100 * d / tot:5.1f}%  {k}")
print(f"{tot:9.1f} us total (one step, graph replay)")
if len(sys.argv) > 2 and sys.argv[2] == "seq":
    print("\n# launch order")
    for i in range(st, en):
        n, d = seq[i]
        k = re.sub(r"\([^()]*\)$", "", n).replace("(anonymous namespace)::", "").replace("tone::", "")[:90]
        print(f"{d:8.2f} us  grid {grids[i]:>8}  {k}")
