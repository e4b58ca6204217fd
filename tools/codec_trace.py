"""Per-kernel breakdown of the last codec decode in a rocprofv3 kernel trace."""
import csv, collections, glob, sys
f = sys.argv[1] if len(sys.argv) > 1 else glob.glob("gpurun_out/p_c/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "istft_ola" in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
win = rows[a + 1:b + 1]
span = (int(win[-1]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e3
agg = collections.OrderedDict()
for r in win:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    n = r["Kernel_Name"].split("(")[0].replace("void lvx::", "")[:80]
    g = agg.setdefault(n, [0, 0., r["Grid_Size_X"] + "x" + r["Grid_Size_Y"] + "x" + r["Grid_Size_Z"]])
    g[0] += 1; g[1] += (e - s) / 1e3
busy = sum(v[1] for v in agg.values())
print(f"{len(win)} kernels, span {span:.1f} us, busy {busy:.1f}")
for k, (c, d, gr) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"  {c:3d} x {d / c:8.2f} us  tot {d:8.1f}  {gr:>16s} {k}")
