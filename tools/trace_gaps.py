"""Per-kernel duration and inter-kernel gap from a rocprofv3 kernel_trace.csv (last N kernels)."""
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
if len(sys.argv) > 3:  # only kernels whose name contains this substring (e.g. "ar_")
    rows = [r for r in rows if sys.argv[3] in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
rows = rows[-n:]
agg = collections.OrderedDict()
prev_end = None
gaps = []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0][:70]
    a = agg.setdefault(name, [0, 0.0, 0.0])
    a[0] += 1
    a[1] += (e - s) / 1e3
    if prev_end is not None:
        g = (s - prev_end) / 1e3
        a[2] += g
        gaps.append(g)
    prev_end = e
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
busy = sum(a[1] for a in agg.values())
print(f"{len(rows)} kernels, span {span:.1f} us, busy {busy:.1f} us, gaps {sum(gaps):.1f} us")
for k, (c, d, g) in agg.items():
    print(f"{c:5d} x {d / c:8.2f} us  (gap before {g / c:6.2f} us)  {k}")
