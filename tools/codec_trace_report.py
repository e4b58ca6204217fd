"""Per-decode kernel breakdown of a rocprofv3 kernel trace of tools/codec_probe.py (one section per
probed (B, L); the last timed decode of each). usage: python tools/codec_trace_report.py trace.csv"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "codes_gather" in r["Kernel_Name"]]
per = 1 + int(sys.argv[2]) if len(sys.argv) > 2 else 11  # warm-up + reps decodes per config
labels = sys.argv[3].split(",") if len(sys.argv) > 3 else [str(i) for i in range(len(starts) // per)]
for c, label in enumerate(labels):
    k = c * per + per - 1
    seg = rows[starts[k]:starts[k + 1]] if k + 1 < len(starts) else rows[starts[k]:]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in seg:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")[:100]
        agg[n][0] += 1
        agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    tot = sum(v[1] for v in agg.values())
    print(f"== {label}: {len(seg)} kernels, kernel time {tot:.1f} us")
    for n, (cnt, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:12]:
        print(f"  {d:8.1f} us {cnt:4d}x {d / cnt:7.2f}  {n}")
