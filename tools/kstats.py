"""Print a rocprofv3 kernel_stats.csv as name / calls / average us / share (development helper).
usage: python tools/kstats.py FILE [name-substring ...]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
keys = sys.argv[2:]
for r in rows:
    n = r["Name"]
    if keys and not any(k in n for k in keys):
        continue
    print(f"{n[:70]:70s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f} us {float(r['Percentage']):6.2f} %")
