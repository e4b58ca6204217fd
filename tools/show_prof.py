import csv, sys, glob
f = sys.argv[1] if len(sys.argv) > 1 else glob.glob('gpurun_out/prof/**/*kernel_stats.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f"{float(r['TotalDurationNs'])/1e3:10.1f}us calls={r['Calls']:>6} avg={float(r['AverageNs'])/1e3:8.2f}us {100*float(r['TotalDurationNs'])/tot:5.1f}% {r['Name'][:100]}")
