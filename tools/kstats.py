import csv, sys, glob
f = sys.argv[1]
if not f.endswith('.csv'):
    import os
    f = max(glob.glob(f + '/**/*kernel_stats.csv', recursive=True), key=os.path.getmtime)
rows = list(csv.DictReader(open(f)))
for r in rows:
    n = r['Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('sfm::', '')
    print(f"{n:34s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:9.2f} min_us={float(r['MinNs'])/1e3:8.2f} max_us={float(r['MaxNs'])/1e3:8.2f} total_ms={float(r['TotalDurationNs'])/1e6:8.3f} pct={float(r['Percentage']):5.1f}")
