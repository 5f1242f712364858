"""Summarise rocprofv3 --pmc counter_collection CSVs: mean counter value per kernel."""
import csv, glob, sys, collections
root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(root + '/**/*counter_collection.csv', recursive=True)):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('sfm::', '')
        acc[n][r['Counter_Name']].append(float(r['Counter_Value']))
for n, cs in acc.items():
    print(n)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} mean={sum(v)/len(v):16.1f}  n={len(v)}")
