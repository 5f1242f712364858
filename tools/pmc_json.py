"""Convert tools/pmc_traffic.sh output (FETCH_SIZE / WRITE_SIZE / TCC hit passes)
into profiles/pmc_c3.json: HBM bytes per launch per kernel.

Units and corrections follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and
WRITE_SIZE are in KiB; gfx950 FETCH_SIZE reports half the bytes of wide
coalesced reads, so reads are doubled (exact for the streamed record/uv
loads, an upper bound for narrow gathers).
usage: python tools/pmc_json.py gpurun_out/pmc_traffic profiles/pmc_c3.json
"""
import collections
import csv
import glob
import json
import sys

root, out = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(root + '/**/*counter_collection.csv', recursive=True)):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('sfm::', '')
        acc[n][r['Counter_Name']].append(float(r['Counter_Value']))
res = {"workload": "C3 (500 cams / 200000 pts / 2000000 obs), tools/pmc_c3.py", "n_obs": 2000000,
       "note": "hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md HBM corrections)",
       "kernels": {}}
for n, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    e = {"fetch_kib": m.get("FETCH_SIZE"), "write_kib": m.get("WRITE_SIZE")}
    if e["fetch_kib"] is not None and e["write_kib"] is not None:
        e["hbm_bytes_per_launch"] = (2 * e["fetch_kib"] + e["write_kib"]) * 1024
    h, mi = m.get("TCC_HIT_sum"), m.get("TCC_MISS_sum")
    if h is not None and mi:
        e["l2_hit_rate"] = h / (h + mi)
    res["kernels"][n] = e
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res["kernels"].get("k_jacobian")))
