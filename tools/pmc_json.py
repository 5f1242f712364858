"""Convert tools/pmc_traffic.sh output (FETCH_SIZE / WRITE_SIZE / TCC hit passes)
into profiles/pmc_c3.json: HBM bytes per launch per kernel.

Units and corrections follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and
WRITE_SIZE are in KiB; gfx950 FETCH_SIZE reports half the bytes read, so
reads are doubled.  The guide calibrates that only for wide streamed reads;
tools/pmc_calib.hip measures it on known byte counts for every width the BA
kernels use (8/16 B per lane streamed, 128-B records gathered by 8 lanes or
one lane, sparse 8-B gathers that pull a 128-B line each) and for 8/16-B
streamed and 128-B scattered stores; the "calibration" section holds the
measured ratios (reported / true bytes).
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
        n = n[5:] if n.startswith('void ') else n
        # the two Jacobian instantiations apart: the solve's record-free pass
        # and the evaluate API's record-writing one
        n = {'k_jacobian<false>': 'k_jacobian', 'k_jacobian<true>': 'k_jacobian_rec'}.get(n, n)
        acc[n][r['Counter_Name']].append(float(r['Counter_Value']))
res = {"workload": "C3 (500 cams / 200000 pts / 2000000 obs), tools/pmc_c3.py (host-driven LM loop: no skipped launches); calibration: tools/pmc_calib.hip", "n_obs": 2000000,
       "note": "hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md HBM corrections)",
       "kernels": {}}
# known bytes of the calibration kernels (tools/pmc_calib.hip): 1 GiB table,
# 8 Mi random indices (32 MiB, streamed 4 B per lane) on the gathers
GiB, IDX = 1 << 30, 32 << 20
known = {"cal_read16": (GiB, 0), "cal_read8": (GiB, 0), "cal_gather128": (GiB + IDX, 0),
         "cal_gather128_lane": (GiB + IDX, 0), "cal_gather8": ((8 << 20) * 128 + IDX, 0),
         "cal_write16": (0, GiB), "cal_write8": (0, GiB), "cal_scatter128": (IDX, GiB)}
cal = {}
for n, (rb, wb) in known.items():
    if n not in acc:
        continue
    m = {c: sum(v) / len(v) for c, v in acc[n].items()}
    e = {"true_read_bytes": rb, "true_write_bytes": wb}
    if rb and "FETCH_SIZE" in m:
        e["fetch_size_over_true"] = round(m["FETCH_SIZE"] * 1024 / rb, 4)
    if wb and "WRITE_SIZE" in m:
        e["write_size_over_true"] = round(m["WRITE_SIZE"] * 1024 / wb, 4)
    cal[n] = e
if cal:
    res["calibration"] = cal
for n, cs in acc.items():
    if n in known or n.startswith("__amd"):
        continue
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    e = {"fetch_kib": m.get("FETCH_SIZE"), "write_kib": m.get("WRITE_SIZE")}
    if e["fetch_kib"] is not None and e["write_kib"] is not None:
        e["hbm_bytes_per_launch"] = (2 * e["fetch_kib"] + e["write_kib"]) * 1024
    h, mi = m.get("TCC_HIT_sum"), m.get("TCC_MISS_sum")
    if h is not None and mi:
        e["l2_hit_rate"] = h / (h + mi)
    res["kernels"][n] = e
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res["kernels"].get("k_jacobian")), json.dumps(res["kernels"].get("k_jacobian_rec")))
