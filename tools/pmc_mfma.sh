#!/bin/bash
# MFMA-busy of the C3 kernels: SQ_VALU_MFMA_BUSY_CYCLES (summed over SIMDs)
# against GRBM_GUI_ACTIVE (summed over the 8 XCDs), one pass, no tracing.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_mfma
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
RX='k_chol_fused|k_schur_pts|k_obs_prep'
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$RX" --output-format csv -d $OUT -- python3 $R/tools/pmc_c3.py solve > $OUT/run.log 2>&1 || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, json
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('sfm::', '')
        acc[n][r['Counter_Name']].append(float(r['Counter_Value']))
res = {}
for n, cs in acc.items():
    n = n[5:] if n.startswith('void ') else n
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    busy, gui = m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0), m.get('GRBM_GUI_ACTIVE', 0.0)
    cyc = gui / 8.0  # per-XCD elapsed cycles
    frac = busy / (cyc * 1024.0) if cyc else 0.0  # 256 CUs x 4 SIMDs
    print(f"{n:20s} mfma_busy_cycles={busy:14.0f} elapsed_cycles={cyc:10.0f} mfma_busy_frac={frac:.4f}")
    res[n] = {"mfma_busy_cycles": busy, "elapsed_cycles_per_xcd": cyc, "mfma_busy_frac": frac}
json.dump({"workload": "C3, tools/pmc_c3.py solve (host-driven LM loop)", "counters":
           "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)", "kernels": res},
          open(sys.argv[1] + "/pmc_mfma.json", "w"), indent=1)
PY
