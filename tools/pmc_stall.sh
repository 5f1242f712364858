#!/bin/bash
# Where the waves of the C3 kernels spend their cycles (MI355X_MICROARCH.md
# "rocprofv3 PMC slots": WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~
# WAVE_CYCLES, all in quad-cycles) plus VALU activity: one pass of 6 SQ
# counters and GRBM_GUI_ACTIVE, no tracing.  -> gpurun_out/pmc_stall/pmc_stall.json
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_stall
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
RX='k_jacobian|k_chol_fused|k_obs_prep|k_backsub|k_schur_pts|k_point_eval'
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex "$RX" --output-format csv -d $OUT -- python3 $R/tools/pmc_c3.py solve > $OUT/run.log 2>&1 || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, json
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('sfm::', '')
        n = n[5:] if n.startswith('void ') else n
        n = {'k_jacobian<false>': 'k_jacobian', 'k_jacobian<true>': 'k_jacobian_rec'}.get(n, n)
        acc[n][r['Counter_Name']].append(float(r['Counter_Value']))
res = {}
for n, cs in sorted(acc.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    wc = m.get('SQ_WAVE_CYCLES', 0.0) or 1.0
    e = {c: m[c] for c in m}
    e["wait_any_frac"] = m.get('SQ_WAIT_ANY', 0.0) / wc
    e["wait_inst_any_frac"] = m.get('SQ_WAIT_INST_ANY', 0.0) / wc
    e["active_inst_any_frac"] = m.get('SQ_ACTIVE_INST_ANY', 0.0) / wc
    e["active_valu_frac_of_wave_cycles"] = m.get('SQ_ACTIVE_INST_VALU', 0.0) / wc
    cyc = m.get('GRBM_GUI_ACTIVE', 0.0) / 8.0
    # VALU issue cycles (quad-cycles x 4) over the SIMD-cycles of the launch
    e["valu_busy_frac_of_simd_cycles"] = 4 * m.get('SQ_ACTIVE_INST_VALU', 0.0) / (cyc * 1024.0) if cyc else None
    res[n] = e
    print(f"{n:22s} wait_any {e['wait_any_frac']:.3f} wait_inst {e['wait_inst_any_frac']:.3f} active {e['active_inst_any_frac']:.3f} valu/wave {e['active_valu_frac_of_wave_cycles']:.3f} valu/simd {e['valu_busy_frac_of_simd_cycles']}")
json.dump({"workload": "C3, tools/pmc_c3.py solve (host-driven LM loop), means per launch",
           "units": "SQ_* in quad-cycles summed over waves (MI355X_MICROARCH.md); GRBM_GUI_ACTIVE summed over 8 XCDs",
           "kernels": res}, open(sys.argv[1] + "/pmc_stall.json", "w"), indent=1)
PY
