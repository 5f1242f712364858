import sys, json, numpy as np
sys.path.insert(0, 'tests'); sys.path.insert(0, '.')
import lm_cases as L
import sfm_amd
FIX = json.load(open('tests/golden/lm_branches.json'))
def seq(tr): return "".join("I" if not it["step_is_valid"] else ("A" if it["step_is_successful"] else "R") for it in tr[1:])
for name in ["gauge_1e15", "gauge_1e16"]:
    c = FIX[name]; build, _, mode = L.cases()[name]; s = build()
    r, t, X = s.copy_params()
    sm, tr = sfm_amd.solve(s.uv, s.cam_idx, s.pt_idx, s.K, r, t, X, mode=mode, options=sfm_amd.make_options(**c["options"]))
    print(name, "GPU", seq(tr)[:40], "costs", ["%.6e" % it["cost"] for it in tr[:5]])
