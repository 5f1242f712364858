"""Which LM decisions of the lm_branches scenes rounding decides: the oracle
(Ceres 1.12 restatement) against itself with (a) its reduced camera matrix's
diagonal blocks summed in another valid order (order=1, the device solver's
association) and (b) 1-64 ulp perturbations of the start / of uv.  Output:
profiles/r04_gauge_order_probe.txt (CPU only)."""
import json
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
import lm_cases as L  # noqa: E402
from oracle import ffi as O  # noqa: E402

FIX = json.load(open(os.path.join(R, "tests", "golden", "lm_branches.json")))


def seq(tr):
    return "".join("I" if not it["step_is_valid"] else ("A" if it["step_is_successful"] else "R") for it in tr[1:])


def agree(a, b):
    return next((i for i in range(min(len(a), len(b))) if a[i] != b[i]), min(len(a), len(b)))


for name in sorted(FIX):
    c = FIX[name]
    build, _, mode = L.cases()[name]
    s = build()
    opts = O.default_options(**c["options"])
    out = []
    for order in (0, 1):
        r, t, X = s.copy_params()
        sm, tr = O.solve(s.uv, s.cam_idx, s.pt_idx, s.K, r, t, X, mode=mode, options=opts, order=order)
        out.append((seq(tr), sm["final_cost"], tr))
    a, b = out[0][0], out[1][0]
    print(f"{name:18s} 1e-6 prefix {L.decisive_prefix(out[0][2], 1e-6):2d}  order-robust prefix {agree(a, b):2d}  "
          f"final cost rel {abs(out[0][1] - out[1][1]) / out[0][1]:.1e}   order 0: {a[:24]}   order 1: {b[:24]}")
    if name.startswith("gauge"):
        print("   cost change / cost per iteration:",
              " ".join(f"{abs(it['cost_change']) / it['cost']:.1e}" for it in out[0][2][1:10]))
        for ulp in (1, 4, 16, 64):
            rng = np.random.default_rng(7)
            ag = []
            for _ in range(8):
                rp, tp, Xp = (x * (1 + ulp * 2.2e-16 * rng.uniform(-1, 1, x.shape)) for x in (s.rot, s.t, s.X))
                _, tr2 = O.solve(s.uv, s.cam_idx, s.pt_idx, s.K, rp.copy(), tp.copy(), Xp.copy(), mode=mode,
                                 options=opts)
                ag.append(agree(seq(tr2), a))
            print(f"   start perturbed by {ulp:2d} ulp: decisions agree for {ag}")
