"""Diagonal-walker phase account of the fused Cholesky, from the stamped
development build (tools/chol_stamps.sh -> abvar/var_stamps.so, compiled with
-DSFM_CHOL_STAMPS: the stamps sit in the production source, so the account is
of the kernel as built).  Usage:
  python tools/walker_phases.py [n] [reps]
Slots (per walker step j, s_memrealtime at 100 MHz): 0 step start, 1 last
update of column block 0 done + F(j,j-1) published, 2..5 after POTRF panel b,
6..8 after the trailing update of column block b+1, 9 W row 3 done (POTRF
end), 10 early loads + W stores issued, 11 F(j,j) published, 12 waits done
(the fallback path when the POTRF's poll missed), 13 TRSM of the sub-diagonal
tile done, 14 its stores issued (step end); 15 = 1 when the poll found both
partial tiles out.  Helper stamps: publication of partial tile (i, j) and of
final tile (i, j)."""
import ctypes
import json
import os
import sys

import numpy as np

R = os.environ.get('GRAFT_REPO_ROOT', os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
os.environ.setdefault("SFM_AMD_LIB", os.path.join(R, "abvar", "var_stamps.so"))
from sfm_amd.ba import dense_spd_solve  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rng = np.random.default_rng(n)
B = rng.uniform(-1, 1, (n, n))
A = B + B.T
A[np.diag_indices(n)] += 2.0 * n
b = rng.standard_normal(n)
y, ms, fail = dense_spd_solve(A, b, reps=reps)
res = float(np.max(np.abs(A @ y - b)) / np.max(np.abs(b)))
L = ctypes.CDLL(os.environ["SFM_AMD_LIB"])
L.sfm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * (256 * 16))()
hb = (ctypes.c_ulonglong * (128 * 128 * 2))()
assert L.sfm_debug_stamps(buf, 256 * 16, hb, 128 * 128 * 2) == 0
raw = np.array(buf[:], dtype=np.float64).reshape(256, 16)
hs = np.array(hb[:], dtype=np.float64).reshape(128, 128, 2) / 100.0
nb = (n + 1 + 63) // 64
st = raw / 100.0  # 100 MHz -> us
js = list(range(2, nb - 2))  # steady-state steps
step = float(np.mean(np.diff(st[2:nb - 1, 0])))


def seg(a, b_):
    return round(float(np.mean([st[j, b_] - st[j, a] for j in js])), 3)


walker = {
    "T in + last update col 0 + publish F(j,j-1)": seg(0, 1),
    "potrf": seg(1, 9),
    "early loads + W stores issued": seg(9, 10),
    "publish F(j,j) (drain)": seg(10, 11),
    "fallback waits": seg(11, 12),
    "trsm sub tile": seg(12, 13),
    "L(j+1,j) stores issued": seg(13, 14),
    "-> next step": round(float(np.mean([st[j + 1, 0] - st[j, 14] for j in js])), 3),
}
potrf = {"panel0 (+ last update rest)": seg(1, 2)}
for b_ in range(3):
    potrf[f"trail{b_}"] = seg(2 + b_, 6 + b_)
    potrf[f"panel{b_ + 1}"] = seg(6 + b_, 3 + b_)
potrf["W row 3"] = seg(5, 9)
early = float(np.mean([raw[j, 15] for j in js]))
# arrival of what the walker awaits, relative to its step start
ev = {
    "P(j+1,j) sub partial": [hs[j + 1, j, 0] - st[j, 0] for j in js if j + 1 < 128],
    "P(j+1,j+1) diag partial": [hs[j + 1, j + 1, 0] - st[j, 0] for j in js if j + 1 < 128],
    "F(j+1,j-1) first final tile of col j-1": [hs[j + 1, j - 1, 1] - st[j, 0] for j in js if j + 1 < 128],
    "potrf end (W_j ready)": [st[j, 9] - st[j, 0] for j in js],
}
arr = {k: (round(float(np.median(v)), 2), round(float(np.percentile(v, 90)), 2)) for k, v in ev.items()}
# per wave: the end of its panel-3 work after the panel's start (slot 8)
pb = (ctypes.c_ulonglong * (256 * 4))()
p3w = None
if hasattr(L, "sfm_debug_pstamps") and L.sfm_debug_pstamps(pb, 256 * 4) == 0:
    ps = np.array(pb[:], dtype=np.float64).reshape(256, 4) / 100.0
    p3w = {f"wave{w}": round(float(np.mean([ps[j, w] - st[j, 8] for j in js])), 3) for w in range(4)}
out = {"n": n, "ms_factor_plus_backsolve": round(ms, 4), "fail": fail, "rel_residual": res,
       "step_us": round(step, 3), "steps": nb, "early_frac": early, "walker_us": walker, "potrf_us": potrf,
       "arrivals_us_median_p90": arr, "panel3_work_end_us_per_wave": p3w}
print(json.dumps(out, indent=1))
