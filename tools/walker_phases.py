"""Diagonal-walker phase times of the fused Cholesky from the stamped
variant abvar/var_stamps.so (tools/chol_stamps.sh).  Usage:
  SFM_CHOL_OPT=<bits> python tools/walker_phases.py [n]"""
import ctypes, os, sys
import numpy as np
R = os.environ.get('GRAFT_REPO_ROOT', os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
os.environ.setdefault("SFM_AMD_LIB", os.path.join(R, "tools", "var_stamps.so"))
from sfm_amd.ba import dense_spd_solve
n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
rng = np.random.default_rng(n)
B = rng.uniform(-1, 1, (n, n)); A = B + B.T; A[np.diag_indices(n)] += 2.0 * n; b = rng.standard_normal(n)
y, ms, fail = dense_spd_solve(A, b, reps=3)
L = ctypes.CDLL(os.environ["SFM_AMD_LIB"])
buf = (ctypes.c_ulonglong * (256 * 16))()
assert L.sfm_debug_stamps(buf, 256 * 16) == 0
raw = np.array(buf[:], dtype=np.float64).reshape(256, 16)
nb = (n + 1 + 63) // 64
st = raw / 100.0  # 100 MHz -> us
js = range(1, nb - 2)
names = ["step start->LU done", "potrf", "W out + fetch what the polls missed", "trsm", "L stores issued",
         "-> next step"]
slots = [0, 1, 2, 3, 5, 6]
seg = {}
for k, nm in enumerate(names[:-1]):
    seg[nm] = np.mean([st[j, slots[k + 1]] - st[j, slots[k]] for j in js])
seg[names[-1]] = np.mean([st[j + 1, 0] - st[j, 6] for j in js])
got = [int(raw[j, 7]) for j in js]
early = f"sub {np.mean([g & 1 for g in got]):.2f} diag {np.mean([(g >> 1) & 1 for g in got]):.2f} (prefetched by wave 1)"
step = np.mean(np.diff(st[1:nb - 2, 0]))
inner = {"panel0": np.mean([st[j, 8] - st[j, 1] for j in js])}
for b_ in range(1, 4):
    inner[f"panel{b_}"] = np.mean([st[j, 8 + b_] - st[j, 7 + b_] for j in js])
inner["Wrow3"] = np.mean([st[j, 12] - st[j, 11] for j in js])
print(f"n={n} ms={ms:.3f} fail={fail} opt={os.environ.get('SFM_CHOL_OPT', 'default')} step={step:.2f} us "
      f"early: {early}")
print("  walker:", {k: round(float(v), 2) for k, v in seg.items()})
print("  potrf :", {k: round(float(v), 2) for k, v in inner.items()})
# helper publications relative to the walker's step start (us): the partial
# tiles it waits for and the first final tile of the previous column
hb = (ctypes.c_ulonglong * (64 * 64 * 2))()
if L.sfm_debug_hstamps(hb, 64 * 64 * 2) == 0:
    hs = np.array(hb[:], dtype=np.float64).reshape(64, 64, 2) / 100.0
    jj = [j for j in js if j + 1 < 64]
    ev = {"Pf(j+1,j) sub partial": [hs[j + 1, j, 0] - st[j, 0] for j in jj],
          "Pf(j+1,j+1) diag partial": [hs[j + 1, j + 1, 0] - st[j, 0] for j in jj],
          "F(j+1,j-1) first final of col j-1": [hs[j + 1, j - 1, 1] - st[j, 0] for j in jj],
          "W_j out (walker, after the POTRF)": [st[j, 2] - st[j, 0] for j in jj],
          "potrf end": [st[j, 2] - st[j, 0] for j in jj]}
    print("  arrivals (us after step start, median / p90):",
          {k: (round(float(np.median(v)), 2), round(float(np.percentile(v, 90)), 2)) for k, v in ev.items()})
