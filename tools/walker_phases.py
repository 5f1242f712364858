"""Diagonal-walker phase times of the fused Cholesky at n=3000 from the
stamped variant tools/var_ws.so (tools/mkvar.sh ws "$(cat tools/walker_stamp_patch.py)" chol_kernels.hip)."""
import ctypes, os, sys
import numpy as np
R = os.environ.get('GRAFT_REPO_ROOT', os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
os.environ.setdefault("SFM_AMD_LIB", os.path.join(R, "tools", "var_ws.so"))
from sfm_amd.ba import dense_spd_solve
n = 3000
rng = np.random.default_rng(n)
B = rng.uniform(-1, 1, (n, n)); A = B + B.T; A[np.diag_indices(n)] += 2.0 * n; b = rng.standard_normal(n)
y, ms, fail = dense_spd_solve(A, b, reps=3)
print('ms', ms, 'fail', fail)
L = ctypes.CDLL(os.environ["SFM_AMD_LIB"])
buf = (ctypes.c_ulonglong * (64 * 16))()
assert L.sfm_debug_stamps(buf, 64 * 16) == 0
st = np.array(buf[:], dtype=np.float64).reshape(64, 16) / 100.0  # 100 MHz -> us
nb = 47
names = ["load+update", "potrf", "store+publish F(j,j)", "wait P(j+1,j)", "load+wait P(j+1,j+1)", "nx+trsm",
         "store+publish F(j+1,j)"]
d = {nm: np.mean([st[j, k + 1] - st[j, k] for j in range(1, nb - 2)]) for k, nm in enumerate(names)}
step = np.mean(np.diff(st[1:nb - 2, 0]))
print("per-step mean us:", {k: round(float(v), 2) for k, v in d.items()}, "step", round(float(step), 2))

inner = [(1, 8, "panel0"), (8, 12, "trail0"), (12, 9, "panel1"), (9, 13, "trail1"), (13, 10, "panel2"),
         (10, 14, "trail2"), (14, 11, "panel3"), (11, 15, "Wrow3"), (15, 2, "ret")]
print("potrf inner us:", {nm: round(float(np.mean([st[j, b] - st[j, a] for j in range(1, nb - 2)])), 2) for a, b, nm in inner})
