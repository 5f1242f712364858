"""Walker / POTRF phase stamps of the fused Cholesky (variant tools/var_cs.so
built by tools/mkvar.sh with /tmp/stamp_patch.py-style s_memrealtime stamps)."""
import ctypes, os, sys
import numpy as np
R = os.environ.get('GRAFT_REPO_ROOT', os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
os.environ.setdefault("SFM_AMD_LIB", os.path.join(R, "tools", "var_cs.so"))
from sfm_amd.ba import dense_spd_solve
from sfm_amd import _ffi
n = 3000
rng = np.random.default_rng(n)
M = rng.standard_normal((n, n)); A = M @ M.T + n * np.eye(n); b = rng.standard_normal(n)
y, ms, fail = dense_spd_solve(A, b, reps=3)
print('ms', ms, 'fail', fail)
L = ctypes.CDLL(os.environ["SFM_AMD_LIB"])
buf = (ctypes.c_ulonglong * (64 * 24))()
L.sfm_debug_stamps(buf, 64 * 24)
st = np.array(buf[:], dtype=np.float64).reshape(64, 24) / 100.0  # 100 MHz -> us
nb = 47
names = {(0, 1): "ldT", (1, 2): "upd", (2, 8): "potrf_pre", (8, 9): "pan0", (9, 10): "trl0", (10, 11): "pan1",
         (11, 12): "trl1", (12, 13): "pan2", (13, 14): "trl2", (14, 15): "pan3", (15, 16): "trl3", (16, 17): "Wrow3",
         (17, 3): "ret", (3, 4): "store+pub", (4, 5): "waitLsub", (5, 6): "ldsub+waitDiag", (6, 7): "trsm+st+pub"}
acc = {v: [] for v in names.values()}
for j in range(1, nb - 2):
    for (a, c), nm in names.items():
        acc[nm].append(st[j, c] - st[j, a])
print("per-step mean us:", {k: round(float(np.mean(v)), 2) for k, v in acc.items()})
print("step total mean", round(float(np.mean(np.diff(st[1:nb - 2, 0]))), 2))
