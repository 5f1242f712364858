# Walker step timings of the fused Cholesky (variant build with g_stamp).
import ctypes, os, sys, numpy as np
sys.path.insert(0, '/root/repo' if not os.environ.get('GRAFT_REPO_ROOT') else os.environ['GRAFT_REPO_ROOT'])
import sfm_amd.ba
from sfm_amd import _ffi
n = 3000
rng = np.random.default_rng(n)
M = rng.standard_normal((n, n)); A = M @ M.T + n * np.eye(n); b = rng.standard_normal(n)
y, ms, fail = sfm_amd.ba.dense_spd_solve(A, b, reps=3)
print('ms', ms, 'fail', fail, 'err', float(np.max(np.abs(A @ y - b))))
lib = _ffi.lib()
buf = (ctypes.c_ulonglong * 2048)()
lib.sfm_debug_stamps(buf, 2048)
st = np.array(buf[:8 * 47], dtype=np.float64).reshape(47, 8) / 100.0  # 100 MHz -> us
t0 = st[0, 0]
names = ["T+upd+potrf", "store L/W+waitP1", "ld T1+waitPd", "trsm1+st", "waitP2", "ld+trsm2+st", "fence+pub"]
for j in range(44):
    d = np.diff(st[j, :8])
    print(f"j={j:2d} start {st[j,0]-t0:8.1f} " + " ".join(f"{nm} {v:5.2f}" for nm, v in zip(names, d)))
print('mean', dict(zip(names, np.round(np.mean(np.diff(st[:44, :8], axis=1), axis=0), 2))))
print('step mean', np.mean(np.diff(st[:46, 0])))
