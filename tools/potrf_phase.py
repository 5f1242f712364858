# Phase times inside potrf_tile for tile 20 (variant build tools/var_pst.so).
import ctypes, os, sys, numpy as np
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '/root/repo'))
import sfm_amd.ba
from sfm_amd import _ffi
n = 3000
rng = np.random.default_rng(n)
M = rng.standard_normal((n, n)); A = M @ M.T + n * np.eye(n); b = rng.standard_normal(n)
y, ms, fail = sfm_amd.ba.dense_spd_solve(A, b, reps=3)
buf = (ctypes.c_ulonglong * 16)()
_ffi.lib().sfm_debug_stamps(buf, 16)
st = np.array(buf[:10], dtype=np.float64) / 100.0
d = np.diff(st)
print('ms', ms, 'total potrf_tile us', st[9] - st[0])
for b in range(4):
    print(f"panel {b}: factor+Woff {d[2*b]:.2f} us, trailing {d[2*b+1]:.2f} us")
print(f"W row 3: {d[8]:.2f} us")
