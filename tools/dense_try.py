import time, numpy as np, sys
sys.path.insert(0, '/root/repo')
import sfm_amd, sfm_amd.ba
from sfm_amd import _ffi
for n in (100, 1000, 3000):
    rng = np.random.default_rng(n)
    M = rng.standard_normal((n, n)); A = M @ M.T + n * np.eye(n); b = rng.standard_normal(n)
    t0 = time.time()
    y, ms, fail = sfm_amd.ba.dense_spd_solve(A, b, reps=5)
    print(n, 'fail', fail, 'ms', ms, 'err', None if y is None else float(np.max(np.abs(A @ y - b))), 'wall', time.time() - t0, flush=True)
