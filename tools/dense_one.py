import sys, time, numpy as np
sys.path.insert(0, '/root/repo')
import sfm_amd.ba
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
rng = np.random.default_rng(n)
M = rng.standard_normal((n, n)); A = M @ M.T + n * np.eye(n); b = rng.standard_normal(n)
t0 = time.time()
y, ms, fail = sfm_amd.ba.dense_spd_solve(A, b, reps=1)
print(n, 'fail', fail, 'ms', ms, 'err', float(np.max(np.abs(A @ y - b))), 'wall', time.time() - t0, flush=True)
