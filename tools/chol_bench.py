import sys, numpy as np
import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sfm_amd.ba import dense_spd_solve
n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
rng = np.random.default_rng(0)
M = rng.standard_normal((n, n)); A = M @ M.T + n * np.eye(n); b = rng.standard_normal(n)
y, ms, fl = dense_spd_solve(A, b, reps=4)
print(f"n={n} ms={ms:.3f} fail={fl} err={np.abs(y-np.linalg.solve(A,b)).max():.2e}")
