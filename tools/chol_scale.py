"""Dense reduced-camera Cholesky (factor + solve, sfm_dense_spd_solve) at the
reduced-system sizes of C3 (n=3000) and C4 (n=12000) and between; SPD by
diagonal dominance (no O(n^3) host product).  Error vs a host solve is
checked only where numpy finishes quickly."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sfm_amd.ba import dense_spd_solve
for n in [int(a) for a in sys.argv[1:]] or [3000, 6000, 12000]:
    rng = np.random.default_rng(n)
    B = rng.uniform(-1, 1, (n, n))
    A = B + B.T
    A[np.diag_indices(n)] += 2.0 * n
    b = rng.standard_normal(n)
    y, ms, fl = dense_spd_solve(A, b, reps=3)
    r = A @ y - b
    tf = n ** 3 / 3 / (ms * 1e-3) / 1e12
    print(f"n={n} ms={ms:.3f} fail={fl} TF/s={tf:.2f} rel_resid={np.abs(r).max() / np.abs(b).max():.2e}", flush=True)
