"""Phases of k_pnp_epnp's beta cases from tools/patch_pnp_stamps2.py's variant."""
import ctypes, os, sys
import numpy as np
R = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["SFM_AMD_LIB"] = os.path.join(R, "tools", "var_pstamps.so")
sys.path.insert(0, R)
import sfm_amd
from sfm_amd import _ffi
from tests.pnp_cases import K, scene
X, uv, _, _ = scene(500, 77, noise=0.5, outliers=0.3)
for _ in range(3):
    sfm_amd.solvePnPRansac(X, uv, K)
buf = (ctypes.c_ulonglong * (64 * 3 * 8))()
assert _ffi.lib().sfm_debug_pstamps(buf, 64 * 3 * 8) == 0
st = np.array(buf, dtype=np.float64).reshape(64, 3, 8)[:20]
for w in range(3):
    d = [(st[:, w, b] - st[:, w, a]) / 100.0 for a, b in [(0, 1), (1, 2), (2, 3)]]
    print(f"case N={w}: least squares {np.median(d[0]):6.2f}  Gauss-Newton {np.median(d[1]):6.2f}  R,t + error {np.median(d[2]):6.2f} us (median over 20 hypotheses)")
