"""Phase times of k_pnp_epnp from the stamped variant (tools/mkvar.sh pstamps
"$(cat tools/patch_pnp_stamps.py)" pnp_kernels.hip): one solvePnPRansac call
on the bench's pnp scene (20 hypotheses), per phase median / max over the
hypotheses' waves, in us (s_memrealtime, 100 MHz)."""
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
lib = _ffi.lib()
buf = (ctypes.c_ulonglong * (64 * 3 * 8))()
assert lib.sfm_debug_pstamps(buf, 64 * 3 * 8) == 0
st = np.array(buf, dtype=np.float64).reshape(64, 3, 8)[:20]
t0 = st[:, :, 0]
names = ["start -> M^T M", "12x12 SVD", "rest of common", "beta case (wave w)"]
print("k_pnp_epnp phases (us, 20 hypotheses; median / max):")
for i, (a, b) in enumerate([(0, 1), (1, 2), (2, 3), (3, 4)]):
    d = (st[:, :, b] - st[:, :, a]) / 100.0
    if i < 3:
        print(f"  {names[i]:22s} {np.median(d):7.2f} / {d.max():7.2f}")
    else:
        for w in range(3):
            print(f"  case N={w} (wave {w})       {np.median(d[:, w]):7.2f} / {d[:, w].max():7.2f}")
tot = (st[:, :, 4] - st[:, :, 0]).max(axis=1) / 100.0
print(f"  hypothesis total       {np.median(tot):7.2f} / {tot.max():7.2f}   (spread of starts {(t0.max() - t0.min()) / 100.0:.2f} us)")
