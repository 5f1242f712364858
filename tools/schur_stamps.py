"""Per-workgroup timestamps of k_schur (needs tools/var_ss.so, an instrumented build)."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("SFM_AMD_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "var_ss.so"))
import sfm_amd
from sfm_amd import scene as S
from sfm_amd._ffi import lib
sc = S.config("C3")
ba = sfm_amd.BundleAdjuster(0)
ba.set_problem(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, sc.rot, sc.t, sc.X)
sm, _ = ba.solve()
buf = np.zeros(4 << 16, dtype=np.int64)
assert lib().sfm_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p)) == 0
nz = np.nonzero(buf[0::4])[0]
st = buf[:4 * (nz.max() + 1)].reshape(-1, 4).astype(np.float64)
print("workgroups", len(st))
for x in range(8):
    m = st[:, 3] == x
    if not m.any():
        continue
    s = st[m]
    t0 = s[:, 0].min()
    print(f"xcc {x}: n={m.sum()} span={s[:,2].max()-t0:.0f} main mean={np.mean(s[:,1]-s[:,0]):.0f} max={np.max(s[:,1]-s[:,0]):.0f} "
          f"tail mean={np.mean(s[:,2]-s[:,1]):.0f}  start q50={np.percentile(s[:,0]-t0,50):.0f} q90={np.percentile(s[:,0]-t0,90):.0f}")
