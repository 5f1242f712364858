"""Per-wave timestamps of k_jacobian (needs the tools/var_st.so instrumented build)."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("SFM_AMD_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "var_st.so"))
import sfm_amd
from sfm_amd import scene as S
from sfm_amd._ffi import lib
sc = S.config("C3")
ba = sfm_amd.BundleAdjuster(0)
ba.set_problem(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, sc.rot, sc.t, sc.X)
print("jacobian ms", ba.bench_jacobian(3))
buf = np.zeros(4 << 16, dtype=np.int64)
assert lib().sfm_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p)) == 0
nw = (sc.n_obs + 63) // 64
st = buf[:4 * nw].reshape(nw, 4).astype(np.float64)
t0 = st[:, 0].min()
span = st[:, 3].max() - t0
print(f"waves {nw} span {span:.0f} ticks")
for name, a, b in (("load", 0, 1), ("compute+store", 1, 2), ("reduce", 2, 3), ("life", 0, 3)):
    d = st[:, b] - st[:, a]
    print(f"{name:14s} mean {d.mean():8.0f} p10 {np.percentile(d,10):8.0f} p50 {np.percentile(d,50):8.0f} p90 {np.percentile(d,90):8.0f}")
starts = np.sort(st[:, 0] - t0)
print("start quantiles", [round(float(np.percentile(starts, q))) for q in (1, 10, 25, 50, 75, 90, 99)])
ends = np.sort(st[:, 3] - t0)
print("end quantiles", [round(float(np.percentile(ends, q))) for q in (1, 10, 25, 50, 75, 90, 99)])
