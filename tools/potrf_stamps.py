"""Phase stamps of k_chol_potrf (tile 5) from the instrumented build tools/var_cs.so."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("SFM_AMD_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "var_cs.so"))
from sfm_amd.ba import dense_spd_solve
from sfm_amd._ffi import lib
n = 3000
rng = np.random.default_rng(0)
M = rng.standard_normal((n, n)); A = M @ M.T + n * np.eye(n); b = rng.standard_normal(n)
y, ms, fl = dense_spd_solve(A, b, reps=2)
buf = np.zeros(16, dtype=np.int64)
assert lib().sfm_debug_pstamps(buf.ctypes.data_as(ctypes.c_void_p)) == 0
names = ["load", "panel0", "trail0", "panel1", "trail1", "panel2", "trail2", "panel3", "trail3", "Wdiag", "Woff", "store"]
d = np.diff(buf[:13])
print("total", buf[12] - buf[0], " ".join(f"{nm}={v}" for nm, v in zip(names, d)))
