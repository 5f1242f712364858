"""Per-hop account of k_backsolve from the stamped development build
(tools/chol_stamps.sh -> abvar/var_stamps.so, -DSFM_CHOL_STAMPS).  Per block
row b (s_memrealtime, 100 MHz): 0 the poll saw y_{b+1}, 1 after the barrier
that hands it to the block, 2 the FMA terms reduced into v, 3 after v's
barrier, 4 y_b stored.  The hop b+1 -> b is 0(b) - 4(b+1) (store to seen),
the block's own part 4(b) - 0(b).
  python tools/backsolve_phases.py [n] [reps]"""
import ctypes
import json
import os
import sys

import numpy as np

R = os.environ.get('GRAFT_REPO_ROOT', os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
os.environ.setdefault("SFM_AMD_LIB", os.path.join(R, "abvar", "var_stamps.so"))
from sfm_amd.ba import dense_spd_solve  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rng = np.random.default_rng(n)
B = rng.uniform(-1, 1, (n, n))
A = B + B.T
A[np.diag_indices(n)] += 2.0 * n
b = rng.standard_normal(n)
y, ms, fail = dense_spd_solve(A, b, reps=reps)
L = ctypes.CDLL(os.environ["SFM_AMD_LIB"])
L.sfm_debug_bstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * (256 * 8))()
assert L.sfm_debug_bstamps(buf, 256 * 8) == 0
st = np.array(buf[:], dtype=np.float64).reshape(256, 8) / 100.0  # us
nb = (n + 63) // 64
rows = list(range(1, nb - 2))  # blocks with a predecessor, away from the ends
hop = [st[r, 0] - st[r + 1, 4] for r in rows]
own = [st[r, 4] - st[r, 0] for r in rows]
parts = {
    "poll seen -> barrier passed": [st[r, 1] - st[r, 0] for r in rows],
    "barrier -> last term reduced into v": [st[r, 2] - st[r, 1] for r in rows],
    "v barrier": [st[r, 3] - st[r, 2] for r in rows],
    "W^T v + y store issued": [st[r, 4] - st[r, 3] for r in rows],
}
out = {"n": n, "ms_factor_plus_backsolve": round(ms, 4), "fail": fail, "blocks": nb,
       "chain_us (first store -> last store)": round(float(st[0, 4] - st[nb - 1, 4]), 2),
       "hop_us_median_p90": [round(float(np.median(hop)), 3), round(float(np.percentile(hop, 90)), 3)],
       "own_us_median": round(float(np.median(own)), 3),
       "own_parts_us_median": {k: round(float(np.median(v)), 3) for k, v in parts.items()}}
print(json.dumps(out, indent=1))
