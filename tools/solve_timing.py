"""Median wall time of resident solves (reset + solve) at a BASELINE config:
    python tools/solve_timing.py C3 [reps]   (SFM_LM_BATCH / SFM_HOST_LM select the loop)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import sfm_amd
from sfm_amd import scene as S

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
sc = S.config(cfg)
ba = sfm_amd.BundleAdjuster(0)
ba.set_problem(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, sc.rot, sc.t, sc.X)
w = []
for k in range(reps + 2):
    ba.reset()
    ba.sync()
    t0 = time.perf_counter()
    sm, _ = ba.solve()
    w.append(time.perf_counter() - t0)
print(f"{cfg} batch={os.environ.get('SFM_LM_BATCH', '4')} host={os.environ.get('SFM_HOST_LM', '0')}: "
      f"solve median {np.median(w[2:]) * 1e3:.3f} ms, iterations {sm.num_iterations}, cost {sm.final_cost.hex()}")
ba.close()
