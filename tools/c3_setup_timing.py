"""sfm_ba_set_problem wall time at C3, four times (SFM_TIMING=1 adds the
host phase breakdown on stderr):  SFM_TIMING=1 python tools/c3_setup_timing.py"""
import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np
import sfm_amd
from sfm_amd import scene as S
sc = S.config("C3")
ba = sfm_amd.BundleAdjuster(0)
for k in range(4):
    t0 = time.perf_counter()
    ba.set_problem(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, sc.rot, sc.t, sc.X)
    print("set_problem ms", (time.perf_counter() - t0) * 1e3, flush=True)
ba.close()
