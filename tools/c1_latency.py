"""Where the one-shot keyframe-sized solve spends its time (C1: 20 cams /
2k pts / 20k obs): handle creation, set_problem, the resident solve,
parameter download, destroy; then the resident solve alone."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import sfm_amd
from sfm_amd import scene as S

sc = S.config(os.environ.get("CFG", "C1"))
for rep in range(4):
    t = [time.perf_counter()]
    ba = sfm_amd.BundleAdjuster(0); t.append(time.perf_counter())
    ba.set_problem(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, sc.rot, sc.t, sc.X); t.append(time.perf_counter())
    sm, _ = ba.solve(); t.append(time.perf_counter())
    ba.parameters(); t.append(time.perf_counter())
    ba.close(); t.append(time.perf_counter())
    d = np.diff(t) * 1e3
    print("create %.3f set_problem %.3f solve %.3f params %.3f destroy %.3f ms" % tuple(d), flush=True)
ba = sfm_amd.BundleAdjuster(0)
ba.set_problem(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, sc.rot, sc.t, sc.X)
ba.solve()
ba.set_profiling(True)
t0 = time.perf_counter()
for _ in range(20):
    ba.reset(); sm, _ = ba.solve()
ba.sync()
print("resident solve %.3f ms, %d iterations" % ((time.perf_counter() - t0) / 20 * 1e3, sm.num_iterations))
print({k: round(v["ms"] / 20, 4) for k, v in ba.phase_times().items()})
