"""Run the live (BRISK-path) driver on the synthetic keypoint stream and
print its statistics: python tools/live_run.py [frames]."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sfm_amd.live import LiveSfM, KeypointStream  # noqa: E402
from sfm_amd.mapping import _rodrigues  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 120
s = LiveSfM(KeypointStream())
t0 = time.perf_counter()
s.run(n)
dt = time.perf_counter() - t0
print("frames", n, "s", round(dt, 3), "fps", round(n / dt, 1))
print("stats", s.stats, "kfs", [f.no for f in s.kfs], "map", s.map.size())
print("times", {k: round(v, 3) for k, v in s.times.items()})
err = []
for f in s.kfs:
    r, t = s.stream.pose(f.no)
    c_gt = -_rodrigues(r).T @ t
    c = -_rodrigues(f.rot).T @ f.t
    err.append(np.linalg.norm(c - c_gt))
print("kf centre error (no alignment)", np.round(err, 4).tolist())
for rec in s.ba_log[-3:]:
    sm = rec["summary"]
    print("ba", rec["uv"].shape[0], "obs", rec["X"].shape[0], "pts", len(rec["rot"]), "cams", "iters", sm.num_iterations,
          "cost", sm.initial_cost, "->", sm.final_cost)
s.close()
