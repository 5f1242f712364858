"""Tracker timing (C5 shape): push a 1280x720 frame + computeOpticalFlow of
500 points per step; prints per-phase device times and wall ms per frame."""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from sfm_amd import klt
from sfm_amd.video import SyntheticVideo

n_pts = int(sys.argv[1]) if len(sys.argv) > 1 else 500
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
v = SyntheticVideo()
frames = [v.frame(k) for k in range(3)]
rng = np.random.default_rng(0)
pts = [v.features(k, n_pts, rng) for k in range(3)]
dets = [v.detections(k, (k + 1) % 3, pts[k], rng) for k in range(3)]
tr = klt.KLTTracker(v.w, v.h)
tr.push_frame(frames[0])
ph = {"pyramid": 0.0, "lk": 0.0, "associate": 0.0}
for it in range(steps + 5):
    if it == 5:
        t0 = time.perf_counter()
        ph = {k: 0.0 for k in ph}
    k = (it + 1) % 3
    tr.push_frame(frames[k])
    pi, ci = tr.compute_optical_flow(pts[(k - 1) % 3], dets[(k - 1) % 3])
    for a, b in tr.phase_times().items():
        ph[a] += b
wall = (time.perf_counter() - t0) / steps
print(f"points {n_pts} matches {len(pi)} wall_ms_per_frame {wall*1e3:.3f} fps {1/wall:.1f} " +
      " ".join(f"{a}_ms {b/steps:.4f}" for a, b in ph.items()))
