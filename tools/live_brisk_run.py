"""The live loop on device BRISK detections of the rendered synthetic video:
python tools/live_brisk_run.py [frames]."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sfm_amd.live import BriskVideoStream, LiveSfM  # noqa: E402
from sfm_amd.mapping import _rodrigues  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60
st = BriskVideoStream()
t0 = time.perf_counter()
frames = [st.frame(k) for k in range(n)]
t1 = time.perf_counter()
print("brisk ms/frame", round((t1 - t0) / n * 1e3, 2), "keypoints/frame", np.mean([len(f[0]) for f in frames]))
s = LiveSfM(st)
t2 = time.perf_counter()
for k in range(n):
    s.process(k, frames[k][0], frames[k][1])
dt = time.perf_counter() - t2
print("live fps", round(n / dt, 1), "stats", s.stats, "kfs", [f.no for f in s.kfs], "map", s.map.size(), "lost", s.lost)
C = np.array([-_rodrigues(f.rot).T @ f.t for f in s.kfs])
Cg = np.array([-_rodrigues(st.pose(f.no)[0]).T @ st.pose(f.no)[1] for f in s.kfs])
print("kf centres", np.round(C, 3).tolist())
print("gt centres", np.round(Cg, 3).tolist())
s.close()
