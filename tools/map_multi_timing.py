"""Wall time of the BA gather (DeviceMap.getPointsInFrameMulti) on the live
loop's map after 300 frames: with the observation CSR current, and after an
append (the CSR is rebuilt), as in the live loop's BA after a keyframe."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from sfm_amd.live import KeypointStream, LiveSfM

s = LiveSfM(KeypointStream())
s.run(300)
frames = [kf.no for kf in s.kfs]
m = s.map
print("map size", m.size(), "keyframes", len(frames))
for label, dirty in (("csr current", False), ("after an append", True)):
    w = []
    for k in range(20):
        if dirty:
            m.addPointMatches([0], [0], 100000 + k)
        t0 = time.perf_counter()
        m.getPointsInFrameMulti(frames)
        w.append(time.perf_counter() - t0)
    print(f"{label}: median {np.median(w[3:]) * 1e3:.3f} ms")
w = []
for k in range(20):
    t0 = time.perf_counter()
    for f in frames:
        m.getPointsInFrame(f)
    w.append(time.perf_counter() - t0)
print(f"per-frame queries: median {np.median(w[3:]) * 1e3:.3f} ms")
s.close()
