"""C5 pipeline dry run: frames through IncrementalMapper, per-keyframe BA sizes and pose errors."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sfm_amd.mapping import IncrementalMapper
from sfm_amd.video import SyntheticVideo
nf = int(sys.argv[1]) if len(sys.argv) > 1 else 61
v = SyntheticVideo()
frames = [v.frame(k) for k in range(nf)]
m = IncrementalMapper(v)
t0 = time.perf_counter()
for f in frames:
    m.process_frame(f)
wall = time.perf_counter() - t0
print(f"{nf} frames in {wall:.3f} s ({nf / wall:.1f} frames/s), keyframes {len(m.kf_frames)}, map points {m.X.shape[0]}, "
      f"pnp frames {m.pnp_frames}, times {m.times}")
for j, rec in enumerate(m.ba_log):
    sm = rec["summary"]
    print(f"BA {j}: cams {rec['rot'].shape[0]} pts {rec['X'].shape[0]} obs {len(rec['uv'])} its {sm.num_iterations} "
          f"cost {sm.initial_cost:.3f} -> {sm.final_cost:.3f}")
for j, k in enumerate(m.kf_frames):
    r, t = m.gt_pose(k)
    print(f"KF {j} frame {k}: |dr| {np.max(np.abs(m.kf_rot[j] - r)):.2e} |dt| {np.linalg.norm(m.kf_t[j] - t):.2e} |t| {np.linalg.norm(t):.2f}")
