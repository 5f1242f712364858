"""Workload for PMC passes: C3 problem, 10 Jacobian passes + one full solve."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sfm_amd
from sfm_amd import scene as S

sc = S.config("C3")
ba = sfm_amd.BundleAdjuster(0)
ba.set_problem(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, sc.rot, sc.t, sc.X)
print("jacobian ms", ba.bench_jacobian(10))
sm, _ = ba.solve()
print("iters", sm.num_iterations)
ba.close()
