"""A/B workload: C3 set_problem + 3 resident solves; prints the final cost
bits so ablation builds (SFM_AMD_LIB) can be checked bitwise against base."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sfm_amd
from sfm_amd import scene as S

sc = S.config("C3")
ba = sfm_amd.BundleAdjuster(0)
ba.set_problem(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, sc.rot, sc.t, sc.X)
for _ in range(3):
    ba.reset()
    sm, _ = ba.solve()
print("final_cost", sm.final_cost.hex(), "iters", sm.num_iterations)
ba.close()
