"""Workload for PMC passes on C3.  argv[1]: "jac" = 10 record-writing Jacobian
passes (the bench's k_jacobian roofline object), "solve" = one full solve
(the record-free production path), "all" (default) = both."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sfm_amd
from sfm_amd import scene as S

what = sys.argv[1] if len(sys.argv) > 1 else "all"
# the host-driven LM loop: the device-driven one also enqueues phases its
# flags then skip, whose near-empty launches would enter the per-launch means
os.environ["SFM_HOST_LM"] = "1"
sc = S.config("C3")
ba = sfm_amd.BundleAdjuster(0)
ba.set_problem(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, sc.rot, sc.t, sc.X)
if what in ("jac", "all"):
    print("jacobian ms", ba.bench_jacobian(10))
if what in ("solve", "all"):
    sm, _ = ba.solve()
    print("iters", sm.num_iterations)
ba.close()
