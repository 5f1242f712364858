"""One-shot C3 solves (sfm_ba_solve from host arrays) with the set_problem
phase timer on (SFM_TIMING=1 prints the phases to stderr)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("SFM_TIMING", "1")
import sfm_amd
from sfm_amd import scene
cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
sc = scene.config(cfg)
for k in range(4):
    r, t, X = sc.copy_params()
    t0 = time.perf_counter()
    sm, _ = sfm_amd.solve(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, r, t, X)
    print(f"{cfg} one-shot {k}: {(time.perf_counter() - t0) * 1e3:.2f} ms, {sm.num_iterations} its, "
          f"cost {sm.final_cost:.6f}", file=sys.stderr, flush=True)
