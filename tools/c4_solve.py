"""BASELINE config C4 (2000 cams / 1M points / 10M obs) on ONE MI355X: the
whole problem fits in one GPU's HBM (288 GB), so the single-GPU solve is the
reference point for the 8-GPU landmark-sharded run.  Prints setup time, one
full solve (LM to Ceres' termination), phase times and the Cholesky rate
(n = 12000, the MFMA-bound regime)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sfm_amd
from sfm_amd import scene as S

t0 = time.perf_counter()
sc = S.config("C4")
t1 = time.perf_counter()
print(f"scene {sc.n_cams} cams {sc.n_pts} pts {sc.n_obs} obs generated in {t1 - t0:.1f} s", flush=True)
ba = sfm_amd.BundleAdjuster(0)
ba.set_problem(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, sc.rot, sc.t, sc.X)
t2 = time.perf_counter()
print(f"set_problem {t2 - t1:.1f} s", flush=True)
sm, tr = ba.solve()  # warm
ba.reset()
ba.set_profiling(True)
ba.sync()
t3 = time.perf_counter()
sm, tr = ba.solve()
ba.sync()
t4 = time.perf_counter()
ph = ba.phase_times()
n = 6 * sc.n_cams
chol = ph["cholesky"]
chol_ms = chol["ms"] / max(1, chol["count"])
out = {"config": "C4", "cams": sc.n_cams, "points": sc.n_pts, "observations": sc.n_obs,
       "solve_ms": (t4 - t3) * 1e3, "lm_iterations": sm.num_iterations,
       "residual_evals": sm.num_residual_evaluations, "initial_cost": sm.initial_cost, "final_cost": sm.final_cost,
       "termination": sm.termination_type,
       "residual_evals_per_s": sc.n_obs * sm.num_residual_evaluations / (t4 - t3),
       "costs": [t["cost"] for t in tr],
       "cholesky_ms": chol_ms, "cholesky_tflops": n ** 3 / 3 / (chol_ms * 1e-3) / 1e12,
       "phase_ms": {k: round(v["ms"], 3) for k, v in ph.items()}}
print(json.dumps(out), flush=True)
ba.close()
