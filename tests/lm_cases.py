"""Seeded bundle-adjustment problems that force every branch of Ceres-1.12's
Levenberg-Marquardt trust-region loop, the
loop behind ceres::Solve in CTracker::bundleAdjustmentStructAndPose
(/root/reference/CTracker.cpp:670-702, options :571-577).

Shared by tests/golden/make_lm_branches.py (which commits the oracle traces
and cross-checks them against a dense numpy restatement of the loop),
tests/test_lm_branches_oracle.py (CPU: the oracle against those fixtures) and
tests/test_gpu_lm_branches.py (GPU: the HIP solver against the oracle).

Every case is small (12 cameras / 600 points / 6 views = 3600 observations,
or fewer) so the oracle solves it in milliseconds.  Branches covered:

  reject_*          rejected steps (rho <= min_relative_decrease): radius /=
                    decrease_factor, decrease_factor *= 2, diagonal reused;
                    several consecutive rejections, then recovery
  no_convergence    max_num_iterations reached -> NO_CONVERGENCE
  min_radius        radius < min_trust_region_radius after a rejection
  parameter_tol     |dx| <= parameter_tolerance (|x| + parameter_tolerance)
  gradient_tol      max|g| <= gradient_tolerance after an accepted step
  gradient_initial  max|g| <= gradient_tolerance at iteration 0 (no step)
  llt_invalid*      LLT failure of the reduced camera matrix (an exactly
                    zero row: a camera that sees only points on its optical
                    axis has zero Jacobian columns for t_z and rot_z, and
                    min_lm_diagonal = 0 leaves them undamped) -> invalid
                    steps, max_num_consecutive_invalid_steps -> FAILURE
  max_diag          max_lm_diagonal clamps the LM diagonal from above
  no_jacobi         jacobi_scaling = false
  min_rel_decrease  a stricter acceptance threshold
  struct_only / pose_only on the rejecting scene (BA_TYPE 0 / 1,
                    CTracker.cpp:679-687)
  gauge_*           long runs with every tolerance 0 from a trust region of
                    1e15 / 1e16 (the max_trust_region_radius clamp): after
                    the first accepted steps the cost changes are rounding
                    noise and the 7-DoF similarity gauge (nothing is held
                    constant, CTracker.cpp:676-696) is regularised only by
                    D^2 = diag / 1e16, so accept / reject decisions and the
                    raw parameters differ between any two correct fp64
                    implementations; these cases are compared on the
                    decisive prefix plus gauge-invariant quantities (SURVEY.md
                    §7 hard part 2)
"""
from __future__ import annotations

import numpy as np

from sfm_amd import scene

SEED = 0x5F3D2017

# (seed offset, pt_sigma, rot_sigma, t_sigma) of the rejecting scenes, found
# by scanning seeds with the oracle (see make_lm_branches.py)
REJECT_SCENES = {
    "reject_a": (204, 1.0, 0.3, 2.0),   # A A R R R A A A A A A A (function tol)
    "reject_b": (200, 0.8, 0.5, 3.0),   # 8 A, 3 R, 6 A
    "reject_c": (205, 0.8, 0.5, 3.0),   # A A A A R R R R A A A R R A ... (24 iterations)
}


def reject_scene(name: str):
    off, ps, rs, ts = REJECT_SCENES[name]
    return scene.generate(12, 600, views=6, seed=SEED + off, pt_sigma=ps, rot_sigma=rs, t_sigma=ts)


def on_axis_scene(n_axis: int = 5):
    """Camera 0 (rot = 0, t = (0, 0, 8): the reference's first keyframe)
    keeps only `n_axis` observations, of points placed exactly on its optical
    axis (X = (0, 0, z)).  Its Jacobian columns for rot_z and t_z are then
    exactly zero: d(w x X)/dw_z = e_z x X = 0 and dr/dt_z ~ (p_x, p_y) = 0."""
    s = scene.generate(10, 300, views=5, seed=SEED + 300, pt_sigma=0.05, rot_sigma=0.01, t_sigma=0.05)
    s.rot[0] = 0.0
    s.t[0] = [0.0, 0.0, 8.0]
    cam0 = np.flatnonzero(s.cam_idx == 0)
    keep_pts = np.unique(s.pt_idx[cam0])[:n_axis]
    drop = cam0[~np.isin(s.pt_idx[cam0], keep_pts)]
    keep = np.ones(s.n_obs, bool)
    keep[drop] = False
    s.uv, s.cam_idx, s.pt_idx = s.uv[keep].copy(), s.cam_idx[keep].copy(), s.pt_idx[keep].copy()
    zs = np.linspace(-0.8, 0.8, len(keep_pts))
    for p, z in zip(keep_pts, zs):
        s.X[p] = [0.0, 0.0, z]
    return s


def cases():
    """name -> (scene builder, options overrides, mode).  Options overrides
    that depend on a reference trajectory are resolved by resolve()."""
    c = {}
    for name in REJECT_SCENES:
        c[name] = (lambda n=name: reject_scene(n), {}, 2)
    a = lambda: reject_scene("reject_a")
    c["no_convergence"] = (a, {"max_num_iterations": 4}, 2)
    c["min_radius"] = (a, {"min_trust_region_radius": "after_first_reject"}, 2)
    c["parameter_tol"] = (a, {"function_tolerance": 0.0, "parameter_tolerance": "between_steps"}, 2)
    c["gradient_tol"] = (a, {"gradient_tolerance": "between_gradients"}, 2)
    c["gradient_initial"] = (a, {"gradient_tolerance": 1e20}, 2)
    c["llt_invalid"] = (on_axis_scene, {"min_lm_diagonal": 0.0}, 2)
    c["llt_invalid_3"] = (on_axis_scene, {"min_lm_diagonal": 0.0, "max_num_consecutive_invalid_steps": 3}, 2)
    c["llt_invalid_pose"] = (on_axis_scene, {"min_lm_diagonal": 0.0}, 1)
    c["max_diag"] = (a, {"max_lm_diagonal": 1e3}, 2)
    c["no_jacobi"] = (a, {"jacobi_scaling": 0}, 2)
    c["min_rel_decrease"] = (lambda: reject_scene("reject_b"), {"min_relative_decrease": 0.5}, 2)
    c["struct_only"] = (a, {}, 0)
    c["pose_only"] = (a, {}, 1)
    g = lambda: scene.generate(12, 600, views=6, seed=SEED + 400)
    loose = {"function_tolerance": 0.0, "gradient_tolerance": 0.0, "parameter_tolerance": 0.0}
    c["gauge_1e15"] = (g, dict(loose, initial_trust_region_radius=1e15), 2)
    c["gauge_1e16"] = (g, dict(loose, initial_trust_region_radius=1e16), 2)
    return c


def decisive_prefix(trace, rel: float = 1e-6) -> int:
    """Leading iterations (after iteration 0) whose outcome no rounding can
    flip: valid steps that change the cost by more than rel * cost."""
    k = 0
    for it in trace[1:]:
        if not it["step_is_valid"] or abs(it["cost_change"]) <= rel * it["cost"]:
            break
        k += 1
    return k


def x_norm(rot, t, X) -> float:
    """|x| over all parameter blocks (the parameter-tolerance scale)."""
    return float(np.sqrt(np.sum(rot ** 2) + np.sum(t ** 2) + np.sum(X ** 2)))


def camera_centres(rot, t):
    """c = -R^T t per camera (angle-axis rot, ceres convention)."""
    from scipy.spatial.transform import Rotation
    R = Rotation.from_rotvec(np.asarray(rot)).as_matrix()
    return -np.einsum("cji,cj->ci", R, np.asarray(t))


def sim3_align(src, dst):
    """Umeyama: (s, R, t) minimising |s R src + t - dst|^2 over rows."""
    mu_s, mu_d = src.mean(0), dst.mean(0)
    a, b = src - mu_s, dst - mu_d
    U, S, Vt = np.linalg.svd(b.T @ a / len(src))
    E = np.eye(3)
    if np.linalg.det(U) * np.linalg.det(Vt) < 0:
        E[2, 2] = -1
    R = U @ E @ Vt
    s = np.trace(np.diag(S) @ E) / (a * a).sum(1).mean()
    return s, R, mu_d - s * R @ mu_s


def gauge_invariant_diff(residual_fn, sc, sol_a, sol_b, extent=False):
    """Gauge-invariant distances between two solutions (rot, t, X) of scene
    `sc`: max |r_a - r_b| over observation residuals (pixels), and the max
    relative distance of camera centres + points after a Sim(3) alignment
    of a onto b (SURVEY.md §7 hard part 2) -- per coordinate (floor 1e-3),
    or with `extent` as max |a - b| over the scene's RMS radius about its
    centroid (for scenes whose first camera sits at the origin, where a
    per-coordinate ratio divides rounding by the floor)."""
    ra = residual_fn(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, *sol_a)
    rb = residual_fn(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, *sol_b)
    pa = np.vstack([camera_centres(sol_a[0], sol_a[1]), sol_a[2]])
    pb = np.vstack([camera_centres(sol_b[0], sol_b[1]), sol_b[2]])
    s, R, t = sim3_align(pa, pb)
    al = s * pa @ R.T + t
    if extent:
        radius = float(np.sqrt(np.mean(np.sum((pb - pb.mean(axis=0)) ** 2, axis=1))))
        return float(np.max(np.abs(ra - rb))), float(np.max(np.linalg.norm(al - pb, axis=1)) / radius)
    return float(np.max(np.abs(ra - rb))), float(np.max(np.abs(al - pb) / np.maximum(np.abs(pb), 1e-3)))
