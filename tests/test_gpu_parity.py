"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Tolerances (north star, BASELINE.json): pose / point parameters within 1e-6
relative after a full solve; residual + Jacobian within 1e-10 relative per
observation (same fp64 formula, different operation order); matcher indices
bit-exact.
"""
import numpy as np
import pytest

import sfm_amd
from sfm_amd import scene
from oracle import ffi as O

pytestmark = pytest.mark.gpu


def _rel(a, b, floor=1e-12):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), floor)))


def test_device_visible():
    assert sfm_amd.device_count() >= 1


@pytest.mark.parametrize("cfg", ["C1"])
def test_residual_jacobian_parity(cfg):
    s = scene.config(cfg)
    with sfm_amd.BundleAdjuster() as ba:
        ba.set_problem(s.uv, s.cam_idx, s.pt_idx, s.K, s.rot, s.t, s.X)
        cost, res, jac = ba.evaluate()
    r_o, j_o = O.residuals_jacobians(s.uv, s.cam_idx, s.pt_idx, s.K, s.rot, s.t, s.X)
    assert np.max(np.abs(res - r_o)) < 1e-9
    scale = np.maximum(np.abs(j_o).max(axis=(1, 2), keepdims=True), 1e-300)
    assert np.max(np.abs(jac - j_o) / scale) < 1e-10
    assert abs(cost - 0.5 * np.sum(r_o ** 2)) <= 1e-10 * cost


def test_small_angle_branch_jacobian():
    # camera 0 sits at rot = 0 exactly (first keyframe): theta^2 <= DBL_EPSILON branch
    s = scene.generate(4, 50, views=4, seed=7)
    s.rot[1] = [1e-9, -2e-9, 5e-10]            # still first-order branch
    s.rot[2] = [1.5e-8, 0.0, 0.0]              # theta^2 = 2.25e-16 > DBL_EPSILON: Rodrigues
    with sfm_amd.BundleAdjuster() as ba:
        ba.set_problem(s.uv, s.cam_idx, s.pt_idx, s.K, s.rot, s.t, s.X)
        _, res, jac = ba.evaluate()
    r_o, j_o = O.residuals_jacobians(s.uv, s.cam_idx, s.pt_idx, s.K, s.rot, s.t, s.X)
    assert np.max(np.abs(res - r_o)) < 1e-9
    scale = np.maximum(np.abs(j_o).max(axis=(1, 2), keepdims=True), 1e-300)
    assert np.max(np.abs(jac - j_o) / scale) < 1e-9


@pytest.mark.parametrize("cfg", ["C1"])
def test_full_solve_parity(cfg):
    s = scene.config(cfg)
    r_o, t_o, X_o = s.copy_params()
    sm_o, tr_o = O.solve(s.uv, s.cam_idx, s.pt_idx, s.K, r_o, t_o, X_o)
    r_g, t_g, X_g = s.copy_params()
    sm_g, tr_g = sfm_amd.solve(s.uv, s.cam_idx, s.pt_idx, s.K, r_g, t_g, X_g)
    assert sm_g.termination_type == sm_o["termination_type"]
    assert sm_g.num_iterations == sm_o["num_iterations"]
    assert [t["step_is_successful"] for t in tr_g] == [t["step_is_successful"] for t in tr_o]
    assert abs(sm_g.final_cost - sm_o["final_cost"]) <= 1e-9 * sm_o["final_cost"]
    for a, b in zip(tr_g, tr_o):
        assert abs(a["cost"] - b["cost"]) <= 1e-9 * b["cost"]
        assert abs(a["trust_region_radius"] - b["trust_region_radius"]) <= 1e-6 * b["trust_region_radius"]
    assert _rel(X_g, X_o, 1e-3) < 1e-6
    assert _rel(t_g, t_o, 1e-3) < 1e-6
    assert _rel(r_g, r_o, 1e-3) < 1e-6


def test_matcher_bit_exact():
    rng = np.random.default_rng(1234)
    for n0, n1 in [(300, 280), (1000, 1200), (5, 2), (64, 65)]:
        d0 = rng.integers(0, 256, (n0, 64), dtype=np.uint8)
        d1 = rng.integers(0, 256, (n1, 64), dtype=np.uint8)
        # plant true correspondences with small descriptor noise and motion
        k = min(n0, n1) // 2
        d1[:k] = d0[:k]
        flip = rng.integers(0, 64, (k, 4))
        for r in range(k):
            d1[r, flip[r]] ^= 1
        p0 = rng.uniform(0, 1280, (n0, 2))
        p1 = rng.uniform(0, 1280, (n1, 2))
        p1[:k] = p0[:k] + rng.normal(0, 8, (k, 2))
        tr = sfm_amd.CTracker()
        g0, g1 = tr.matchFeatures(p0, d0, p1, d1)
        o0, o1 = O.match_features(p0, d0, p1, d1)
        assert np.array_equal(g0, o0) and np.array_equal(g1, o1)
        kg = tr.knnMatch2(d0, d1)
        ko = O.knn2(d0, d1)
        for a, b in zip(kg, ko):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("path", ["fused", "stepwise"])
@pytest.mark.parametrize("n", [6, 63, 64, 65, 130, 600, 3000])
def test_dense_cholesky_solve(n, path, monkeypatch):
    """Both factorisations: the persistent single-launch one (default) and
    the three-launches-per-column one (SFM_CHOL_STEPWISE=1)."""
    from sfm_amd.ba import dense_spd_solve
    if path == "stepwise":
        monkeypatch.setenv("SFM_CHOL_STEPWISE", "1")
    rng = np.random.default_rng(n)
    M = rng.standard_normal((n, n))
    A = M @ M.T + n * np.eye(n)
    b = rng.standard_normal(n)
    y, ms, fl = dense_spd_solve(A, b, reps=3 if n >= 600 else 1)
    assert fl == 0
    ref = np.linalg.solve(A, b)
    assert np.max(np.abs(y - ref)) <= 1e-10 * np.max(np.abs(ref))
    print(f"n={n}: {ms:.3f} ms per factor+solve")


@pytest.mark.parametrize("path", ["fused", "stepwise"])
@pytest.mark.parametrize("n", [100, 700])
def test_dense_cholesky_reports_indefinite(n, path, monkeypatch):
    from sfm_amd.ba import dense_spd_solve
    if path == "stepwise":
        monkeypatch.setenv("SFM_CHOL_STEPWISE", "1")
    A = np.eye(n)
    A[n // 2, n // 2] = -1.0
    _, _, fl = dense_spd_solve(A, np.ones(n))
    assert fl == 1


def test_small_system_factor_bitwise_equals_persistent():
    """k_chol_small (nblk <= 2: factor + back substitution in one workgroup)
    repeats the persistent walker's and k_backsolve's arithmetic in the same
    order: y bitwise equal to the persistent pair's (SFM_CHOL_NO_SMALL=1, a
    child process: the knob is read once per process)."""
    import json, os, subprocess, sys
    from sfm_amd.ba import dense_spd_solve
    sizes = [6, 63, 64, 100, 127]
    code = ("import json, numpy as np\n"
            "from sfm_amd.ba import dense_spd_solve\n"
            "out = {}\n"
            f"for n in {sizes}:\n"
            "    rng = np.random.default_rng(n)\n"
            "    M = rng.standard_normal((n, n)); A = M @ M.T + n * np.eye(n); b = rng.standard_normal(n)\n"
            "    out[n] = dense_spd_solve(A, b)[0].tobytes().hex()\n"
            "print(json.dumps(out))\n")
    env = dict(os.environ, SFM_CHOL_NO_SMALL="1")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    ref = json.loads(r.stdout.strip().splitlines()[-1])
    for n in sizes:
        rng = np.random.default_rng(n)
        M = rng.standard_normal((n, n))
        A = M @ M.T + n * np.eye(n)
        b = rng.standard_normal(n)
        y = dense_spd_solve(A, b)[0]
        assert y.tobytes().hex() == ref[str(n)], n


def test_schur_cholesky_overlap_bitwise(monkeypatch):
    """SFM_OVERLAP=1 (opt-in, read at set_problem): the off-diagonal Schur
    pass beside the factorisation on a second stream, half the CUs each.
    Same S tiles, same factor order: the solve bitwise equal to the default
    one-stream schedule (60 cameras: a 6-tile reduced system)."""
    s = scene.generate(60, 3000, views=6, seed=11)
    runs = []
    for ov in ("0", "1"):
        monkeypatch.setenv("SFM_OVERLAP", ov)
        r, t, X = s.copy_params()
        sm, tr = sfm_amd.solve(s.uv, s.cam_idx, s.pt_idx, s.K, r, t, X)
        runs.append((sm.final_cost, sm.num_iterations, r, t, X))
    (c0, n0, *p0), (c1, n1, *p1) = runs
    assert n0 == n1 and n0 >= 1
    assert c0 == c1
    for a, b in zip(p0, p1):
        assert a.tobytes() == b.tobytes()
