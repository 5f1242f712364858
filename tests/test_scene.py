"""CPU: synthetic scene generator properties."""
import numpy as np

from sfm_amd import scene


def test_first_keyframe_and_intrinsics():
    s = scene.config("C1")
    assert np.array_equal(s.rot[0], [0.0, 0.0, 0.0])          # CFrame.cpp:229-235
    assert np.array_equal(s.rot_true[0], [0.0, 0.0, 0.0])
    assert np.array_equal(s.t_true[0], [0.0, 0.0, 8.0])
    assert s.K[0, 0] == 1072.606693272117800 and s.K[0, 4] == 1067.197515608619600   # main.cpp:47-50
    assert s.K[0, 2] == 648.780750477178910 and s.K[0, 5] == 364.503435962496890


def test_observation_layout():
    s = scene.generate(30, 500, views=10, seed=3)
    assert s.n_obs == 5000
    key = s.pt_idx.astype(np.int64) * 1000 + s.cam_idx
    assert np.all(np.diff(key) > 0)                 # sorted by (point, camera), distinct cameras per point
    assert np.all((s.uv[:, 0] > 0) & (s.uv[:, 0] < 1280) & (s.uv[:, 1] > 0) & (s.uv[:, 1] < 720))
    assert np.all(np.abs(s.X_true) <= 1.0)


def test_deterministic_and_shardable():
    a = scene.generate(12, 300, views=5, seed=11)
    b = scene.generate(12, 300, views=5, seed=11)
    for f in ("uv", "cam_idx", "X", "rot", "t"):
        assert np.array_equal(getattr(a, f), getattr(b, f))
    # a point range generated alone equals the same slice of the whole scene
    lo = scene.generate(12, 300, views=5, seed=11, p_begin=100, p_end=220)
    sel = (a.pt_idx >= 100) & (a.pt_idx < 220)
    assert np.array_equal(lo.uv, a.uv[sel])
    assert np.array_equal(lo.cam_idx, a.cam_idx[sel])
    assert np.array_equal(lo.pt_idx + 100, a.pt_idx[sel])
    assert np.array_equal(lo.X, a.X[100:220])
    assert np.array_equal(lo.rot, a.rot) and np.array_equal(lo.t, a.t)
