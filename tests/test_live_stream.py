"""CPU: the synthetic detector stream of the live driver (sfm_amd.live) is
self-consistent (keypoints are the ground-truth projections, descriptors
within the bit noise of their landmark's), and the restated filterMatches
keeps true correspondences and drops wrong ones."""
import numpy as np

from sfm_amd.live import KeypointStream, _filter_matches, _Frame, _project
from sfm_amd.mapping import _rodrigues


def test_keypoints_are_noisy_ground_truth_projections():
    s = KeypointStream(n_landmarks=800, seed=3)
    for k in (0, 17):
        pts, desc, lid = s.frame(k)
        real = lid >= 0
        r, t = s.pose(k)
        uv, z = _project(s.K, r, t, s.L[lid[real]])
        assert np.all(z > 0)
        err = np.linalg.norm(pts[real] - uv, axis=1)
        assert np.sqrt(np.mean(err ** 2)) < 0.6          # 0.3 px per axis
        ham = np.unpackbits(desc[real] ^ s.D[lid[real]], axis=1).sum(1)
        assert ham.max() <= s.bit_noise                   # flips may repeat a bit
        assert 0.1 < (~real).mean() / max(real.mean(), 1e-9) < 0.2


def test_frames_are_deterministic_and_move_about_2px():
    s = KeypointStream(n_landmarks=500, seed=5)
    a, b = s.frame(4), s.frame(4)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    r0, t0 = s.pose(10)
    r1, t1 = s.pose(11)
    uv0, _ = _project(s.K, r0, t0, s.L)
    uv1, _ = _project(s.K, r1, t1, s.L)
    d = np.median(np.linalg.norm(uv1 - uv0, axis=1))
    assert 1.5 < d < 4.0   # inside the frame-to-frame match window (1.5, 40)


def test_filter_matches_keeps_true_and_drops_wrong_pairs():
    s = KeypointStream(n_landmarks=400, seed=9)
    f0, f1 = _Frame(0, np.zeros((0, 2)), None), _Frame(12, np.zeros((0, 2)), None)
    f0.rot, f0.t = s.pose(0)
    f1.rot, f1.t = s.pose(12)
    X = s.L
    uv0, z0 = _project(s.K, f0.rot, f0.t, X)
    uv1, z1 = _project(s.K, f1.rot, f1.t, X)
    ok = _filter_matches(s.K, f0, f1, uv0, uv1, X, 7.0)
    assert ok.all()
    wrong = np.roll(uv1, 7, axis=0)
    ok2 = _filter_matches(s.K, f0, f1, uv0, wrong, X, 7.0)
    assert ok2.mean() < 0.2
    behind = X.copy()
    behind[:, 2] *= -1
    assert not _filter_matches(s.K, f0, f1, uv0, uv1, behind, 7.0).any()
    assert np.allclose(_rodrigues(f0.rot), np.eye(3))


def test_pair_frame_observations_recovers_each_observation():
    """live._bundle_adjust's pairing of getPointsInFrame's 3D and 2D lists
    (points matched two and three times in one frame: k^2 2D entries) gives
    every observation its own 2D index, in the frame's emplace order."""
    from oracle.cmap_oracle import CMapOracle
    from sfm_amd.live import pair_frame_observations
    m = CMapOracle()
    m.addNewPoints(np.zeros((6, 3)), [[10, 11, 12, 13, 14, 15]], [0])
    adds = [([0, 1, 2], [20, 21, 22]), ([1], [30]), ([3, 1, 4], [40, 41, 42]), ([5], [50])]
    truth = []
    for pts, uv in adds:
        m.addPointMatches(pts, uv, 7)
        truth += list(zip(pts, uv))
    p3, p2 = m.getPointsInFrame(7)
    assert len(p2) > len(p3)                            # 3^2 entries for point 1
    i2 = pair_frame_observations(p3, p2)
    assert list(zip(np.asarray(p3).tolist(), np.asarray(i2).tolist())) == truth
    p3, p2 = m.getPointsInFrame(0)                      # no duplicates: p2 itself
    assert np.asarray(pair_frame_observations(p3, p2)).tolist() == list(p2)
