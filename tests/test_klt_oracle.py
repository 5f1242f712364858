"""CPU: the tracker oracle (oracle/klt_oracle.cpp) pinned against an
independent numpy restatement (tests/klt_ref.py) of the same published
semantics, plus size-independent tracking properties on the synthetic video.

PARITY UNPINNED at the OpenCV boundary: cv::calcOpticalFlowPyrLK is absent
here and the reference holds no test or fixture for this path (SURVEY.md
§8c); the two restatements agreeing bit-exactly is the pin available.
"""
import numpy as np
import pytest

import klt_ref as R
from oracle import ffi as O
from sfm_amd.video import SyntheticVideo


@pytest.mark.parametrize("shape", [(1, 1), (1, 7), (2, 2), (7, 9), (33, 64), (150, 201), (359, 643)])
def test_pyramid_and_derivatives_match_numpy(shape):
    rng = np.random.default_rng(shape[0] * 1000 + shape[1])
    img = rng.integers(0, 256, shape, dtype=np.uint8)
    assert np.array_equal(O.pyr_down(img), R.pyr_down(img))
    assert np.array_equal(O.scharr(img), R.scharr(img))


def _edge_points(w, h):
    return np.array([[0, 0], [w - 1, h - 1], [-5, 3], [w + 10, 20], [w / 2 + 0.5, h / 2 + 0.25], [10.0, h - 10.5],
                     [-21.0, 5.0], [-30.0, 5.0], [w - 1e-3, 7.0]], np.float64)


@pytest.mark.parametrize("win,max_level", [(21, 3), (7, 1), (9, 0), (21, 5)])
def test_lk_oracle_matches_numpy(win, max_level):
    v = SyntheticVideo(200, 150, seed=11 + win)
    f0, f1 = v.frame(0), v.frame(1)
    rng = np.random.default_rng(win)
    p = np.concatenate([v.features(0, 16, rng, border=5), _edge_points(200, 150)])
    a, sa = R.calc_optical_flow_pyr_lk(f0, f1, p, win=win, max_level=max_level)
    b, sb = O.calc_optical_flow_pyr_lk(f0, f1, p, win=win, max_level=max_level)
    assert np.array_equal(sa, sb)
    assert np.array_equal(a, b)


def test_lk_flat_and_random_images():
    z = np.full((100, 120), 77, np.uint8)
    a, sa = O.calc_optical_flow_pyr_lk(z, z, [[50, 50], [10, 10]])
    assert sa.tolist() == [0, 0]  # minEig below threshold at level 0
    rng = np.random.default_rng(5)
    f0 = rng.integers(0, 256, (90, 110), dtype=np.uint8)
    f1 = np.roll(f0, (2, -3), axis=(0, 1))
    p = rng.uniform(25, 65, (12, 2))
    a, sa = R.calc_optical_flow_pyr_lk(f0, f1, p, win=11, max_level=2)
    b, sb = O.calc_optical_flow_pyr_lk(f0, f1, p, win=11, max_level=2)
    assert np.array_equal(sa, sb) and np.array_equal(a, b)


def test_lk_tracks_synthetic_motion_full_size():
    """Size-independent property at C5's frame size: tracked points land on
    the true image motion (3-10 px per frame) within a few hundredths of a px."""
    v = SyntheticVideo()
    f0, f1 = v.frame(0), v.frame(1)
    rng = np.random.default_rng(0)
    p0 = v.features(0, 500, rng)
    nxt, st = O.calc_optical_flow_pyr_lk(f0, f1, p0)
    truth = v.map_points(0, 1, p0)
    err = np.linalg.norm(nxt - truth, axis=1)[st == 1]
    assert st.mean() > 0.98
    assert np.median(err) < 0.05 and np.percentile(err, 95) < 0.2


def test_association_matches_transliteration_with_ties():
    rng = np.random.default_rng(9)
    for trial in range(30):
        n, m = int(rng.integers(0, 60)), int(rng.integers(0, 40))
        prev = rng.uniform(0, 100, (n, 2)).astype(np.float32)
        flowed = (prev + rng.uniform(-8, 8, (n, 2))).astype(np.float32)
        # detections on a coarse grid so that equal distances (ties) occur
        curr = np.round(rng.uniform(0, 100, (m, 2)) * 2) / 2
        if m > 3 and n > 3:
            curr[1] = curr[0]                  # duplicate detection: equal nearest distance
            flowed[2] = flowed[1]              # two flows onto the same point: equal e
            flowed[3] = np.float32(curr[0]) + np.float32(0.25)
        st = (rng.uniform(size=n) > 0.1).astype(np.uint8)
        a = O.klt_associate(prev, flowed, st, curr, max_org_feat_dist=2.0)
        b = R.klt_associate(prev, flowed, st, curr, max_org_feat_dist=2.0)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]), trial


def test_association_on_video():
    v = SyntheticVideo(320, 240, seed=3)
    f0, f1 = v.frame(0), v.frame(1)
    rng = np.random.default_rng(1)
    p0 = v.features(0, 80, rng, border=25)
    nxt, st = O.calc_optical_flow_pyr_lk(f0, f1, p0)
    det = v.detections(0, 1, p0, rng, n_extra=30)
    a = O.klt_associate(p0, nxt, st, det)
    b = R.klt_associate(p0.astype(np.float32), nxt, st, det)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert len(a[0]) > 50
    # every match pairs a point with the detection of its true image
    truth = v.map_points(0, 1, p0[a[0]])
    assert np.max(np.linalg.norm(det[a[1]] - truth, axis=1)) < 1.5
