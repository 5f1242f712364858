"""GPU parity of the T7 corner detector (CTracker::
detectFeaturesOpticalFlow, /root/reference/CTracker.cpp:252-272) through the
C ABI: goodFeaturesToTrack + cornerSubPix on the device against the oracle
restatement (oracle/gftt_oracle.cpp, pinned by tests/gftt_ref.py) —
bit-exact corner lists (order included) and refined positions.  Frames: the
C5 synthetic video, noise, hard-edged blocks (response plateaus and ties),
a flat frame; parameter variants cover the distance-free path, tight and
wide spacings, corner caps and every subpixel window size."""
import numpy as np
import pytest

import sfm_amd
from sfm_amd import klt
from sfm_amd.video import SyntheticVideo
from oracle import ffi as O

pytestmark = pytest.mark.gpu

V = SyntheticVideo()
RNG = np.random.default_rng(11)
FRAMES = {
    "video0": V.frame(0),
    "video50": V.frame(50),
    "noise": RNG.integers(0, 256, (240, 320), dtype=np.uint8),
    "blocks": (np.kron(RNG.integers(0, 2, (30, 40)), np.ones((8, 8))) * 200 + 20).astype(np.uint8),
    "small": RNG.integers(0, 256, (9, 13), dtype=np.uint8),
}


def _oracle(img, p):
    c = O.good_features(img, p["max_corners"], p["quality_level"], p["min_distance"])
    if p["subpix_win"] > 0:
        c = O.corner_subpix(img, c, p["subpix_win"], p["subpix_max_iter"], p["subpix_epsilon"])
    return c


BASE = dict(max_corners=500, quality_level=0.05, min_distance=10.0, subpix_win=5, subpix_max_iter=20,
            subpix_epsilon=0.03)
CASES = [("video0", {}), ("video50", {}), ("noise", {}), ("blocks", {}), ("small", {}),
         ("video0", dict(subpix_win=0)), ("noise", dict(subpix_win=0, min_distance=0.5, max_corners=3000)),
         ("noise", dict(min_distance=3.0, quality_level=0.01, max_corners=2000)),
         ("video0", dict(min_distance=25.0, max_corners=100)), ("blocks", dict(subpix_win=3, subpix_max_iter=5)),
         ("video50", dict(subpix_win=7, subpix_epsilon=0.0)), ("noise", dict(subpix_win=1, max_corners=1))]


@pytest.mark.parametrize("name,over", CASES, ids=[f"{n}-{i}" for i, (n, _) in enumerate(CASES)])
def test_detect_features_bit_exact(name, over):
    img = FRAMES[name]
    p = dict(BASE, **over)
    g = klt.good_features_to_track(img, **p)
    o = _oracle(img, p)
    assert g.shape == o.shape
    assert np.array_equal(g, o)


def test_resident_frame_sequence_and_ctracker_mirror():
    """Detection on the handle's resident current frame across pushes, and the
    CTracker mirror's bool (n >= _minFeatures, CTracker.cpp:267)."""
    tr = sfm_amd.CTracker()
    for k in (0, 1, 2):
        f = V.frame(k)
        tr.pushFrame(f)
        assert tr.detectFeaturesOpticalFlow()
        assert np.array_equal(tr.currPoints, O.detect_features_of(f))
    tr.pushFrame(np.full((720, 1280), 90, np.uint8))
    assert not tr.detectFeaturesOpticalFlow()
    assert tr.currPoints.shape == (0, 2)


def test_detected_corners_feed_the_tracker():
    """T7 -> T6 chain: corners detected on frame k are tracked into frame k+1
    and associated with the corners detected there (the C5 loop)."""
    tr = klt.KLTTracker(V.w, V.h)
    tr.push_frame(V.frame(3))
    c0 = tr.detect_features()
    tr.push_frame(V.frame(4))
    c1 = tr.detect_features()
    pi, ci, fl, st = tr.compute_optical_flow(c0, c1, with_flow=True)
    nx, st_o = O.calc_optical_flow_pyr_lk(V.frame(3), V.frame(4), c0)
    assert np.array_equal(st, st_o) and np.array_equal(fl[st == 1], nx[st_o == 1])
    po, co = O.klt_associate(c0, nx, st_o, c1)
    assert np.array_equal(pi, po) and np.array_equal(ci, co)
    assert len(pi) > 100


def test_bad_arguments_fail_loudly():
    img = FRAMES["noise"]
    with pytest.raises(sfm_amd.SfmError):
        klt.good_features_to_track(img, max_corners=5000)
    with pytest.raises(sfm_amd.SfmError):
        klt.good_features_to_track(img, subpix_win=8)
