"""CPU: the T7 corner-detector oracle (oracle/gftt_oracle.cpp) pinned by the
independent numpy restatement tests/gftt_ref.py — bit-exact min-eigenvalue
map, identical corner lists and identical subpixel refinements — on the C5
synthetic video, on noise and on small frames with corners near the border.
PARITY UNPINNED against OpenCV (absent; the reference holds no fixture)."""
import numpy as np
import pytest

from oracle import ffi as O
from tests import gftt_ref as R


def _frames():
    from sfm_amd.video import SyntheticVideo
    v = SyntheticVideo()
    rng = np.random.default_rng(5)
    noise = rng.integers(0, 256, (97, 131), dtype=np.uint8)
    blocks = np.kron(rng.integers(0, 2, (12, 16)), np.ones((8, 8))).astype(np.uint8) * 200 + 20
    return {"video0": v.frame(0), "video7": v.frame(7), "noise": noise, "blocks": blocks}


FR = _frames()


@pytest.mark.parametrize("name", ["video0", "noise", "blocks"])
def test_min_eigen_bit_exact(name):
    img = FR[name]
    assert np.array_equal(O.min_eigen(img).view(np.uint32), R.min_eigen(img).view(np.uint32))


@pytest.mark.parametrize("name,maxc,q,md", [("video0", 500, 0.05, 10.0), ("video7", 500, 0.05, 10.0),
                                             ("noise", 200, 0.01, 3.0), ("blocks", 500, 0.05, 10.0),
                                             ("noise", 50, 0.05, 0.5)])
def test_good_features_identical(name, maxc, q, md):
    img = FR[name]
    a = O.good_features(img, maxc, q, md)
    b = R.good_features(img, maxc, q, md)
    assert a.shape == b.shape and a.shape[0] > 0
    assert np.array_equal(a, b)


@pytest.mark.parametrize("name", ["video0", "blocks", "noise"])
def test_corner_subpix_identical(name):
    img = FR[name]
    c = O.good_features(img, 40, 0.05, 10.0)
    # corners near the frame edge take the clamped-sampling path
    h, w = img.shape
    c = np.vstack([c, np.array([[1, 1], [w - 2, h - 2], [2.5, h - 3.25]], np.float32)])
    a = O.corner_subpix(img, c)
    b = R.corner_subpix(img, c)
    assert np.array_equal(a, b)
    assert np.all(np.abs(a - c) <= 5.0)


def test_detect_features_of_is_gftt_then_subpix():
    img = FR["video0"]
    d = O.detect_features_of(img)
    assert d.shape[0] == 500
    assert np.array_equal(d, O.corner_subpix(img, O.good_features(img)))


def test_flat_frame_has_no_corners():
    assert O.good_features(np.full((40, 50), 77, np.uint8)).shape == (0, 2)
