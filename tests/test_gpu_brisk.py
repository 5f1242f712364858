"""GPU: the BRISK descriptor (sfm_brisk_describe) against the restatement
(oracle/brisk_oracle.py): the same keypoints kept, the same orientation,
bit-identical 64-byte descriptors, on a textured 1280x720 frame at sizes
covering the 64 pattern scales.  (Parity against the reference's ethz-asl
BRISK 2 library is unpinned: it is not in the tree.)"""
import numpy as np
import pytest

from oracle import brisk_oracle as B

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pattern():
    return B.make_pattern()


def _frame(seed=0):
    from sfm_amd.video import SyntheticVideo
    return SyntheticVideo().frame(seed)


@pytest.mark.parametrize("seed", [0, 1])
def test_descriptor_bit_exact(pattern, seed):
    from sfm_amd import brisk
    img = _frame(seed * 7)
    h, w = img.shape
    rng = np.random.default_rng(seed)
    n = 120
    kps = np.column_stack([rng.uniform(0, w, n), rng.uniform(0, h, n),
                           np.exp(rng.uniform(np.log(8.0), np.log(120.0), n))]).astype(np.float32)
    kept, ang, desc = brisk.describe(img, kps)
    okept, oang, odesc = B.describe(img, kps, pattern)
    assert kept.tolist() == okept.tolist()
    assert len(kept) > n // 2                      # most keypoints survive the border rule
    np.testing.assert_array_equal(ang, oang)
    assert (desc == odesc).all()


def test_descriptor_rotates_with_the_image(pattern):
    """A patch rotated by 90 degrees: the orientation turns by 90 degrees and
    most descriptor bits survive (the published invariance, a sanity check)."""
    from sfm_amd import brisk
    img = _frame(3)[200:520, 400:720].copy()
    rot = np.ascontiguousarray(np.rot90(img))
    c = (img.shape[1] - 1) / 2.0
    kp = np.float32([[c, c, 20.0]])
    kr = np.float32([[c, c, 20.0]])
    _, a0, d0 = brisk.describe(img, kp)
    _, a1, d1 = brisk.describe(rot, kr)
    turn = (a0[0] - a1[0]) % 360.0
    assert min(abs(turn - 90.0), abs(turn - 270.0)) < 3.0
    same = np.unpackbits(d0 ^ d1).sum()
    assert same < 0.2 * 512


def test_bad_keypoints_are_rejected():
    from sfm_amd import brisk
    img = np.zeros((64, 64), np.uint8)
    with pytest.raises(Exception):
        brisk.describe(img, [[10.0, 10.0, -1.0]])
    k, a, d = brisk.describe(img, np.zeros((0, 3)))
    assert len(k) == 0


@pytest.mark.parametrize("frame,thr", [(0, 60), (5, 60), (9, 30)])
def test_detector_matches_restatement(frame, thr):
    """Same keypoints in BRISK's order (layer, row-major): layer, response
    and position bit-equal (float32 step for step)."""
    from sfm_amd import brisk
    img = _frame(frame)
    kp, lay, _ = brisk.detect(img, threshold=thr, describe=False)
    ok = B.detect(img, threshold=thr)
    assert len(kp) == len(ok) and len(kp) > 500
    assert lay.tolist() == ok[:, 4].astype(int).tolist()
    np.testing.assert_array_equal(kp[:, [0, 1, 2, 4]], ok[:, [0, 1, 2, 3]])
    assert (kp[:, 3] == -1).all()


def test_detect_describe_end_to_end(pattern):
    """detectFeatures as the reference runs it: the descriptor's border rule
    drops keypoints; the kept ones carry the restatement's descriptors."""
    from sfm_amd import brisk
    img = _frame(2)
    kp, lay, desc = brisk.detect(img)
    ok = B.detect(img)
    kept, oang, odesc = B.describe(img, ok[:, :3], pattern)
    assert len(kp) == len(kept) > 300
    np.testing.assert_array_equal(kp[:, :3], ok[kept, :3])
    np.testing.assert_array_equal(kp[:, 3], oang)
    assert (desc == odesc).all()


def test_detector_on_the_resident_klt_frame():
    """sfm_klt_brisk_detect_describe: BRISK on the frame the KLT handle
    already holds (one upload per frame) equals the host-image call exactly,
    for the current frame after several pushes (ping-pong slots)."""
    from sfm_amd import brisk
    from sfm_amd.klt import KLTTracker
    img0 = _frame(3)
    klt = KLTTracker(img0.shape[1], img0.shape[0])
    try:
        for k in (3, 4, 5):
            img = _frame(k)
            klt.push_frame(img)
            a = brisk.detect_resident(klt)
            b = brisk.detect(img)
            assert len(a[0]) > 300
            for x, y in zip(a, b):
                np.testing.assert_array_equal(x, y)
        # the corner detector and LK keep working on the same resident frame
        assert len(klt.detect_features()) > 100
    finally:
        klt.close()
