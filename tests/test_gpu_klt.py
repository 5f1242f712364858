"""GPU parity of the tracker through the C ABI:
pyramid + Scharr derivatives bit-exact, calcOpticalFlowPyrLK next points
and status bit-exact (float equality), computeOpticalFlow index lists
bit-exact, all against the CPU oracle on the same frames; tracking accuracy
on the synthetic video as the size-independent property at C5's size."""
import numpy as np
import pytest

from oracle import ffi as O
from sfm_amd import klt
from sfm_amd.video import SyntheticVideo

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def video():
    v = SyntheticVideo()
    return v, [v.frame(k) for k in range(4)]


@pytest.mark.parametrize("shape", [(720, 1280), (359, 643), (61, 97), (23, 23)])
def test_pyramid_levels_bit_exact(shape):
    rng = np.random.default_rng(shape[1])
    f0 = rng.integers(0, 256, shape, dtype=np.uint8)
    f1 = rng.integers(0, 256, shape, dtype=np.uint8)
    tr = klt.KLTTracker(shape[1], shape[0])
    tr.push_frame(f0)
    tr.push_frame(f1)
    ref = f0
    for lv in range(tr.num_levels):
        img, dxy = tr.level(0, lv)
        assert np.array_equal(img, ref), lv
        assert np.array_equal(dxy, O.scharr(ref)), lv
        ref = O.pyr_down(ref)
    img, _ = tr.level(1, 0)
    assert np.array_equal(img, f1)
    tr.close()


def _edge_points(w, h):
    return np.array([[0, 0], [w - 1, h - 1], [-5, 3], [w + 10, 20], [w / 2 + 0.5, h / 2 + 0.25], [10.0, h - 10.5],
                     [-21.0, 5.0], [-30.0, 5.0], [w - 1e-3, 7.0]], np.float64)


def test_calc_flow_bit_exact_full_size(video):
    v, frames = video
    rng = np.random.default_rng(0)
    p0 = np.concatenate([v.features(0, 500, rng), _edge_points(v.w, v.h)])
    tr = klt.KLTTracker(v.w, v.h)
    tr.push_frame(frames[0])
    tr.push_frame(frames[1])
    g, gs = tr.calc_flow(p0)
    o, os_ = O.calc_optical_flow_pyr_lk(frames[0], frames[1], p0)
    assert np.array_equal(gs, os_)
    assert np.array_equal(g, o)
    truth = v.map_points(0, 1, p0[:500])
    err = np.linalg.norm(g[:500] - truth, axis=1)[gs[:500] == 1]
    assert np.median(err) < 0.05
    tr.close()


@pytest.mark.parametrize("win,max_level,max_count,eps", [(7, 1, 20, 0.03), (21, 0, 5, 0.01), (31, 5, 30, 0.0),
                                                         (3, 2, 20, 0.03)])
def test_calc_flow_parameter_variants(win, max_level, max_count, eps):
    v = SyntheticVideo(320, 240, seed=win)
    f0, f1 = v.frame(0), v.frame(1)
    rng = np.random.default_rng(win)
    p0 = np.concatenate([v.features(0, 100, rng, border=10), _edge_points(320, 240)])
    g, gs = klt.calc_optical_flow_pyr_lk(f0, f1, p0, win_size=win, max_level=max_level, max_count=max_count,
                                         epsilon=eps)
    o, os_ = O.calc_optical_flow_pyr_lk(f0, f1, p0, win=win, max_level=max_level, max_count=max_count, eps=eps)
    assert np.array_equal(gs, os_) and np.array_equal(g, o)


def test_flat_frames_fail_min_eig():
    z = np.full((120, 160), 77, np.uint8)
    g, gs = klt.calc_optical_flow_pyr_lk(z, z, [[50, 50], [10, 10]])
    assert gs.tolist() == [0, 0]


def test_compute_optical_flow_sequence(video):
    """Four frames pushed in turn (ping-pong slots); each step's match lists
    equal the oracle's (LK + association), and matched detections are the
    true images of the tracked points."""
    v, frames = video
    rng = np.random.default_rng(4)
    tr = klt.KLTTracker(v.w, v.h)
    tr.push_frame(frames[0])
    prev = v.features(0, 500, rng)
    for k in range(1, 4):
        tr.push_frame(frames[k])
        det = v.detections(k - 1, k, prev, rng)
        pi, ci, fl, st = tr.compute_optical_flow(prev, det, with_flow=True)
        o, os_ = O.calc_optical_flow_pyr_lk(frames[k - 1], frames[k], prev)
        assert np.array_equal(st, os_) and np.array_equal(fl, o), k
        opi, oci = O.klt_associate(prev.astype(np.float32), o, os_, det)
        assert np.array_equal(pi, opi) and np.array_equal(ci, oci), k
        assert len(pi) > 400
        truth = v.map_points(k - 1, k, prev[pi])
        assert np.max(np.linalg.norm(det[ci] - truth, axis=1)) < 1.5
        prev = det  # the current frame's detections become the next prev points
    tr.close()


def test_compute_optical_flow_edge_cases(video):
    v, frames = video
    tr = klt.KLTTracker(v.w, v.h)
    tr.push_frame(frames[0])
    tr.push_frame(frames[1])
    rng = np.random.default_rng(2)
    prev = v.features(0, 50, rng)
    # no detections: no matches (the reference would index position -1)
    pi, ci = tr.compute_optical_flow(prev, np.zeros((0, 2)))
    assert len(pi) == 0 and len(ci) == 0
    # no previous points
    pi, ci = tr.compute_optical_flow(np.zeros((0, 2)), v.detections(0, 1, prev, rng))
    assert len(pi) == 0
    # duplicated detections and duplicated prev points: ties resolved as the oracle does
    det = v.detections(0, 1, prev, rng, jitter=0.0, drop=0.0, n_extra=0)
    det = np.concatenate([det, det[:10]])
    prev2 = np.concatenate([prev, prev[:10]])
    pi, ci, fl, st = tr.compute_optical_flow(prev2, det, with_flow=True)
    opi, oci = O.klt_associate(prev2.astype(np.float32), fl, st, det)
    assert np.array_equal(pi, opi) and np.array_equal(ci, oci)
    tr.close()


def test_ctracker_mirror_compute_optical_flow(video):
    """The CTracker mirror's pushFrame / computeOpticalFlow members."""
    import sfm_amd
    v, frames = video
    rng = np.random.default_rng(8)
    prev = v.features(0, 200, rng)
    det = v.detections(0, 1, prev, rng)
    t = sfm_amd.CTracker()
    t.pushFrame(frames[0])
    t.pushFrame(frames[1])
    ok = t.computeOpticalFlow(prev, det)
    o, os_ = O.calc_optical_flow_pyr_lk(frames[0], frames[1], prev)
    opi, oci = O.klt_associate(prev.astype(np.float32), o, os_, det)
    assert ok == (len(opi) >= 5)
    assert np.array_equal(t._prevIdx, opi) and np.array_equal(t._currIdx, oci)
