"""CPU: the BRISK restatement (oracle/brisk_oracle.py) on published facts
and hand-checked cases: the pattern's 512 short / 870 long pairs (the
paper's and the reference implementation's counts), the layer geometry of
BriskScaleSpace, the FAST 9-16 score on constructed corners, subpixel2D on
exact quadratics, and the descriptor's smoothing on flat images."""
import numpy as np
import pytest

from oracle import brisk_oracle as B


@pytest.fixture(scope="module")
def pattern():
    return B.make_pattern()


def test_pattern_pair_counts_and_sizes(pattern):
    pts, size_list, short, long = pattern
    assert pts.shape == (64, 1024, 60, 3)
    assert len(short) == 512 and len(long) == 870
    assert size_list[0] == 13 and np.all(np.diff(size_list) >= 0)
    # the pattern at rotation 0, scale 0: centre, then rings of radius 0.85 r
    r = np.hypot(pts[0, 0, :, 0], pts[0, 0, :, 1])
    assert r[0] == 0 and np.allclose(r[1:11], 0.85 * 2.9, rtol=1e-6) and np.allclose(r[40:], 0.85 * 10.8, rtol=1e-6)
    # a quarter turn maps point k of ring 4 (20 points) onto point k + 5
    q = pts[0, 256, 40:, :2]
    assert np.allclose(q[0], pts[0, 0, 45, :2], atol=1e-5)


def test_layers_follow_brisk_scale_space():
    img = np.zeros((720, 1280), np.uint8)
    L = B.pyramid(img, 6)
    assert [l[0].shape for l in L][:4] == [(720, 1280), (480, 852), (360, 640), (240, 426)]
    assert [float(l[1]) for l in L] == [1.0, 1.5, 2.0, 3.0, 4.0, 6.0, 8.0, 12.0, 16.0, 24.0, 32.0, 48.0]
    assert [float(l[2]) for l in L][:3] == [0.0, 0.25, 0.5]


def test_area_resize_matches_inter_area():
    """resize(INTER_AREA): ratio 2 on both axes is resizeAreaFast's
    (a + b + c + d + 2) >> 2; an exact 3/2 ratio gives the (4, 2, 2, 1) / 9
    weights (cvRound: N / 9 never ties); a constant image stays constant at
    any ratio; 1280 -> 852 columns (BRISK's d0 width) uses fractional cells."""
    a = np.array([[0, 1, 2], [3, 4, 5], [6, 7, 8]], np.uint8)
    assert B.area_resize(np.array([[0, 1], [3, 4]], np.uint8), 1, 1).tolist() == [[2]]
    t = B.area_resize(a, 2, 2)
    assert t.tolist() == [[round((4 * 0 + 2 * 1 + 2 * 3 + 4) / 9), round((4 * 2 + 2 * 1 + 2 * 5 + 4) / 9)],
                          [round((4 * 6 + 2 * 3 + 2 * 7 + 4) / 9), round((4 * 8 + 2 * 5 + 2 * 7 + 4) / 9)]]
    c = np.full((30, 1280), 137, np.uint8)
    assert (B.area_resize(c, 852, 20) == 137).all()
    tab = B._area_tab(1280, 852, 1.0 / (852 / 1280))
    assert all(abs(sum(float(al) for _, al in t) - 1.0) < 1e-6 for t in tab)
    assert len(tab[1]) == 3 and tab[1][0][0] == 1        # a cell straddling three source columns
    ramp = np.tile(np.arange(1280, dtype=np.float64) % 256, (3, 1)).astype(np.uint8)
    r = B.area_resize(ramp, 852, 2)
    assert abs(int(r[0, 100]) - np.mean(ramp[0, 150:152])) <= 1


def test_refine1d_finds_the_parabola_vertex():
    """refine1D / _1 / _2: samples of a parabola peaking at scale 1.1 (octave),
    1.05 (intra), 0.9 (layer 0) give back the vertex and its height."""
    for kind, xs, peak in ((0, (0.75, 1.0, 1.5), 1.1), (1, (2 / 3, 1.0, 4 / 3), 1.05), (2, (2 / 3, 1.0, 1.5), 0.9)):
        s = [np.float32(90.0 - 200.0 * (x - peak) ** 2) for x in xs]
        r, m = B._refine1d(*s, kind)
        assert abs(float(r) - peak) < 2e-3 and abs(float(m) - 90.0) < 0.05


def test_fast_score_of_a_constructed_corner():
    img = np.full((15, 15), 100, np.uint8)
    # 9 contiguous circle pixels of the centre (7, 7) at 180: score = 80 - 1
    for (dx, dy) in B._CIRCLE[:9]:
        img[7 + dy, 7 + dx] = 180
    R = B.fast_score(img)
    assert R[7, 7] == 79
    img[7 + B._CIRCLE[4][1], 7 + B._CIRCLE[4][0]] = 100   # break the arc: 8 left
    assert B.fast_score(img)[7, 7] == 0
    assert B.fast_score(img)[:3].sum() == 0               # border rows


def test_subpixel2d_recovers_a_quadratic_peak():
    # s(x, y) = 100 - 10 (x - 0.3)^2 - 10 (y + 0.2)^2; s[i][j] at (x, y) = (i - 1, j - 1)
    s = [[int(round(100 - 10 * (x - 0.3) ** 2 - 10 * (y + 0.2) ** 2)) for y in (-1, 0, 1)] for x in (-1, 0, 1)]
    dx, dy, m = B.subpixel2d(s)
    assert abs(dx - 0.3) < 0.05 and abs(dy + 0.2) < 0.05 and abs(m - 100) < 1.0
    flat = [[5, 5, 5], [5, 5, 5], [5, 5, 5]]
    assert B.subpixel2d(flat)[:2] == (0.0, 0.0)


def test_detector_refines_towards_the_peak():
    """A blurred blob corner: the refined keypoint lies within a pixel of the
    integer maximum, on the side of the stronger neighbour."""
    img = np.full((64, 64), 60, np.uint8)
    img[20:44, 20:44] = 200
    k = B.detect(img, threshold=30, octaves=1)
    assert len(k) >= 4                                    # the square's corners
    for x, y, size, resp, oc in k:
        assert min(abs(x - 20), abs(x - 43)) < 2.5 and min(abs(y - 20), abs(y - 43)) < 2.5


def test_smoothing_of_a_flat_image(pattern):
    """Every pattern point of a flat image smooths to the same intensity
    x ~1024 to within the fixed-point border weights (the reference's
    truncated weights leave +-1-2 counts, so flat-region bits are not all 0)."""
    flat = np.full((200, 200), 77, np.uint8)
    ii = B.integral(flat)
    for sc in (0, 20, 40):
        v = np.array([B.smoothed_intensity(flat, ii, 100.0, 100.0, p) for p in pattern[0][sc, 0]])
        assert np.all(np.abs(v - 77 * 1024) <= 0.01 * 77 * 1024)
    k2, _, _ = B.describe(flat, np.float32([[3, 100, 12]]), pattern)
    assert len(k2) == 0                                    # too near the border for its scale
