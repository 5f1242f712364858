"""CPU restatement of BRISK (TEST INFRASTRUCTURE ONLY: the checker of the
device BRISK path, imported by tests/ and never by the product).

The reference constructs `brisk::BriskFeatureDetector(60, 6, true)` and
`brisk::BriskDescriptorExtractor(true, true, Version::briskV2, 1.0)`
(/root/reference/CTracker.cpp:43-45, used at :275-287) from the ethz-asl
BRISK 2 library, which is NOT in /root/reference (no source, no fixtures):
parity against it is UNPINNED.  What is restated here is BRISK as published
(Leutenegger, Chli, Siegwart, "BRISK: Binary Robust Invariant Scalable
Keypoints", ICCV 2011) in the form of its reference implementation (the
code OpenCV ships as cv::BRISK, version 1 of the same authors' library):

Descriptor (BRISK_Impl::generateKernel / smoothedIntensity /
computeDescriptorsAndOrOrientation):
* pattern: rings r = 0.85 * {0, 2.9, 4.9, 7.4, 10.8} with {1, 10, 14, 15,
  20} points, Gaussian sigma 1.3 * s * r * sin(pi / n) (0.65 s on the
  centre), 64 discrete scales s = 2^(i * log2(30) / 64), 1024 rotations;
* pairs: long if |d|^2 > (8.2)^2 (orientation, weights int(d / |d|^2 *
  2048 + 0.5)), short if |d|^2 < (5.85)^2 (the descriptor bits);
* smoothed intensity: box of side 2 sigma around the point with fractional
  border weights, fixed point (scaling 2^22 / area), integral image for the
  inner part;
* orientation: atan2 of the long-pair gradient sums; descriptor bit k =
  I(short pair k, i) > I(short pair k, j) on the pattern rotated by the
  quantised orientation (64 bytes for the 512 short pairs of this pattern);
* keypoints nearer the border than the scale's pattern size are removed.

Detector (BriskScaleSpace): 2 * octaves layers (c_i: halving; d_i: 2/3 of
c_0, then halving; OpenCV resizes INTER_AREA), FAST 9-16 corner score
(OpenCV's cornerScore<16>) per layer, candidates with score >= threshold
that are 3x3 maxima of their layer and not below the score at the same
position of the layers above and below (nearest sample), refined by
BRISK's subpixel2D quadratic fit.  The published detector's 3-D refinement
(refine3D with interpolated neighbour-layer scores) is replaced by that
nearest-sample scale test: documented simplification, unpinned either way.
"""
from __future__ import annotations

import math

import numpy as np

N_ROT = 1024
SCALES = 64
SCALE_RANGE = 30.0
BASIC_SIZE = 12.0


def make_pattern(pattern_scale: float = 1.0):
    """-> (points [scales][rot][points] (x, y, sigma) float32, size_list
    [scales] int, short pairs [m][2] (i, j), long pairs [l][4] (i, j,
    weighted_dx, weighted_dy))."""
    f = 0.85 * pattern_scale
    r_list = np.float32([f * 0.0, f * 2.9, f * 4.9, f * 7.4, f * 10.8])
    n_list = [1, 10, 14, 15, 20]
    d_max = np.float32(5.85 * pattern_scale)
    d_min = np.float32(8.2 * pattern_scale)
    n_pts = sum(n_list)
    lb_scale = np.float32(math.log(SCALE_RANGE) / math.log(2.0))
    lb_scale_step = np.float32(lb_scale / SCALES)
    sigma_scale = np.float32(1.3)
    # cos / sin of (alpha + theta) per (rotation, point) from libm (math.*),
    # the rest vectorised over the scales with the C++ code's float / double
    # steps (IEEE products and casts, so identical to the scalar form)
    rings = np.repeat(np.arange(5), n_list)
    nums = np.concatenate([np.arange(n) for n in n_list])
    cs = np.zeros((N_ROT, n_pts))
    sn = np.zeros((N_ROT, n_pts))
    for rot in range(N_ROT):
        theta = float(rot) * 2 * math.pi / float(N_ROT)
        for k in range(n_pts):
            alpha = float(nums[k]) * 2 * math.pi / float(n_list[rings[k]])
            cs[rot, k] = math.cos(alpha + theta)
            sn[rot, k] = math.sin(alpha + theta)
    sin_ring = np.array([math.sin(math.pi / n) for n in n_list])
    s_list = np.array([np.float32(math.pow(2.0, float(np.float32(np.float32(sc) * lb_scale_step)))) for sc in range(SCALES)],
                      np.float32)
    sr = (s_list[:, None] * r_list[None, :]).astype(np.float32)                 # [scales][rings] float
    pts = np.zeros((SCALES, N_ROT, n_pts, 3), np.float32)
    srp = sr[:, rings].astype(np.float64)                                       # [scales][points]
    pts[..., 0] = (srp[:, None, :] * cs[None, :, :]).astype(np.float32)
    pts[..., 1] = (srp[:, None, :] * sn[None, :, :]).astype(np.float32)
    sig = ((sigma_scale * s_list).astype(np.float32).astype(np.float64)[:, None] * r_list.astype(np.float64)[None, :] *
           sin_ring[None, :]).astype(np.float32)
    sig[:, 0] = (sigma_scale * s_list * np.float32(0.5)).astype(np.float32)
    sigp = sig[:, rings]
    pts[..., 2] = sigp[:, None, :]
    size = np.ceil((sr[:, rings] + sigp).astype(np.float32).astype(np.float64)).astype(np.int64) + 1
    size_list = size.max(axis=1)
    short, long = [], []
    p0 = pts[0, 0]
    for i in range(1, n_pts):
        for j in range(i):
            dx = np.float32(p0[j, 0] - p0[i, 0])
            dy = np.float32(p0[j, 1] - p0[i, 1])
            nsq = np.float32(dx * dx + dy * dy)
            if nsq > np.float32(d_min * d_min):
                long.append((i, j, int(float(np.float32(dx / nsq)) * 2048.0 + 0.5),
                             int(float(np.float32(dy / nsq)) * 2048.0 + 0.5)))
            elif nsq < np.float32(d_max * d_max):
                short.append((i, j))
    return pts, size_list, np.array(short, np.int32), np.array(long, np.int64)


def integral(img: np.ndarray) -> np.ndarray:
    s = np.zeros((img.shape[0] + 1, img.shape[1] + 1), np.int64)
    s[1:, 1:] = np.cumsum(np.cumsum(img.astype(np.int64), 0), 1)
    return s


def smoothed_intensity(img, ii, key_x, key_y, pt):
    """BRISK_Impl::smoothedIntensity for one pattern point (x, y, sigma)."""
    f32 = np.float32
    xf = f32(f32(pt[0]) + f32(key_x))
    yf = f32(f32(pt[1]) + f32(key_y))
    x, y = int(xf), int(yf)
    cols = img.shape[1]
    sigma_half = f32(pt[2])
    area = f32(f32(4.0) * sigma_half * sigma_half)
    if sigma_half < 0.5:
        r_x = int(f32(xf - f32(x)) * 1024)
        r_y = int(f32(yf - f32(y)) * 1024)
        r_x_1, r_y_1 = 1024 - r_x, 1024 - r_y
        v = (r_x_1 * r_y_1 * int(img[y, x]) + r_x * r_y_1 * int(img[y, x + 1]) + r_x * r_y * int(img[y + 1, x + 1]) +
             r_x_1 * r_y * int(img[y + 1, x]))
        return (v + 512) // 1024
    scaling = int(4194304.0 / float(area))
    scaling2 = int(float(f32(f32(scaling) * area)) / 1024.0)
    x_1 = f32(xf - sigma_half)
    x1 = f32(xf + sigma_half)
    y_1 = f32(yf - sigma_half)
    y1 = f32(yf + sigma_half)
    x_left = int(f32(x_1 + f32(0.5)))
    y_top = int(f32(y_1 + f32(0.5)))
    x_right = int(f32(x1 + f32(0.5)))
    y_bottom = int(f32(y1 + f32(0.5)))
    r_x_1 = f32(f32(f32(x_left) - x_1) + f32(0.5))
    r_y_1 = f32(f32(f32(y_top) - y_1) + f32(0.5))
    r_x1 = f32(f32(x1 - f32(x_right)) + f32(0.5))
    r_y1 = f32(f32(y1 - f32(y_bottom)) + f32(0.5))
    dx = x_right - x_left - 1
    dy = y_bottom - y_top - 1
    A = int(f32(r_x_1 * r_y_1) * f32(scaling))
    B = int(f32(r_x1 * r_y_1) * f32(scaling))
    C = int(f32(r_x1 * r_y1) * f32(scaling))
    D = int(f32(r_x_1 * r_y1) * f32(scaling))
    r_x_1_i = int(r_x_1 * f32(scaling))
    r_y_1_i = int(r_y_1 * f32(scaling))
    r_x1_i = int(r_x1 * f32(scaling))
    r_y1_i = int(r_y1 * f32(scaling))
    # corners
    v = (A * int(img[y_top, x_left]) + B * int(img[y_top, x_left + dx + 1]) +
         C * int(img[y_top + dy + 1, x_left + dx + 1]) + D * int(img[y_top + dy + 1, x_left]))
    if dx + dy > 2:
        # edges and the middle from the integral image: S(r0, r1, c0, c1) =
        # sum of img[r0:r1, c0:c1]
        def S(r0, r1, c0, c1):
            return int(ii[r1, c1] - ii[r0, c1] - ii[r1, c0] + ii[r0, c0])
        xl, yt = x_left, y_top
        upper = S(yt, yt + 1, xl + 1, xl + 1 + dx) * r_y_1_i
        middle = S(yt + 1, yt + 1 + dy, xl + 1, xl + 1 + dx) * scaling
        left = S(yt + 1, yt + 1 + dy, xl, xl + 1) * r_x_1_i
        right = S(yt + 1, yt + 1 + dy, xl + dx + 1, xl + dx + 2) * r_x1_i
        bottom = S(yt + dy + 1, yt + dy + 2, xl + 1, xl + 1 + dx) * r_y1_i
        return _c_div(v + upper + middle + left + right + bottom + scaling2 // 2, scaling2)
    for c in range(x_left + 1, x_left + 1 + dx):
        v += r_y_1_i * int(img[y_top, c]) + r_y1_i * int(img[y_top + dy + 1, c])
    for r in range(y_top + 1, y_top + 1 + dy):
        v += r_x_1_i * int(img[r, x_left]) + r_x1_i * int(img[r, x_left + dx + 1])
        for c in range(x_left + 1, x_left + 1 + dx):
            v += int(img[r, c]) * scaling
    return _c_div(v + scaling2 // 2, scaling2)


def _c_div(a: int, b: int) -> int:
    """C integer division (truncation toward zero)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def _wrap32(v: int) -> int:
    return (v + 2 ** 31) % 2 ** 32 - 2 ** 31


def describe(img: np.ndarray, kps: np.ndarray, pattern=None):
    """kps [n][3] (x, y, size) float32 -> (kept index [m], angle [m] degrees
    in [0, 360), descriptors [m][n_bytes] uint8).  Orientation and
    descriptor as computeDescriptorsAndOrOrientation with both enabled."""
    if pattern is None:
        pattern = make_pattern()
    pts, size_list, short, long = pattern
    img = np.ascontiguousarray(img, np.uint8)
    ii = integral(img)
    rows, cols = img.shape
    n_bytes = int(math.ceil(len(short) / 128.0)) * 4 * 4
    lb_scalerange = np.float32(math.log(SCALE_RANGE) / np.float32(0.693147180559945))
    basic06 = np.float32(BASIC_SIZE * np.float32(0.6))
    kept, angles, descs = [], [], []
    for k, (x, y, size) in enumerate(np.asarray(kps, np.float32)):
        lg = np.float32(np.float32(math.log(float(np.float32(size / basic06)))) / np.float32(0.693147180559945))
        sc = int(float(np.float32(np.float32(SCALES / lb_scalerange) * lg)) + 0.5)
        sc = max(sc, 0)
        if sc >= SCALES:
            sc = SCALES - 1
        border = int(size_list[sc])
        if x < border or x >= cols - border or y < border or y >= rows - border:
            continue
        vals = [smoothed_intensity(img, ii, x, y, p) for p in pts[sc, 0]]
        d0 = d1 = 0
        for (i, j, wdx, wdy) in long:
            dt = vals[i] - vals[j]
            d0 += _c_div(dt * int(wdx), 1024)
            d1 += _c_div(dt * int(wdy), 1024)
        angle = np.float32(math.atan2(float(np.float32(d1)), float(np.float32(d0))) / math.pi * 180.0)
        theta = int(N_ROT * (float(angle) / 360.0) + 0.5)
        if theta < 0:
            theta += N_ROT
        if theta >= N_ROT:
            theta -= N_ROT
        if angle < 0:
            angle = np.float32(angle + np.float32(360.0))
        vals = [smoothed_intensity(img, ii, x, y, p) for p in pts[sc, theta]]
        bits = np.zeros(n_bytes * 8, np.uint8)
        for b, (i, j) in enumerate(short):
            bits[b] = vals[i] > vals[j]
        # bit b of 32-bit word b // 32 (little endian bytes)
        desc = np.packbits(bits.reshape(-1, 8)[:, ::-1], axis=1).reshape(-1)
        kept.append(k)
        angles.append(float(angle))
        descs.append(desc)
    return np.array(kept, np.int64), np.array(angles, np.float32), np.array(descs, np.uint8).reshape(-1, n_bytes)


# ---------------------------------------------------------------------------
# Detector
_CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
           (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]  # (x, y), OpenCV offsets16


def halfsample(img):
    """2x area average, (a + b + c + d + 2) >> 2 (an odd last row / column is dropped)."""
    h2, w2 = img.shape[0] // 2, img.shape[1] // 2
    a = img[:2 * h2, :2 * w2].astype(np.int32)
    s = a[0::2, 0::2] + a[0::2, 1::2] + a[1::2, 0::2] + a[1::2, 1::2]
    return ((s + 2) >> 2).astype(np.uint8)


def twothirdsample(img):
    """2/3 area average: every 3x3 block -> 2x2 with weights (4, 2, 2, 1) / 9,
    rounded ((x + 4) / 9); the remainder rows / columns are dropped."""
    h3, w3 = img.shape[0] // 3, img.shape[1] // 3
    a = img[:3 * h3, :3 * w3].astype(np.int32)
    p = [[a[r::3, c::3] for c in range(3)] for r in range(3)]
    out = np.zeros((2 * h3, 2 * w3), np.int32)
    out[0::2, 0::2] = 4 * p[0][0] + 2 * p[0][1] + 2 * p[1][0] + p[1][1]
    out[0::2, 1::2] = 4 * p[0][2] + 2 * p[0][1] + 2 * p[1][2] + p[1][1]
    out[1::2, 0::2] = 4 * p[2][0] + 2 * p[1][0] + 2 * p[2][1] + p[1][1]
    out[1::2, 1::2] = 4 * p[2][2] + 2 * p[1][2] + 2 * p[2][1] + p[1][1]
    return ((out + 4) // 9).astype(np.uint8)


def pyramid(img, octaves: int = 6):
    """BriskScaleSpace::constructPyramid: [(layer image, scale, offset)]
    c0, d0 = 2/3 c0, then every layer halves the one two before it."""
    f32 = np.float32
    L = [(np.ascontiguousarray(img, np.uint8), f32(1.0), f32(0.0))]
    n = max(1, 2 * octaves)
    if n > 1:
        s = f32(1.5)
        L.append((twothirdsample(img), s, f32(f32(0.5) * s - f32(0.5))))
    for i in range(2, n, 2):
        for b in (i - 2, i - 1):
            s = f32(L[b][1] * f32(2.0))
            L.append((halfsample(L[b][0]), s, f32(f32(0.5) * s - f32(0.5))))
    return L


def fast_score(img):
    """R = cornerScore<16>(p, threshold 0) when >= 1, else 0 (BriskLayer::
    getAgastScore(x, y, 1)); 0 within 3 pixels of the border."""
    h, w = img.shape
    R = np.zeros((h, w), np.int32)
    if h < 7 or w < 7:
        return R
    v = img[3:h - 3, 3:w - 3].astype(np.int32)
    d = np.stack([v - img[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx].astype(np.int32) for (dx, dy) in _CIRCLE])
    dark = np.full(v.shape, -10 ** 6, np.int32)
    bright = np.full(v.shape, -10 ** 6, np.int32)
    for s in range(16):
        arc = d[[(s + m) % 16 for m in range(9)]]
        dark = np.maximum(dark, arc.min(0))
        bright = np.maximum(bright, (-arc).min(0))
    sc = np.maximum(np.maximum(dark, bright), 0) - 1
    R[3:h - 3, 3:w - 3] = np.where(sc >= 1, sc, 0)
    return R


def _is_max2d(S, x, y):
    """BriskScaleSpace::isMax2D on the thresholded score map S."""
    c = S[y, x]
    nb = [(-1, -1), (0, -1), (1, -1), (-1, 0), (1, 0), (-1, 1), (0, 1), (1, 1)]
    for dx, dy in nb:
        if S[y + dy, x + dx] > c:
            return False
    eq = [(dx, dy) for dx, dy in nb if S[y + dy, x + dx] == c]
    if not eq:
        return True

    def smooth(cx, cy):
        w = ((1, 2, 1), (2, 4, 2), (1, 2, 1))
        return sum(w[j][i] * int(S[cy - 1 + j, cx - 1 + i]) for j in range(3) for i in range(3))

    sc = smooth(x, y)
    for dx, dy in eq:
        if smooth(x + dx, y + dy) > sc:
            return False
    return True


def subpixel2d(s):
    """BriskScaleSpace::subpixel2D on the 3x3 scores s[i][j] = score at
    (x + i - 1, y + j - 1) (the reference's s_i_j: i along x) -> (dx, dy,
    max), float32 step for step (the reference's delta_y = delta_x1 / _x2
    assignment in the clamped branch included)."""
    f = np.float32
    s_0_0, s_0_1, s_0_2 = int(s[0][0]), int(s[0][1]), int(s[0][2])
    s_1_0, s_1_1, s_1_2 = int(s[1][0]), int(s[1][1]), int(s[1][2])
    s_2_0, s_2_1, s_2_2 = int(s[2][0]), int(s[2][1]), int(s[2][2])
    tmp1 = s_0_0 + s_0_2 - 2 * s_1_1 + s_2_0 + s_2_2
    coeff1 = 3 * (tmp1 + s_0_1 - ((s_1_0 + s_1_2) << 1) + s_2_1)
    coeff2 = 3 * (tmp1 - ((s_0_1 + s_2_1) << 1) + s_1_0 + s_1_2)
    tmp2 = s_0_2 - s_2_0
    tmp3 = s_0_0 + tmp2 - s_2_2
    tmp4 = tmp3 - 2 * tmp2
    coeff3 = -3 * (tmp3 + s_0_1 - s_2_1)
    coeff4 = -3 * (tmp4 + s_1_0 - s_1_2)
    coeff5 = (s_0_0 - s_0_2 - s_2_0 + s_2_2) << 2
    coeff6 = -((s_0_0 + s_0_2 - ((s_1_0 + s_0_1 + s_1_2 + s_2_1) << 1) - 5 * s_1_1 + s_2_0 + s_2_2) << 1)
    H_det = 4 * coeff1 * coeff2 - coeff5 * coeff5

    def quad(dx, dy):
        v = f(f(f(coeff1) * dx) * dx)
        v = f(v + f(f(f(coeff2) * dy) * dy))
        v = f(v + f(f(coeff3) * dx))
        v = f(v + f(f(coeff4) * dy))
        v = f(v + f(f(f(coeff5) * dx) * dy))
        v = f(v + f(coeff6))
        return f(v / f(18.0))

    if H_det == 0:
        return f(0.0), f(0.0), f(f(coeff6) / f(18.0))
    if not (H_det > 0 and coeff1 < 0):
        tmp_max = coeff3 + coeff4 + coeff5
        dx, dy = f(1.0), f(1.0)
        t = -coeff3 + coeff4 - coeff5
        if t > tmp_max:
            tmp_max, dx, dy = t, f(-1.0), f(1.0)
        t = coeff3 - coeff4 - coeff5
        if t > tmp_max:
            tmp_max, dx, dy = t, f(1.0), f(-1.0)
        t = -coeff3 - coeff4 + coeff5
        if t > tmp_max:
            tmp_max, dx, dy = t, f(-1.0), f(-1.0)
        return dx, dy, f(f(tmp_max + coeff1 + coeff2 + coeff6) / f(18.0))
    dx = f(f(2 * coeff2 * coeff3 - coeff4 * coeff5) / f(-H_det))
    dy = f(f(2 * coeff1 * coeff4 - coeff3 * coeff5) / f(-H_det))
    tx, tx_, ty, ty_ = dx > 1.0, dx < -1.0 and not dx > 1.0, dy > 1.0, dy < -1.0
    if tx or tx_ or ty or ty_:
        dx1 = dx2 = dy1 = dy2 = f(0.0)
        if tx:
            dx1 = f(1.0)
            dy1 = f(-f(coeff4 + coeff5) / f(2 * coeff2))
        elif tx_:
            dx1 = f(-1.0)
            dy1 = f(-f(coeff4 - coeff5) / f(2 * coeff2))
        dy1 = f(min(max(dy1, f(-1.0)), f(1.0)))
        if ty:
            dy2 = f(1.0)
            dx2 = f(-f(coeff3 + coeff5) / f(2 * coeff1))
        elif ty_:
            dy2 = f(-1.0)
            dx2 = f(-f(coeff3 - coeff5) / f(2 * coeff1))
        dx2 = f(min(max(dx2, f(-1.0)), f(1.0)))
        m1, m2 = quad(dx1, dy1), quad(dx2, dy2)
        if m1 > m2:
            return dx1, dx1, m1
        return dx2, dx2, m2
    return dx, dy, quad(dx, dy)


def detect(img, threshold: int = 60, octaves: int = 6):
    """-> keypoints [n][5] (x, y, size, response, octave) float32, in layer
    order, row-major within a layer (the order BRISK emits them)."""
    f = np.float32
    L = pyramid(img, octaves)
    R = [fast_score(l[0]) for l in L]
    S = [np.where(r >= threshold, r, 0) for r in R]
    out = []
    for i, (li, sc, off) in enumerate(L):
        h, w = li.shape
        ys, xs = np.nonzero(S[i])
        for y, x in zip(ys.tolist(), xs.tolist()):
            if not _is_max2d(S[i], x, y):
                continue
            c = S[i][y, x]
            ok = True
            for j in (i - 1, i + 1):
                if j < 0 or j >= len(L):
                    continue
                _, scj, offj = L[j]
                hj, wj = S[j].shape
                X = f(f(f(x) * sc) + off)
                Y = f(f(f(y) * sc) + off)
                xj = int(f(f(f(X - offj) / scj) + f(0.5)))
                yj = int(f(f(f(Y - offj) / scj) + f(0.5)))
                x0, x1 = max(xj - 1, 0), min(xj + 1, wj - 1)
                y0, y1 = max(yj - 1, 0), min(yj + 1, hj - 1)
                if x0 <= x1 and y0 <= y1 and S[j][y0:y1 + 1, x0:x1 + 1].max() > c:
                    ok = False
                    break
            if not ok:
                continue
            # s_i_j of subpixel2D is the score at (x + i - 1, y + j - 1)
            dx, dy, mx = subpixel2d(R[i][y - 1:y + 2, x - 1:x + 2].T)
            kx = f(f(f(f(x) + dx) * sc) + off)
            ky = f(f(f(f(y) + dy) * sc) + off)
            out.append((kx, ky, f(f(BASIC_SIZE) * sc), mx, f(i)))
    return np.array(out, np.float32).reshape(-1, 5)
