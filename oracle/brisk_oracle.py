"""CPU restatement of BRISK (TEST INFRASTRUCTURE ONLY: the checker of the
device BRISK path, imported by tests/ and never by the product).

The reference constructs `brisk::BriskFeatureDetector(60, 6, true)` and
`brisk::BriskDescriptorExtractor(true, true, Version::briskV2, 1.0)`
(/root/reference/CTracker.cpp:43-45, used at :275-287) from the ethz-asl
BRISK 2 library, which is NOT in /root/reference (no source, no fixtures):
parity against it is UNPINNED.  What is restated here is BRISK as published
(Leutenegger, Chli, Siegwart, "BRISK: Binary Robust Invariant Scalable
Keypoints", ICCV 2011) in the form of its reference implementation (the
code OpenCV ships as cv::BRISK, version 1 of the same authors' library).
What the reference's BRISK 2 / briskV2 descriptor changes over version 1
is not documented in any published description available here, so no
difference is restated (unpinned):

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

Detector (BriskScaleSpace::constructPyramid / getKeypoints / refine3D):
* pyramid: 2 * octaves layers, c_0 the image, d_0 = 2/3 of it, every later
  layer half the one two before; each resampled by OpenCV 3.0's
  resize(INTER_AREA) (what cv::BRISK's halfsample / twothirdsample call):
  the exact 2x2 average (a + b + c + d + 2) >> 2 when both ratios are 2,
  else the general area filter (computeResizeAreaTab's float weights,
  float accumulation in table order, cvRound);
* candidates: FAST 9-16 corners at the threshold after FAST's own 3x3
  non-maximum suppression (strictly above every neighbouring corner score),
  in FAST's row-major order; BRISK's isMax2D on the layer's score image
  then always passes (a suppressed neighbour scores strictly lower and a
  non-corner scores below the threshold), so it is not restated;
* scores: s(x, y) = cornerScore<16> with threshold 0, kept when >= 1
  (BriskLayer::getAgastScore(x, y, 1)), 0 within 3 pixels of the border;
  between pixels, the bilinear float interpolation of getAgastScore(xf, yf)
  truncated to uchar; layer 0's virtual lower layer uses the 5-8 score
  (cornerScore<8>, radius 1, getAgastScore_5_8);
* 3-D non-maximum suppression and scale refinement (refine3D): the
  interpolated scores of the neighbouring layers over the candidate's
  footprint (getScoreMaxAbove / getScoreMaxBelow, with the footprint
  transforms derived from the layers' scale and offset), any sample above
  the candidate's score rejects it; subpixel2D on the best neighbour-layer
  sample and on the candidate's own 3x3; a parabola through the three
  layers' maxima gives the scale (refine1D at 3/4, 1, 3/2 around an octave,
  refine1D_1 at 2/3, 1, 4/3 around an intra-octave, refine1D_2 at 2/3, 1,
  3/2 on layer 0), the position is interpolated between the layers'
  subpixel offsets; kept when the refined score exceeds the threshold;
  the last layer is refined in 2-D against the layer below only.
Choices where the published description leaves the arithmetic open (and
the reference's library cannot be consulted): every footprint sample is
tested against the candidate's score (all rows); the below-layer offsets
map back through the exact inverse transforms; the layer-0 virtual layer
sits at scale 2/3 (refine1D_2's sample points); a negative cornerScore
(no corner even at threshold 0) is taken as 0, not wrapped to 255 by a
uchar cast; keypoint size = 12 x scale (BRISK's basicSize).
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


def _area_tab(ssize: int, dsize: int, scale: float):
    """computeResizeAreaTab (OpenCV 3.0 imgwarp.cpp) for one axis: per
    destination index the (source index, float32 weight) entries in table
    order (double geometry, float weights)."""
    tab = [[] for _ in range(dsize)]
    for dx in range(dsize):
        fsx1 = dx * scale
        fsx2 = fsx1 + scale
        cell = min(scale, ssize - fsx1)
        sx1, sx2 = math.ceil(fsx1), math.floor(fsx2)
        sx2 = min(sx2, ssize - 1)
        sx1 = min(sx1, sx2)
        if sx1 - fsx1 > 1e-3:
            tab[dx].append((sx1 - 1, np.float32((sx1 - fsx1) / cell)))
        for sx in range(sx1, sx2):
            tab[dx].append((sx, np.float32(1.0 / cell)))
        if fsx2 - sx2 > 1e-3:
            tab[dx].append((sx2, np.float32(min(min(fsx2 - sx2, 1.0), cell) / cell)))
    return tab


def area_resize(img, dw: int, dh: int):
    """resize(img, (dw, dh), INTER_AREA) for 8-bit downscaling, OpenCV 3.0:
    ratios of exactly 2 take resizeAreaFast's (a + b + c + d + 2) >> 2; any
    other ratio the general area filter: per source row, buf[dx] += S * alpha
    (float32, table order), per destination row sum = sum of beta * buf
    (float32, table order), then cvRound (half to even)."""
    sh, sw = img.shape
    scale_x = 1.0 / (dw / sw)
    scale_y = 1.0 / (dh / sh)
    if scale_x == 2.0 and scale_y == 2.0:
        a = img[:2 * dh, :2 * dw].astype(np.int32)
        s4 = a[0::2, 0::2] + a[0::2, 1::2] + a[1::2, 0::2] + a[1::2, 1::2]
        return ((s4 + 2) >> 2).astype(np.uint8)
    xt, yt = _area_tab(sw, dw, scale_x), _area_tab(sh, dh, scale_y)
    kx = max(len(t) for t in xt)
    xs = np.zeros((kx, dw), np.int64)
    xa = np.zeros((kx, dw), np.float32)
    for dx, t in enumerate(xt):
        for k, (sx, al) in enumerate(t):
            xs[k, dx], xa[k, dx] = sx, al
    out = np.zeros((dh, dw), np.uint8)
    f = np.float32
    for dy, t in enumerate(yt):
        acc = np.zeros(dw, np.float32)
        for sy, beta in t:
            row = img[sy].astype(np.float32)
            buf = np.zeros(dw, np.float32)
            for k in range(kx):  # padding entries add 0 * S = 0 (exact)
                buf = (buf + (row[xs[k]] * xa[k]).astype(f)).astype(f)
            acc = (acc + (f(beta) * buf).astype(f)).astype(f)
        out[dy] = np.clip(np.rint(acc), 0, 255).astype(np.uint8)
    return out


def pyramid(img, octaves: int = 6):
    """BriskScaleSpace::constructPyramid: [(layer image, scale, offset)]
    c0, d0 = 2/3 c0, then every layer halves the one two before it."""
    f32 = np.float32
    L = [(np.ascontiguousarray(img, np.uint8), f32(1.0), f32(0.0))]
    n = max(1, 2 * octaves)
    h, w = img.shape
    if n > 1:
        s = f32(1.5)
        L.append((area_resize(img, 2 * (w // 3), 2 * (h // 3)), s, f32(f32(0.5) * s - f32(0.5))))
    for i in range(2, n, 2):
        for b in (i - 2, i - 1):
            s = f32(L[b][1] * f32(2.0))
            src = L[b][0]
            L.append((area_resize(src, src.shape[1] // 2, src.shape[0] // 2), s, f32(f32(0.5) * s - f32(0.5))))
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


_CIRCLE8 = [(1, 0), (1, 1), (0, 1), (-1, 1), (-1, 0), (-1, -1), (0, -1), (1, -1)]  # OpenCV offsets8


def fast58_score(img):
    """BriskLayer::getAgastScore_5_8(x, y, 1): cornerScore<8> (5 contiguous
    of the 8 radius-1 neighbours) with threshold 0, kept when >= 1; 0 within
    2 pixels of the border."""
    h, w = img.shape
    R = np.zeros((h, w), np.int32)
    if h < 5 or w < 5:
        return R
    v = img[2:h - 2, 2:w - 2].astype(np.int32)
    d = np.stack([v - img[2 + dy:h - 2 + dy, 2 + dx:w - 2 + dx].astype(np.int32) for (dx, dy) in _CIRCLE8])
    dark = np.full(v.shape, -10 ** 6, np.int32)
    bright = np.full(v.shape, -10 ** 6, np.int32)
    for st in range(8):
        arc = d[[(st + m) % 8 for m in range(5)]]
        dark = np.maximum(dark, arc.min(0))
        bright = np.maximum(bright, (-arc).min(0))
    sc = np.maximum(np.maximum(dark, bright), 0) - 1
    R[2:h - 2, 2:w - 2] = np.where(sc >= 1, sc, 0)
    return R


def fast_nms_candidates(R, threshold: int):
    """FAST 9-16 corners at `threshold` after FAST's 3x3 non-maximum
    suppression (strictly above every neighbouring corner's score), in
    row-major order -> (ys, xs)."""
    S = np.where(R >= threshold, R, 0)
    h, w = S.shape
    keep = S > 0
    P = np.pad(S, 1)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dx or dy:
                keep &= S > P[1 + dy:1 + dy + h, 1 + dx:1 + dx + w]
    return np.nonzero(keep)


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


class _Layer:
    def __init__(self, img, scale, offset):
        self.img, self.scale, self.offset = img, scale, offset
        self.h, self.w = img.shape
        self.R = fast_score(img)

    def score(self, x: int, y: int) -> int:
        """getAgastScore(x, y, 1)"""
        if x < 3 or y < 3 or x >= self.w - 3 or y >= self.h - 3:
            return 0
        return int(self.R[y, x])

    def score_f(self, xf, yf) -> int:
        """getAgastScore(xf, yf, 1, scale 1): bilinear in float32, truncated
        to uchar (int() truncates toward zero, as the C++ casts)."""
        f = np.float32
        xf, yf = f(xf), f(yf)
        x, y = int(xf), int(yf)
        rx1 = f(xf - f(x))
        rx = f(f(1.0) - rx1)
        ry1 = f(yf - f(y))
        ry = f(f(1.0) - ry1)
        v = f(f(rx * ry) * f(self.score(x, y)))
        v = f(v + f(f(rx1 * ry) * f(self.score(x + 1, y))))
        v = f(v + f(f(rx * ry1) * f(self.score(x, y + 1))))
        v = f(v + f(f(rx1 * ry1) * f(self.score(x + 1, y + 1))))
        return int(v) & 0xFF


def _patch(get, cx, cy):
    """s[i][j] = score at (cx + i - 1, cy + j - 1) (subpixel2D's s_i_j)."""
    return [[get(cx + i - 1, cy + j - 1) for j in range(3)] for i in range(3)]


def _footprint(layer: int, x: int, y: int, above: bool):
    """The candidate's footprint in the neighbouring layer (float32 bounds),
    from the layers' scale / offset: octave layer -> intra above (x'' =
    (4x - 1) / 6, +-2/6) or intra below (x' = (8x + 1) / 6, +-4/6); intra
    layer -> octave above ((6x - 1) / 8, +-3/8) or octave below ((6x + 1) /
    4, +-3/4)."""
    f = np.float32
    if above:
        a, b, c, d = (4, -1, 2, 6) if layer % 2 == 0 else (6, -1, 3, 8)
    else:
        a, b, c, d = (8, 1, 4, 6) if layer % 2 == 0 else (6, 1, 3, 4)
    return (f(f(a * x + b - c) / f(d)), f(f(a * x + b + c) / f(d)),
            f(f(a * y + b - c) / f(d)), f(f(a * y + b + c) / f(d)))


def _back(layer: int, real: np.float32, coord: int, above: bool):
    """The neighbouring layer's coordinate mapped back to this layer, minus
    the candidate's (the inverse of _footprint's transform)."""
    f = np.float32
    if above:
        m, o, dv = (6, 1, 4) if layer % 2 == 0 else (8, 1, 6)
    else:
        m, o, dv = (6, -1, 8) if layer % 2 == 0 else (4, -1, 6)
    return f(f(f(f(real * f(m)) + f(o)) / f(dv)) - f(coord))


def score_max_neighbour(L, layer: int, x: int, y: int, thr: int, above: bool):
    """getScoreMaxAbove / getScoreMaxBelow: -> (ismax, score, dx, dy).
    Scans the footprint (corners and edges interpolated, inner samples on
    the grid) in BRISK's order; any sample above `thr` (the candidate's
    score) rejects."""
    f = np.float32
    M = L[layer + 1] if above else L[layer - 1]
    x_1, x1, y_1, y1 = _footprint(layer, x, y, above)
    ix_1, ix1, iy_1, iy1 = int(x_1), int(x1), int(y_1), int(y1)
    max_x, max_y = ix_1 + 1, iy_1 + 1
    best = f(M.score_f(x_1, y_1))
    if best > thr:
        return False, f(0), f(0), f(0)

    def take(v, mx, my):
        nonlocal best, max_x, max_y
        if v > best:
            best, max_x, max_y = v, mx, my

    for xx in range(ix_1 + 1, ix1 + 1):
        v = f(M.score_f(f(xx), y_1))
        if v > thr:
            return False, f(0), f(0), f(0)
        take(v, xx, max_y)
    v = f(M.score_f(x1, y_1))
    if v > thr:
        return False, f(0), f(0), f(0)
    take(v, ix1, max_y)
    for yy in range(iy_1 + 1, iy1 + 2):  # middle rows, then the bottom row at y1
        last = yy == iy1 + 1
        yv = y1 if last else f(yy)
        yi = iy1 if last else yy
        v = f(M.score_f(x_1, yv))
        if v > thr:
            return False, f(0), f(0), f(0)
        take(v, int(f(x_1 + f(1.0))), yi)
        for xx in range(ix_1 + 1, ix1 + 1):
            v = f(M.score(xx, yy)) if not last else f(M.score_f(f(xx), yv))
            if v > thr:
                return False, f(0), f(0), f(0)
            take(v, xx, yi)
        v = f(M.score_f(x1, yv))
        if v > thr:
            return False, f(0), f(0), f(0)
        take(v, ix1, yi)
    dx1, dy1, refined = subpixel2d(_patch(M.score, max_x, max_y))
    real_x = f(f(max_x) + dx1)
    real_y = f(f(max_y) + dy1)
    ret_refined = True
    if real_x > x1:
        ret_refined, real_x = False, x1
    if real_x < x_1:
        ret_refined, real_x = False, x_1
    if real_y > y1:
        ret_refined, real_y = False, y1
    if real_y < y_1:
        ret_refined, real_y = False, y_1
    dx = _back(layer, real_x, x, above)
    dy = _back(layer, real_y, y, above)
    dx = f(min(max(dx, f(-1.0)), f(1.0)))
    dy = f(min(max(dy, f(-1.0)), f(1.0)))
    return True, (f(max(refined, best)) if ret_refined else best), dx, dy


def _refine1d(s_05, s0, s05, kind: int):
    """refine1D (kind 0: samples at 3/4, 1, 3/2), refine1D_1 (kind 1: 2/3, 1,
    4/3), refine1D_2 (kind 2: 2/3, 1, 3/2): the parabola through the three
    layers' maxima -> (relative scale, refined maximum)."""
    f = np.float32
    i_05 = int(1024.0 * float(s_05) + 0.5)
    i0 = int(1024.0 * float(s0) + 0.5)
    i05 = int(1024.0 * float(s05) + 0.5)
    if kind == 0:
        A, B, C, lo, hi, den = (16, -24, 8), (-40, 54, -14), (24, -27, 6), f(0.75), f(1.5), f(3072.0)
    elif kind == 1:
        A, B, C, lo, hi, den = (9, -18, 9), (-21, 36, -15), (12, -16, 6), f(2.0 / 3.0), f(4.0 / 3.0), f(2048.0)
    else:
        A, B, C, lo, hi, den = (18, -30, 12), (-45, 65, -20), (27, -30, 8), f(2.0 / 3.0), f(1.5), f(5120.0)
    a = A[0] * i_05 + A[1] * i0 + A[2] * i05
    if a >= 0:
        if s0 >= s_05 and s0 >= s05:
            return f(1.0), f(s0)
        if s_05 >= s0 and s_05 >= s05:
            return lo, f(s_05)
        if s05 >= s0 and s05 >= s_05:
            return hi, f(s05)
    b = B[0] * i_05 + B[1] * i0 + B[2] * i05
    r = f(-f(b) / f(2 * a))
    if r < lo:
        r = lo
    elif r > hi:
        r = hi
    c = C[0] * i_05 + C[1] * i0 + C[2] * i05
    mx = f(f(f(c) + f(f(f(a) * r) * r)) + f(f(b) * r))
    return r, f(mx / den)


def refine3d(L, R58, layer: int, x: int, y: int):
    """BriskScaleSpace::refine3D -> None (not a 3-D maximum) or (score, x,
    y, scale) in image coordinates."""
    f = np.float32
    T = L[layer]
    center = T.score(x, y)
    ok, max_above, dxa, dya = score_max_neighbour(L, layer, x, y, center, True)
    if not ok:
        return None
    if layer % 2 == 0 and layer == 0:
        def s58(px, py):
            return int(R58[py, px]) if 0 <= px < T.w and 0 <= py < T.h else 0
        patch = _patch(s58, x, y)
        max_below = f(max(max(r) for r in patch))
        dxb, dyb, _ = subpixel2d(patch)
    else:
        ok, max_below, dxb, dyb = score_max_neighbour(L, layer, x, y, center, False)
        if not ok:
            return None
    dxl, dyl, max_layer = subpixel2d(_patch(T.score, x, y))
    mid = f(max(f(center), max_layer))
    kind = 2 if layer == 0 else (0 if layer % 2 == 0 else 1)
    scale, mx = _refine1d(max_below, mid, max_above, kind)
    if layer % 2 == 0:
        if scale > 1.0:
            r0 = f(f(f(1.5) - scale) / f(0.5))
            r_o, odx, ody = f(f(1.0) - r0), dxa, dya
        else:
            lo = f(2.0 / 3.0) if layer == 0 else f(0.75)
            r0 = f(f(scale - lo) / f(f(1.0) - lo))
            r_o, odx, ody = f(f(1.0) - r0), dxb, dyb
    else:
        if scale > 1.0:
            r0 = f(f(4.0) - f(scale * f(3.0)))
            r_o, odx, ody = f(f(1.0) - r0), dxa, dya
        else:
            r0 = f(f(scale * f(3.0)) - f(2.0))
            r_o, odx, ody = f(f(1.0) - r0), dxb, dyb
    kx = f(f(f(f(r0 * dxl) + f(r_o * odx)) + f(x)) * T.scale) + T.offset
    ky = f(f(f(f(r0 * dyl) + f(r_o * ody)) + f(y)) * T.scale) + T.offset
    return mx, f(kx), f(ky), f(scale * T.scale)


def detect(img, threshold: int = 60, octaves: int = 6):
    """-> keypoints [n][5] (x, y, size, response, octave) float32 in the
    order BRISK emits them (layer, then FAST's row-major candidate order)."""
    f = np.float32
    L = [_Layer(im, sc, off) for (im, sc, off) in pyramid(img, octaves)]
    R58 = fast58_score(L[0].img)
    n = len(L)
    out = []
    for i, T in enumerate(L):
        ys, xs = fast_nms_candidates(T.R, threshold)
        for y, x in zip(ys.tolist(), xs.tolist()):
            if n == 1:
                dx, dy, mx = subpixel2d(_patch(T.score, x, y))
                out.append((f(f(f(x) + dx) * T.scale + T.offset), f(f(f(y) + dy) * T.scale + T.offset),
                            f(f(BASIC_SIZE) * T.scale), mx, f(i)))
                continue
            if i == n - 1:
                ok, _, _, _ = score_max_neighbour(L, i, x, y, T.score(x, y), False)
                if not ok:
                    continue
                dx, dy, mx = subpixel2d(_patch(T.score, x, y))
                out.append((f(f(f(f(x) + dx) * T.scale) + T.offset), f(f(f(f(y) + dy) * T.scale) + T.offset),
                            f(f(BASIC_SIZE) * T.scale), mx, f(i)))
                continue
            r = refine3d(L, R58, i, x, y)
            if r is None:
                continue
            mx, kx, ky, sc = r
            if mx > f(threshold):
                out.append((kx, ky, f(f(BASIC_SIZE) * sc), mx, f(i)))
    return np.array(out, np.float32).reshape(-1, 5)
