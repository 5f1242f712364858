"""Independent numpy restatement of the T7 corner detector,
written from the same published OpenCV 3.0 semantics as
oracle/gftt_oracle.cpp but sharing no code with it:

  goodFeaturesToTrack(grey, pts, 500, 0.05, 10)   /root/reference/CTracker.cpp:262
  cornerSubPix(grey, pts, Size(5,5), Size(-1,-1),
               TermCriteria(COUNT|EPS, 20, 0.03)) /root/reference/CTracker.cpp:265

Used only to pin the C++ oracle (tests/test_gftt_oracle.py); vectorised
where the oracle loops, pure Python where the oracle is vectorisable.
"""
from __future__ import annotations

import ctypes
import ctypes.util

import numpy as np

_libm = ctypes.CDLL(ctypes.util.find_library("m"))
_libm.expf.argtypes = [ctypes.c_float]
_libm.expf.restype = ctypes.c_float


def _reflect101(idx: np.ndarray, n: int) -> np.ndarray:
    idx = np.abs(idx)
    return np.where(idx >= n, 2 * n - 2 - idx, idx)


def min_eigen(img: np.ndarray) -> np.ndarray:
    h, w = img.shape
    ys = _reflect101(np.arange(-1, h + 1), h)
    xs = _reflect101(np.arange(-1, w + 1), w)
    p = img.astype(np.int32)[np.ix_(ys, xs)]          # (h+2, w+2), reflect-101 border
    gx = p[:, 2:] - p[:, :-2]                          # horizontal differences
    dx = gx[:-2] + 2 * gx[1:-1] + gx[2:]
    gy = p[2:, :] - p[:-2, :]
    dy = gy[:, :-2] + 2 * gy[:, 1:-1] + gy[:, 2:]
    scale = 1.0 / (4.0 * 3.0 * 255.0)
    ix = (dx.astype(np.float64) * scale).astype(np.float32)
    iy = (dy.astype(np.float64) * scale).astype(np.float32)
    prods = [ix * ix, ix * iy, iy * iy]
    sums = []
    for c in prods:
        cx = c[:, xs]                                   # columns reflect-101
        r = (cx[:, :-2] + cx[:, 1:-1]) + cx[:, 2:]
        ry = r[ys]                                      # rows reflect-101
        sums.append((ry[:-2] + ry[1:-1]) + ry[2:])
    a = sums[0] * np.float32(0.5)
    b = sums[1]
    c = sums[2] * np.float32(0.5)
    return (a + c) - np.sqrt((a - c) * (a - c) + b * b)


def good_features(img: np.ndarray, max_corners=500, quality=0.05, min_distance=10.0) -> np.ndarray:
    h, w = img.shape
    eig = min_eigen(img)
    thr = np.float32(float(eig.max()) * quality)
    t = np.where(eig > thr, eig, np.float32(0))
    pad = np.full((h + 2, w + 2), -np.inf, np.float32)
    pad[1:-1, 1:-1] = t
    dil = np.max(np.stack([pad[dy:dy + h, dx:dx + w] for dy in range(3) for dx in range(3)]), axis=0)
    cand = (t != 0) & (t == dil)
    cand[0, :] = cand[-1, :] = False
    cand[:, 0] = cand[:, -1] = False
    ys, xs = np.nonzero(cand)
    lin = ys * w + xs
    vals = t[ys, xs]
    order = np.lexsort((-lin, -vals.astype(np.float64)))   # value desc, raster index desc
    md2 = min_distance * min_distance
    acc = []
    for k in order:
        x, y = int(xs[k]), int(ys[k])
        if min_distance >= 1.0 and any((x - ax) ** 2 + (y - ay) ** 2 < md2 for ax, ay in acc):
            continue
        acc.append((x, y))
        if len(acc) == max_corners:
            break
    return np.array(acc, np.float32).reshape(-1, 2)


def _butterfly_sum(terms: np.ndarray) -> float:
    n = len(terms)
    padded = np.zeros(((n + 63) // 64) * 64)
    padded[:n] = terms
    rows = padded.reshape(-1, 64)
    v = rows[0].copy()
    for r in range(1, rows.shape[0]):      # lane L: pixels L, L+64, ... in turn
        lanes_live = np.arange(64) + 64 * r < n
        v = np.where(lanes_live, v + rows[r], v)
    lanes = np.arange(64)
    off = 32
    while off >= 1:
        v = v + v[lanes ^ off]
        off //= 2
    return float(v[0])


def corner_subpix(img: np.ndarray, pts: np.ndarray, win=5, max_iter=20, eps=0.03) -> np.ndarray:
    h, w = img.shape
    ww, sw = 2 * win + 1, 2 * win + 3
    mask = np.zeros((ww, ww), np.float32)
    for i in range(ww):
        y = np.float32(i - win) / np.float32(win)
        vy = _libm.expf(float(-y * y))
        for j in range(ww):
            x = np.float32(j - win) / np.float32(win)
            mask[i, j] = np.float32(vy) * np.float32(_libm.expf(float(-x * x)))
    m = mask.astype(np.float64).ravel()
    pj = np.tile(np.arange(ww) - win, ww).astype(np.float64)
    pi = np.repeat(np.arange(ww) - win, ww).astype(np.float64)
    max_iter = min(max(max_iter, 1), 100)
    eps2 = max(eps, 0.0) ** 2
    imgf = img.astype(np.float32)
    out = np.array(pts, np.float32).reshape(-1, 2).copy()
    f32 = np.float32
    for p in range(out.shape[0]):
        tx, ty = out[p]
        cx, cy = tx, ty
        it = 0
        while True:
            ox, oy = f32(cx - f32(sw - 1) * f32(0.5)), f32(cy - f32(sw - 1) * f32(0.5))
            ix, iy = int(np.floor(ox)), int(np.floor(oy))
            a, b = f32(ox - f32(ix)), f32(oy - f32(iy))
            a11, a12 = f32((f32(1) - a) * (f32(1) - b)), f32(a * (f32(1) - b))
            a21, a22 = f32((f32(1) - a) * b), f32(a * b)
            X = np.clip(np.arange(ix, ix + sw + 1), 0, w - 1)
            Y = np.clip(np.arange(iy, iy + sw + 1), 0, h - 1)
            q = imgf[np.ix_(Y, X)]
            sub = ((q[:-1, :-1] * a11 + q[:-1, 1:] * a12) + q[1:, :-1] * a21) + q[1:, 1:] * a22
            tgx = (sub[1:-1, 2:] - sub[1:-1, :-2]).astype(np.float64).ravel()
            tgy = (sub[2:, 1:-1] - sub[:-2, 1:-1]).astype(np.float64).ravel()
            gxx, gxy, gyy = tgx * tgx * m, tgx * tgy * m, tgy * tgy * m
            A, B, C = _butterfly_sum(gxx), _butterfly_sum(gxy), _butterfly_sum(gyy)
            bb1 = _butterfly_sum(gxx * pj + gxy * pi)
            bb2 = _butterfly_sum(gxy * pj + gyy * pi)
            det = A * C - B * B
            if abs(det) <= np.finfo(np.float64).eps ** 2:
                break
            sc = 1.0 / det
            nx = f32(float(cx) + C * sc * bb1 - B * sc * bb2)
            ny = f32(float(cy) - B * sc * bb1 + A * sc * bb2)
            err = float(f32(f32(f32(nx - cx) * f32(nx - cx)) + f32(f32(ny - cy) * f32(ny - cy))))
            cx, cy = nx, ny
            if cx < 0 or cx >= w or cy < 0 or cy >= h:
                break
            it += 1
            if not (it < max_iter and err > eps2):
                break
        if abs(f32(cx - tx)) > win or abs(f32(cy - ty)) > win:
            cx, cy = tx, ty
        out[p] = (cx, cy)
    return out
