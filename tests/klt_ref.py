"""Independent numpy restatement of the tracker path, used only to pin the C++
oracle (oracle/klt_oracle.cpp) in the CPU tests.

Written separately from the oracle from the same published semantics
(OpenCV 3.0 lkpyramid.cpp: buildOpticalFlowPyramid / calcSharrDeriv /
LKTrackerInvoker; CTracker.cpp:480-562; CFrame.cpp:437-450): whole-array
numpy for the pyramid and derivatives, np.float32 scalars for the float
steps (IEEE single ops in the same order), np.rint for cvRound.
Pure-Python loops: small images and a few points only.
"""
from __future__ import annotations

import numpy as np

F = np.float32


def reflect101(i, n):
    i = np.asarray(i)
    if n == 1:
        return np.zeros_like(i)
    period = 2 * n - 2
    i = np.abs(i) % period
    return np.where(i >= n, period - i, i)


def pyr_down(img):
    h, w = img.shape
    dh, dw = (h + 1) // 2, (w + 1) // 2
    k = np.array([1, 4, 6, 4, 1], np.int64)
    rows = reflect101(2 * np.arange(dh)[:, None] + np.arange(5)[None, :] - 2, h)  # [dh][5]
    cols = reflect101(2 * np.arange(dw)[:, None] + np.arange(5)[None, :] - 2, w)  # [dw][5]
    src = img.astype(np.int64)
    hs = (src[:, cols] * k[None, None, :]).sum(-1)          # [h][dw]
    acc = (hs[rows, :] * k[None, :, None]).sum(1)           # [dh][dw]
    return ((acc + 128) >> 8).astype(np.uint8)


def scharr(img):
    h, w = img.shape
    s = img.astype(np.int64)
    ym = reflect101(np.arange(h) - 1, h)
    yp = reflect101(np.arange(h) + 1, h)
    t0 = (s[ym] + s[yp]) * 3 + s * 10
    t1 = s[yp] - s[ym]
    xm = reflect101(np.arange(w) - 1, w)
    xp = reflect101(np.arange(w) + 1, w)
    dx = t0[:, xp] - t0[:, xm]
    dy = (t1[:, xp] + t1[:, xm]) * 3 + t1 * 10
    return np.stack([dx, dy], -1).astype(np.int16)


def pyramid(img, max_level, win):
    levels = [img]
    while len(levels) - 1 < max_level:
        p = levels[-1]
        if (p.shape[1] + 1) // 2 <= win or (p.shape[0] + 1) // 2 <= win:
            break
        levels.append(pyr_down(p))
    return levels


def _bilinear(img, X, Y, w4, shift, zero_outside):
    h, w = img.shape[:2]
    acc = 0
    for (dx, dy), wt in zip(((0, 0), (1, 0), (0, 1), (1, 1)), w4):
        xs, ys = X + dx, Y + dy
        if zero_outside:
            inside = (xs >= 0) & (xs < w) & (ys >= 0) & (ys < h)
            v = np.where(inside[..., None] if img.ndim == 3 else inside,
                         img[np.clip(ys, 0, h - 1), np.clip(xs, 0, w - 1)], 0).astype(np.int64)
        else:
            v = img[reflect101(ys, h), reflect101(xs, w)].astype(np.int64)
        acc = acc + v * wt
    return (acc + (1 << (shift - 1))) >> shift


def _weights(a, b):
    a, b = F(a), F(b)
    one = F(1)
    w00 = int(np.rint((one - a) * (one - b) * F(16384)))
    w01 = int(np.rint(a * (one - b) * F(16384)))
    w10 = int(np.rint((one - a) * b * F(16384)))
    return (w00, w01, w10, 16384 - w00 - w01 - w10)


def calc_optical_flow_pyr_lk(prev, nxt, pts, win=21, max_level=3, max_count=20, eps=0.03, min_eig=1e-3):
    I = pyramid(prev, max_level, win)
    J = pyramid(nxt, max_level, win)
    L = len(I) - 1
    D = [scharr(x) for x in I]
    eps2 = min(max(eps, 0.0), 10.0) ** 2
    half = F((win - 1) * 0.5)
    yy, xx = np.mgrid[0:win, 0:win]
    out = np.zeros((len(pts), 2), np.float32)
    status = np.ones(len(pts), np.uint8)
    for i, (px, py) in enumerate(np.asarray(pts, np.float32)):
        nx = ny = F(0)
        for level in range(L, -1, -1):
            li, lj, ld = I[level], J[level], D[level]
            h, w = li.shape
            sc = F(1.0 / (1 << level))
            ppx, ppy = F(px) * sc, F(py) * sc
            if level == L:
                npx, npy = ppx, ppy
            else:
                npx, npy = nx * F(2), ny * F(2)
            nx, ny = npx, npy
            ppx, ppy = ppx - half, ppy - half
            ipx, ipy = int(np.floor(ppx)), int(np.floor(ppy))
            if ipx < -win or ipx >= w or ipy < -win or ipy >= h:
                if level == 0:
                    status[i] = 0
                continue
            w4 = _weights(ppx - F(ipx), ppy - F(ipy))
            X, Y = ipx + xx, ipy + yy
            Ip = _bilinear(li, X, Y, w4, 9, False)
            dI = _bilinear(ld, X, Y, w4, 14, True)
            Ix, Iy = dI[..., 0], dI[..., 1]
            scale = F(1.0 / (1 << 20))
            A11 = F(int((Ix * Ix).sum())) * scale
            A12 = F(int((Ix * Iy).sum())) * scale
            A22 = F(int((Iy * Iy).sum())) * scale
            Dt = A11 * A22 - A12 * A12
            me = (A22 + A11 - np.sqrt((A11 - A22) * (A11 - A22) + F(4) * A12 * A12)) / F(2 * win * win)
            if float(me) < min_eig or Dt < F(np.finfo(np.float32).eps):
                if level == 0:
                    status[i] = 0
                continue
            Dt = F(1) / Dt
            npx, npy = npx - half, npy - half
            pdx = pdy = F(0)
            hj, wj = lj.shape
            for j in range(min(max(max_count, 0), 100)):
                inx, iny = int(np.floor(npx)), int(np.floor(npy))
                if inx < -win or inx >= wj or iny < -win or iny >= hj:
                    if level == 0:
                        status[i] = 0
                    break
                w4 = _weights(npx - F(inx), npy - F(iny))
                diff = _bilinear(lj, inx + xx, iny + yy, w4, 9, False) - Ip
                b1 = F(int((diff * Ix).sum())) * scale
                b2 = F(int((diff * Iy).sum())) * scale
                dx = (A12 * b2 - A22 * b1) * Dt
                dy = (A12 * b1 - A11 * b2) * Dt
                npx, npy = npx + dx, npy + dy
                nx, ny = npx + half, npy + half
                if float(dx) * float(dx) + float(dy) * float(dy) <= eps2:
                    break
                if j > 0 and abs(float(dx + pdx)) < 0.01 and abs(float(dy + pdy)) < 0.01:
                    nx, ny = nx - dx * F(0.5), ny - dy * F(0.5)
                    break
                pdx, pdy = dx, dy
        out[i] = (nx, ny)
    return out, status


def klt_associate(prev_pts, flowed, status, curr_pts, max_match_distance=40.0, min_match_distance=1.5,
                  max_org_feat_dist=1.0):
    """CTracker.cpp:515-545 transliterated (sequential loop)."""
    prev_pts = np.asarray(prev_pts, np.float32)
    flowed = np.asarray(flowed, np.float32)
    curr = np.asarray(curr_pts, np.float64)
    curr_f = curr.astype(np.float32)
    maxDistSq, minDistSq = max_match_distance ** 2, min_match_distance ** 2
    maxFeatDistSq = max_org_feat_dist ** 2
    m = len(curr)
    matchDistance = [-1.0] * m
    matchStatus = [False] * m
    matchedIdx = [-1] * m
    prevIdx, currIdx = [], []
    if m == 0:
        return np.zeros(0, np.int32), np.zeros(0, np.int32)
    for i in range(len(prev_pts)):
        if not status[i]:
            continue
        c = flowed[i]
        dd = (curr[:, 0] - float(c[0])) ** 2 + (curr[:, 1] - float(c[1])) ** 2
        idx = int(np.argmin(dd))  # first minimum
        ex, ey = c[0] - curr_f[idx, 0], c[1] - curr_f[idx, 1]
        e = ex * ex + ey * ey
        px, py = prev_pts[i, 0] - c[0], prev_pts[i, 1] - c[1]
        d = px * px + py * py
        if d < maxDistSq and e < maxFeatDistSq and d > minDistSq and (matchDistance[idx] >= e or
                                                                        matchDistance[idx] == -1):
            if matchStatus[idx]:
                prevIdx[matchedIdx[idx]] = i
            else:
                prevIdx.append(i)
                currIdx.append(idx)
                matchStatus[idx] = True
                matchedIdx[idx] = len(prevIdx) - 1
            matchDistance[idx] = float(e)
    return np.array(prevIdx, np.int32), np.array(currIdx, np.int32)
