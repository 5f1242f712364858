"""Synthetic grey video for the tracker config C5: a
textured plane under smooth similarity motion, rendered on the host.

The texture is two-octave value noise (random lattice values, bilinear
between nodes), which has trackable structure everywhere.  Frame k shows
texture point q at pixel  x = s_k R(theta_k) (q - c) + c + t_k,  so the true
position of any tracked point in any frame is known in closed form — the
size-independent property the tracker tests check against.  Per-frame
image motion is 3-10 px, inside the (1.5, 40) px gates of
CTracker.cpp:30-31.  Host data only (no device code).
"""
from __future__ import annotations

import numpy as np


class SyntheticVideo:
    def __init__(self, width: int = 1280, height: int = 720, seed: int = 0x5F3D2017 + 5, speed: float = 5.0,
                 spacing=(11.0, 4.5), amplitude=(150.0, 70.0)):
        self.w, self.h = int(width), int(height)
        self.c = np.array([(self.w - 1) / 2.0, (self.h - 1) / 2.0])
        rng = np.random.default_rng(seed)
        self.speed = float(speed)
        self.phase = rng.uniform(0, 2 * np.pi, 3)
        self.octaves = []
        margin = 200.0 + 40.0 * 300  # texture extent covers long sequences
        for sp, amp in zip(spacing, amplitude):
            n = int(2 * margin / sp) + 4
            self.octaves.append((sp, amp, rng.uniform(-1.0, 1.0, (n, n)), margin))

    # ---- motion ---------------------------------------------------------
    def pose(self, k: int):
        """(scale, theta, t) of frame k: a drifting, slowly turning similarity."""
        k = float(k)
        th = 0.004 * np.sin(0.05 * k + self.phase[0])
        s = 1.0 + 0.01 * np.sin(0.03 * k + self.phase[1])
        t = self.speed * np.array([k * np.cos(0.3) + 3.0 * np.sin(0.11 * k), k * np.sin(0.3) + 3.0 * np.cos(0.07 * k)])
        return s, th, t

    def _A(self, k):
        s, th, t = self.pose(k)
        R = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
        return s * R, t

    def to_texture(self, k: int, x: np.ndarray) -> np.ndarray:
        A, t = self._A(k)
        return (np.asarray(x, np.float64) - self.c - t) @ np.linalg.inv(A).T + self.c

    def from_texture(self, k: int, q: np.ndarray) -> np.ndarray:
        A, t = self._A(k)
        return (np.asarray(q, np.float64) - self.c) @ A.T + self.c + t

    def map_points(self, k0: int, k1: int, x: np.ndarray) -> np.ndarray:
        """True positions in frame k1 of pixels x of frame k0."""
        return self.from_texture(k1, self.to_texture(k0, x))

    # ---- rendering -------------------------------------------------------
    def _texture(self, q: np.ndarray) -> np.ndarray:
        val = np.full(q.shape[:-1], 128.0)
        for sp, amp, lat, margin in self.octaves:
            u = (q[..., 0] + margin) / sp
            v = (q[..., 1] + margin) / sp
            iu = np.clip(np.floor(u).astype(np.int64), 0, lat.shape[1] - 2)
            iv = np.clip(np.floor(v).astype(np.int64), 0, lat.shape[0] - 2)
            fu, fv = u - iu, v - iv
            val += amp * ((1 - fu) * (1 - fv) * lat[iv, iu] + fu * (1 - fv) * lat[iv, iu + 1] +
                          (1 - fu) * fv * lat[iv + 1, iu] + fu * fv * lat[iv + 1, iu + 1])
        return val

    def frame(self, k: int) -> np.ndarray:
        ys, xs = np.mgrid[0:self.h, 0:self.w]
        x = np.stack([xs, ys], axis=-1).astype(np.float64)
        q = self.to_texture(k, x.reshape(-1, 2)).reshape(self.h, self.w, 2)
        return np.clip(np.rint(self._texture(q)), 0, 255).astype(np.uint8)

    # ---- features ----------------------------------------------------------
    def features(self, k: int, n: int, rng: np.random.Generator, border: float = 40.0) -> np.ndarray:
        """n feature positions (double) spread over frame k's interior."""
        x = rng.uniform(border, self.w - border, n)
        y = rng.uniform(border, self.h - border, n)
        return np.stack([x, y], axis=1)

    def detections(self, k0: int, k1: int, prev_pts: np.ndarray, rng: np.random.Generator, jitter: float = 0.15,
                   n_extra: int = 100, drop: float = 0.1) -> np.ndarray:
        """Detected points of frame k1: the true images of frame k0's points
        (jittered, a fraction dropped) plus unrelated detections, shuffled."""
        true = self.map_points(k0, k1, prev_pts)
        keep = rng.uniform(size=len(true)) >= drop
        det = true[keep] + rng.normal(0, jitter, (int(keep.sum()), 2))
        extra = self.features(k1, n_extra, rng, border=5.0)
        det = np.concatenate([det, extra])
        return det[rng.permutation(len(det))]
