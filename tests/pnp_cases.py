"""Seeded PnP scenes shared by the CPU oracle tests and the GPU parity
tests (pose of a keyframe-like camera over map points, pixel noise, gross
outliers), with the reference's intrinsics (main/main.cpp:47-50)."""
import numpy as np

from oracle import pnp_oracle as P

K = np.array([[1072.606693272117800, 0.0, 648.780750477178910],
              [0.0, 1067.197515608619600, 364.503435962496890],
              [0.0, 0.0, 1.0]])


def scene(n, seed, noise=0.5, outliers=0.2, planar=False, depth=6.0):
    rng = np.random.default_rng(seed)
    X = rng.uniform(-1, 1, (n, 3))
    if planar:
        X[:, 2] = 0.0
    rv = rng.normal(0, 0.2, 3)
    tv = np.array([rng.normal(0, 0.3), rng.normal(0, 0.3), depth + rng.normal(0, 0.5)])
    R = P.rodrigues_v2m(rv)
    x = X @ R.T + tv
    uv = x[:, :2] / x[:, 2:] * [K[0, 0], K[1, 1]] + [K[0, 2], K[1, 2]]
    uv = uv + rng.normal(0, noise, uv.shape)
    k = int(round(outliers * n))
    if k:
        bad = rng.choice(n, k, replace=False)
        uv[bad] += rng.uniform(-300, 300, (k, 2))
    return X, uv, rv, tv


CASES = [  # (n, seed, noise, outliers, planar)
    (5, 1, 0.0, 0.0, False),
    (6, 2, 0.3, 0.0, False),
    (40, 3, 0.5, 0.2, False),
    (300, 4, 0.5, 0.2, False),
    (300, 5, 1.0, 0.5, False),
    (2000, 6, 0.5, 0.3, False),
    (200, 7, 0.5, 0.2, True),
    (120, 8, 0.2, 0.9, False),
]
