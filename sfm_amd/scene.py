"""Synthetic bundle-adjustment scenes through the C generator.

Configurations named by BASELINE.json:
  C1  20 cams /     2k points /    20k observations  (CPU plumbing)
  C2 100 cams /    50k points /   500k observations  (Jacobian kernel)
  C3 500 cams /   200k points /     2M observations  (full LM + Schur, 1 GPU)
  C4 2000 cams /    1M points /    10M observations  (landmark-sharded, 8 GPUs)
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ._ffi import check, lib, ptr

CONFIGS = {
    "C1": (20, 2_000),
    "C2": (100, 50_000),
    "C3": (500, 200_000),
    "C4": (2_000, 1_000_000),
}
SEED_BASE = 0x5F3D2017
VIEWS = 10


@dataclass
class Scene:
    n_cams: int
    n_pts: int            # points in this slice
    n_pts_total: int
    p_begin: int
    K: np.ndarray         # [C][9]
    rot_true: np.ndarray  # [C][3]
    t_true: np.ndarray
    X_true: np.ndarray    # [P][3]
    rot: np.ndarray       # initial guess
    t: np.ndarray
    X: np.ndarray
    uv: np.ndarray        # [N][2]
    cam_idx: np.ndarray   # [N] int32
    pt_idx: np.ndarray    # [N] int32 (relative to p_begin)

    @property
    def n_obs(self) -> int:
        return int(self.uv.shape[0])

    def copy_params(self):
        return self.rot.copy(), self.t.copy(), self.X.copy()


def generate(n_cams: int, n_pts: int, views: int = VIEWS, seed: int = SEED_BASE, p_begin: int = 0,
             p_end: int | None = None, pixel_sigma: float = 0.5, pt_sigma: float = 0.01, rot_sigma: float = 1e-3,
             t_sigma: float = 0.01) -> Scene:
    if p_end is None:
        p_end = n_pts
    P = p_end - p_begin
    C = n_cams
    N = P * views
    K = np.zeros((C, 9))
    rt, tt, ri, ti = (np.zeros((C, 3)) for _ in range(4))
    Xt, Xi = np.zeros((P, 3)), np.zeros((P, 3))
    uv = np.zeros((N, 2))
    ci = np.zeros(N, np.int32)
    pi = np.zeros(N, np.int32)
    rc = lib().sfm_scene_generate(C, n_pts, p_begin, p_end, views, seed & 0xFFFFFFFFFFFFFFFF, pixel_sigma,
                                  pt_sigma, rot_sigma, t_sigma, ptr(K), ptr(rt), ptr(tt), ptr(Xt), ptr(ri), ptr(ti),
                                  ptr(Xi), ptr(uv), ptr(ci), ptr(pi))
    check(rc, "sfm_scene_generate")
    return Scene(C, P, n_pts, p_begin, K, rt, tt, Xt, ri, ti, Xi, uv, ci, pi)


def config(name: str, **kw) -> Scene:
    idx = list(CONFIGS).index(name) + 1
    C, P = CONFIGS[name]
    return generate(C, P, seed=SEED_BASE + idx, **kw)
