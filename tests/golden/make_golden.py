#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/.

The reference (hulop/SfM) has no tests, fixtures or sample data for the hot
path and cannot be built or run here (OpenCV / Ceres / Eigen / BRISK absent;
SURVEY.md §8c), so every vector below is produced by restatements written
for this repository, each independent of the C++ oracle it checks:

  jacobian_small.npz  residual + 2x9 Jacobian of BAStructAndPoseFunctor
                      (CTracker.cpp:585-604) by torch fp64 autograd through
                      ceres::AngleAxisRotatePoint (both branches).
  lm_micro.json       Levenberg-Marquardt trace + final parameters of a
                      3-camera / 40-point scene by a dense numpy restatement
                      of Ceres 1.12's trust-region loop (no Schur complement:
                      normal equations formed and factored densely).
  lm_c1.npz/.json     the C++ oracle's trace and final parameters on config
                      C1 (20 / 2k / 20k), cross-checked here against the
                      numpy restatement's step sequence.
  matcher.npz         matchFeatures (CTracker.cpp:211-250) on seeded
                      descriptors with planted ties and replacements, by a
                      pure-Python restatement of the sequential loop.

Run from the repository root:  python tests/golden/make_golden.py
(needs libsfm_amd.so for the scene generator and oracle/liboracle.so).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

DBL_EPS = np.finfo(np.float64).eps


# --------------------------------------------------------------------------
# torch restatement of the functor
def torch_functor(R, t, X, K, uv):
    import torch
    theta2 = (R * R).sum(-1)
    big = theta2 > DBL_EPS
    theta = torch.sqrt(torch.where(big, theta2, torch.ones_like(theta2)))
    c, s = torch.cos(theta), torch.sin(theta)
    w = R / theta[..., None]
    wxp = torch.cross(w, X, dim=-1)
    tmp = (w * X).sum(-1) * (1 - c)
    rod = X * c[..., None] + wxp * s[..., None] + w * tmp[..., None]
    lin = X + torch.cross(R, X, dim=-1)
    p = torch.where(big[..., None], rod, lin) + t
    xp, yp = p[..., 0] / p[..., 2], p[..., 1] / p[..., 2]
    r0 = K[..., 0] * xp + K[..., 1] * yp + K[..., 2] - uv[..., 0]
    r1 = K[..., 4] * yp + K[..., 5] - uv[..., 1]
    return torch.stack([r0, r1], -1)


def torch_residuals_jacobians(uv, cam, pt, K9, rot, t, X):
    import torch
    from torch.func import jacrev, vmap
    Rb = torch.tensor(rot[cam]); tb = torch.tensor(t[cam]); Xb = torch.tensor(X[pt])
    Kb = torch.tensor(K9[cam]); uvb = torch.tensor(uv)

    def f(params, k, o):
        return torch_functor(params[0:3], params[3:6], params[6:9], k, o)

    P = torch.cat([Rb, tb, Xb], -1)
    res = vmap(f)(P, Kb, uvb)
    jac = vmap(jacrev(f))(P, Kb, uvb)
    return res.numpy(), jac.numpy()


# --------------------------------------------------------------------------
# dense numpy restatement of Ceres-1.12 LM
def np_functor(Rv, tv, Xv, k, uv):
    th2 = Rv @ Rv
    if th2 > DBL_EPS:
        th = np.sqrt(th2)
        w = Rv / th
        p = Xv * np.cos(th) + np.cross(w, Xv) * np.sin(th) + w * (w @ Xv) * (1 - np.cos(th))
    else:
        p = Xv + np.cross(Rv, Xv)
    p = p + tv
    xp, yp = p[0] / p[2], p[1] / p[2]
    return np.array([k[0] * xp + k[1] * yp + k[2] - uv[0], k[4] * yp + k[5] - uv[1]])


def np_lm(uv, cam, pt, K9, rot, t, X, max_iter=50):
    C, P = rot.shape[0], X.shape[0]
    n = 6 * C + 3 * P
    x = np.concatenate([np.hstack([rot, t]).ravel(), X.ravel()])
    N = uv.shape[0]

    def residuals(xx):
        r = np.zeros(2 * N)
        for i in range(N):
            c, p = cam[i], pt[i]
            r[2 * i:2 * i + 2] = np_functor(xx[6 * c:6 * c + 3], xx[6 * c + 3:6 * c + 6],
                                            xx[6 * C + 3 * p:6 * C + 3 * p + 3], K9[c], uv[i])
        return r

    def jacobian(xx):
        res, jac = torch_residuals_jacobians(uv, cam, pt, K9, xx[:6 * C].reshape(C, 6)[:, :3],
                                             xx[:6 * C].reshape(C, 6)[:, 3:], xx[6 * C:].reshape(P, 3))
        J = np.zeros((2 * N, n))
        for i in range(N):
            c, p = cam[i], pt[i]
            J[2 * i:2 * i + 2, 6 * c:6 * c + 6] = jac[i][:, :6]
            J[2 * i:2 * i + 2, 6 * C + 3 * p:6 * C + 3 * p + 3] = jac[i][:, 6:]
        return res.reshape(-1), J

    r, J = jacobian(x)
    cost = 0.5 * r @ r
    scale = 1.0 / (1.0 + np.sqrt((J * J).sum(0)))
    Js = J * scale
    g = J.T @ r
    trace = [dict(iteration=0, cost=cost, gradient_max_norm=float(np.abs(g).max()), step_is_successful=1)]
    radius, decrease, reuse, diag = 1e4, 2.0, False, None
    it = 0
    while it < max_iter:
        it += 1
        if not reuse:
            diag = np.clip((Js * Js).sum(0), 1e-6, 1e32)
        D = np.sqrt(diag / radius)
        A = Js.T @ Js + np.diag(D * D)
        try:
            L = np.linalg.cholesky(A)
            y = np.linalg.solve(L.T, np.linalg.solve(L, Js.T @ r))
            step = -y
            ok = np.all(np.isfinite(step))
        except np.linalg.LinAlgError:
            ok = False
        reuse = True
        mr = Js @ step if ok else None
        mcc = -(mr @ (r + mr / 2.0)) if ok else 0.0
        if not ok or mcc < 0:
            radius /= decrease; decrease *= 2
            trace.append(dict(iteration=it, cost=cost, step_is_successful=0))
            continue
        delta = step * scale
        xn = x + delta
        newc = 0.5 * np.sum(residuals(xn) ** 2)
        if np.linalg.norm(x - xn) <= 1e-8 * (np.linalg.norm(x) + 1e-8):
            trace.append(dict(iteration=it, cost=cost, step_is_successful=0, stop="parameter"))
            break
        dc = cost - newc
        if abs(dc) <= 1e-6 * cost:
            trace.append(dict(iteration=it, cost=cost, step_is_successful=0, stop="function"))
            break
        rho = dc / mcc
        if rho > 1e-3:
            radius = min(1e16, radius / max(1 / 3, 1 - (2 * rho - 1) ** 3))
            decrease, reuse = 2.0, False
            x = xn
            r, J = jacobian(x)
            cost = 0.5 * r @ r
            Js = J * scale
            trace.append(dict(iteration=it, cost=cost, step_is_successful=1, relative_decrease=rho,
                              trust_region_radius=radius))
        else:
            radius /= decrease; decrease *= 2
            trace.append(dict(iteration=it, cost=cost, step_is_successful=0, relative_decrease=rho,
                              trust_region_radius=radius))
    xc = x[:6 * C].reshape(C, 6)
    return trace, xc[:, :3].copy(), xc[:, 3:].copy(), x[6 * C:].reshape(P, 3).copy()


# --------------------------------------------------------------------------
# pure-Python restatement of matchFeatures (CTracker.cpp:211-250) + knnMatch
def py_match(p0, d0, p1, d1, ratio=0.8, mn=1.5, mx=40.0):
    n0, n1 = len(d0), len(d1)
    if n0 == 0 or n1 < 2:
        return [], []
    x0 = np.unpackbits(d0, axis=1).astype(np.int32)
    x1 = np.unpackbits(d1, axis=1).astype(np.int32)
    dist = (x0[:, None, :] != x1[None, :, :]).sum(-1)
    m0, m1, mdist, slot = [], [], {}, {}
    for i in range(n0):
        order = sorted(range(n1), key=lambda j: (dist[i, j], j))
        j0, j1 = order[0], order[1]
        f0, f1 = np.float32(dist[i, j0]), np.float32(dist[i, j1])
        with np.errstate(divide="ignore", invalid="ignore"):
            rr = float(np.float32(f0 / f1))
        dx, dy = p0[i, 0] - p1[j0, 0], p0[i, 1] - p1[j0, 1]
        dd = dx * dx + dy * dy
        new = j0 not in mdist
        better = (not new) and float(f0) < mdist[j0]
        if dd > mn * mn and dd < mx * mx and rr < ratio and (new or better):
            if new:
                slot[j0] = len(m0); m0.append(i); m1.append(j0)
            else:
                m0[slot[j0]] = i
            mdist[j0] = float(f0)
    return m0, m1


def make_matcher_case(rng, n0, n1, nbytes=64):
    d0 = rng.integers(0, 256, (n0, nbytes), dtype=np.uint8)
    d1 = rng.integers(0, 256, (n1, nbytes), dtype=np.uint8)
    k = min(n0, n1) // 2
    d1[:k] = d0[:k]
    for r in range(k):
        d1[r, rng.integers(0, nbytes, 3)] ^= np.uint8(1 << int(rng.integers(0, 8)))
    # duplicates in the query set compete for one train row (replacement rule)
    if n0 > 8:
        d0[n0 - 4:] = d0[:4]
    # exact 2-NN ties in the train set (tie -> lower train index)
    if n1 > k + 4:
        d1[k:k + 2] = d1[0]
    p0 = rng.uniform(0, 1280, (n0, 2))
    p1 = rng.uniform(0, 1280, (n1, 2))
    p1[:k] = p0[:k] + rng.normal(0, 10, (k, 2))
    if n0 > 8:
        p0[n0 - 4:] = p0[:4] + rng.normal(0, 2, (4, 2))
    return p0, d0, p1, d1


def main():
    import sfm_amd
    from sfm_amd import scene
    from oracle import ffi as O

    out = {}
    # ---- Jacobian fixture -------------------------------------------------
    s = scene.generate(5, 40, views=4, seed=0x1234)
    s.rot[1] = [1e-9, -2e-9, 5e-10]        # first-order branch (theta^2 <= DBL_EPSILON)
    s.rot[2] = [1.5e-8, 0.0, 0.0]          # just above DBL_EPSILON: Rodrigues branch
    s.rot[3] = [2.0, -1.0, 0.5]            # large rotation
    res, jac = torch_residuals_jacobians(s.uv, s.cam_idx, s.pt_idx, s.K, s.rot, s.t, s.X)
    np.savez_compressed(os.path.join(HERE, "jacobian_small.npz"), uv=s.uv, cam_idx=s.cam_idx, pt_idx=s.pt_idx,
                        K=s.K, rot=s.rot, t=s.t, X=s.X, res=res, jac=jac)
    r_o, j_o = O.residuals_jacobians(s.uv, s.cam_idx, s.pt_idx, s.K, s.rot, s.t, s.X)
    out["jacobian_oracle_vs_torch_max_abs"] = float(np.abs(j_o - jac).max())

    # ---- LM micro-scene: numpy restatement -----------------------------
    m = scene.generate(3, 40, views=3, seed=0x77)
    tr_np, rn, tn, Xn = np_lm(m.uv, m.cam_idx, m.pt_idx, m.K, m.rot.copy(), m.t.copy(), m.X.copy())
    ro, to_, Xo = m.copy_params()
    sm_o, tr_o = O.solve(m.uv, m.cam_idx, m.pt_idx, m.K, ro, to_, Xo)
    micro = dict(inputs=dict(uv=m.uv.tolist(), cam_idx=m.cam_idx.tolist(), pt_idx=m.pt_idx.tolist(),
                             K=m.K.tolist(), rot=m.rot.tolist(), t=m.t.tolist(), X=m.X.tolist()),
                 numpy_trace=tr_np, numpy_final=dict(rot=rn.tolist(), t=tn.tolist(), X=Xn.tolist()),
                 oracle_summary=sm_o, oracle_trace=tr_o)
    with open(os.path.join(HERE, "lm_micro.json"), "w") as f:
        json.dump(micro, f, indent=0)
    out["micro_final_param_max_rel_oracle_vs_numpy"] = float(
        np.max(np.abs(Xo - Xn) / np.maximum(np.abs(Xn), 1e-3)))

    # ---- LM on C1: oracle trace ---------------------------------------
    c1 = scene.config("C1")
    r1, t1, X1 = c1.copy_params()
    sm1, tr1 = O.solve(c1.uv, c1.cam_idx, c1.pt_idx, c1.K, r1, t1, X1)
    np.savez_compressed(os.path.join(HERE, "lm_c1.npz"), rot=r1, t=t1, X=X1)
    with open(os.path.join(HERE, "lm_c1.json"), "w") as f:
        json.dump(dict(summary=sm1, trace=tr1, seed=scene.SEED_BASE + 1, cams=20, points=2000), f, indent=0)

    # ---- matcher --------------------------------------------------------
    rng = np.random.default_rng(20171017)
    cases = {}
    for ci, (n0, n1) in enumerate([(40, 36), (200, 180), (3, 2), (12, 1), (0, 5), (64, 64)]):
        p0, d0, p1, d1 = make_matcher_case(rng, n0, n1)
        a, b = py_match(p0, d0, p1, d1)
        cases[f"case{ci}_p0"], cases[f"case{ci}_d0"] = p0, d0
        cases[f"case{ci}_p1"], cases[f"case{ci}_d1"] = p1, d1
        cases[f"case{ci}_idx0"] = np.array(a, np.int32)
        cases[f"case{ci}_idx1"] = np.array(b, np.int32)
    np.savez_compressed(os.path.join(HERE, "matcher.npz"), **cases)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
