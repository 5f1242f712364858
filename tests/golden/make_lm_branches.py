#!/usr/bin/env python3
"""Generates tests/golden/lm_branches.{json,npz}: oracle trajectories of the
LM-branch cases of tests/lm_cases.py, each cross-checked against a dense
numpy restatement of Ceres-1.12's trust-region loop written independently of
the C++ oracle (the loop behind ceres::Solve at
/root/reference/CTracker.cpp:700-701, options CTracker.cpp:571-577).

The reference has no tests or fixtures for this path and cannot be built
here (Ceres / Eigen / OpenCV absent): the oracle is pinned by
this second restatement, not by the reference (parity unpinned at the Ceres
boundary).  The numpy loop solves the full damped normal equations densely
(no Schur complement, numpy's LAPACK Cholesky), so agreement of the
accept / reject / invalid sequence, radii and costs is evidence for the
bookkeeping, not for a shared arithmetic path.

Symbolic options of lm_cases.cases() are resolved here from the
default-option trajectory of the same scene and VERIFIED: the stop they
target must fire at the intended iteration with a >= 1.5x margin on both
sides, so that a different summation order cannot move it.

Run from the repository root:  python tests/golden/make_lm_branches.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from make_golden import torch_residuals_jacobians  # noqa: E402  (torch fp64 autograd of the functor)

FIELDS = ["max_num_iterations", "max_num_consecutive_invalid_steps", "jacobi_scaling", "function_tolerance",
          "gradient_tolerance", "parameter_tolerance", "initial_trust_region_radius", "max_trust_region_radius",
          "min_trust_region_radius", "min_lm_diagonal", "max_lm_diagonal", "min_relative_decrease"]


def seq_of(trace):
    return "".join("I" if not it["step_is_valid"] else ("A" if it["step_is_successful"] else "R") for it in trace[1:])


# --------------------------------------------------------------------------
# dense numpy restatement of TrustRegionMinimizer + LevenbergMarquardtStrategy
def np_lm(uv, cam, pt, K9, rot, t, X, mode, o):
    C, P = rot.shape[0], X.shape[0]
    cams_var, pts_var = mode != 0, mode != 1
    used_c = np.zeros(C, bool); used_c[cam] = True
    used_p = np.zeros(P, bool); used_p[pt] = True
    full = np.concatenate([np.hstack([rot, t]).ravel(), X.ravel()])
    act = np.zeros(full.size, bool)
    if cams_var:
        act[:6 * C] = np.repeat(used_c, 6)
    if pts_var:
        act[6 * C:] = np.repeat(used_p, 3)
    N = uv.shape[0]

    def evaluate(xf, want_j):
        xc = xf[:6 * C].reshape(C, 6)
        res, jac = torch_residuals_jacobians(uv, cam, pt, K9, xc[:, :3], xc[:, 3:], xf[6 * C:].reshape(P, 3))
        r = res.reshape(-1)
        if not want_j:
            return r, None
        J = np.zeros((2 * N, full.size))
        rows = np.arange(2 * N).reshape(N, 2)
        for k in range(6):
            J[rows, (6 * cam + k)[:, None]] = jac[:, :, k]
        for k in range(3):
            J[rows, (6 * C + 3 * pt + k)[:, None]] = jac[:, :, 6 + k]
        return r, J[:, act]

    x = full.copy()
    r, J = evaluate(x, True)
    cost = 0.5 * r @ r
    scale = 1.0 / (1.0 + np.sqrt((J * J).sum(0))) if o["jacobi_scaling"] else np.ones(J.shape[1])
    Js = J * scale
    gmax = float(np.abs(J.T @ r).max())
    trace = [dict(iteration=0, step_is_valid=1, step_is_successful=1, cost=cost, gradient_max_norm=gmax,
                  trust_region_radius=o["initial_trust_region_radius"])]
    if gmax <= o["gradient_tolerance"]:
        return trace, "CONVERGENCE", x
    radius, decrease, reuse, diag, n_inv, it = o["initial_trust_region_radius"], 2.0, False, None, 0, 0
    xnorm = np.linalg.norm(x[act])
    while True:
        if it >= o["max_num_iterations"]:
            return trace, "NO_CONVERGENCE", x
        it += 1
        if not reuse:
            diag = np.clip((Js * Js).sum(0), o["min_lm_diagonal"], o["max_lm_diagonal"])
        reuse = True
        A = Js.T @ Js + np.diag(diag / radius)
        ok = True
        try:
            L = np.linalg.cholesky(A)
            step = -np.linalg.solve(L.T, np.linalg.solve(L, Js.T @ r))
            ok = bool(np.all(np.isfinite(step)))
        except np.linalg.LinAlgError:
            ok = False
        rec = dict(iteration=it, step_is_valid=0, step_is_successful=0)
        if ok:
            mr = Js @ step
            mcc = -(mr @ (r + mr / 2.0))
            rec["step_is_valid"] = int(mcc >= 0.0)
        if not rec["step_is_valid"]:
            n_inv += 1
            if n_inv >= o["max_num_consecutive_invalid_steps"]:
                rec.update(cost=cost, trust_region_radius=radius)
                trace.append(rec)
                return trace, "FAILURE", x
            radius /= decrease
            decrease *= 2
            rec.update(cost=cost, trust_region_radius=radius)
            trace.append(rec)
            if radius < o["min_trust_region_radius"]:
                return trace, "CONVERGENCE", x
            continue
        n_inv = 0
        xn = x.copy()
        xn[act] += step * scale
        rn, _ = evaluate(xn, False)
        new_cost = 0.5 * rn @ rn if np.all(np.isfinite(rn)) else np.finfo(float).max
        step_norm = float(np.linalg.norm(x - xn))
        rec["step_norm"] = step_norm
        if step_norm <= o["parameter_tolerance"] * (xnorm + o["parameter_tolerance"]):
            rec.update(cost=cost, trust_region_radius=radius, stop="parameter")
            trace.append(rec)
            return trace, "CONVERGENCE", x
        dc = cost - new_cost
        if abs(dc) <= o["function_tolerance"] * cost:
            rec.update(cost=cost, trust_region_radius=radius, stop="function")
            trace.append(rec)
            return trace, "CONVERGENCE", x
        rho = dc / mcc
        rec["relative_decrease"] = rho
        if rho > o["min_relative_decrease"]:
            rec["step_is_successful"] = 1
            radius = min(o["max_trust_region_radius"], radius / max(1 / 3, 1 - (2 * rho - 1) ** 3))
            decrease, reuse = 2.0, False
            x = xn
            xnorm = np.linalg.norm(x[act])
            r, J = evaluate(x, True)
            cost = 0.5 * r @ r
            Js = J * scale
            gmax = float(np.abs(J.T @ r).max())
        else:
            radius /= decrease
            decrease *= 2
        rec.update(cost=cost, trust_region_radius=radius, gradient_max_norm=gmax)
        trace.append(rec)
        if rec["step_is_successful"] and gmax <= o["gradient_tolerance"]:
            return trace, "CONVERGENCE", x
        if not rec["step_is_successful"] and radius < o["min_trust_region_radius"]:
            return trace, "CONVERGENCE", x


def opts_dict(O, **kw):
    o = O.default_options(**kw)
    return {f: getattr(o, f) for f in FIELDS}


def run_oracle(O, s, mode, od, max_iter=None):
    kw = dict(od)
    if max_iter is not None:
        kw["max_num_iterations"] = max_iter
    r, t, X = s.copy_params()
    sm, tr = O.solve(s.uv, s.cam_idx, s.pt_idx, s.K, r, t, X, mode=mode, options=O.default_options(**kw))
    return sm, tr, (r, t, X)


def resolve(O, L, s, mode, spec):
    """Numeric options for the symbolic entries of `spec`, verified margins."""
    base = opts_dict(O)
    _, btr, _ = run_oracle(O, s, mode, base)
    od = opts_dict(O, **{k: v for k, v in spec.items() if not isinstance(v, str)})
    for k, v in spec.items():
        if v == "after_first_reject":
            # Ceres requires min_trust_region_radius <= initial radius
            # (TrustRegionOptionsAreValid): fire at the first rejection that
            # takes the radius below the initial one, between its radius and
            # every radius an earlier rejection left
            r0 = od["initial_trust_region_radius"]
            rej = [(i, it["trust_region_radius"]) for i, it in enumerate(btr) if i > 0 and not it["step_is_successful"]]
            j, rj = next((i, r) for i, r in rej if r < r0 / 1.69)
            floor = min([r0] + [r for i, r in rej if i < j])
            od[k] = float(np.sqrt(rj * floor))
            assert floor / od[k] >= 1.3 and od[k] / rj >= 1.3
        elif v == "between_gradients":
            g = [(i, it["gradient_max_norm"]) for i, it in enumerate(btr) if it["step_is_successful"]]
            a, b = next((a, b) for a, b in zip(g, g[1:]) if b[1] < a[1] / 4 and b[0] >= 2)
            od[k] = float(np.sqrt(a[1] * b[1]))
        elif v == "between_steps":
            # fire at the first valid step whose norm is < 1/4 of every earlier
            # valid step, measured against |x| at that iteration
            ftr = run_oracle(O, s, mode, od)[1]
            valid = [(i, it["step_norm"]) for i, it in enumerate(ftr) if i > 0 and it["step_is_valid"]]
            j = next(i for (i, sn) in valid[1:] if sn < min(s2 for (i2, s2) in valid if i2 < i) / 4)
            xn = L.x_norm(*run_oracle(O, s, mode, od, max_iter=j - 1)[2])
            s_prev = min(s2 for (i2, s2) in valid if i2 < j)
            s_j = dict(valid)[j]
            od[k] = float(np.sqrt(s_prev * s_j)) / xn
    return od


def main():
    import lm_cases as L
    from oracle import ffi as O

    cases = L.cases()
    out, arrays, report = {}, {}, []
    for name, (build, spec, mode) in cases.items():
        s = build()
        od = resolve(O, L, s, mode, spec)
        sm, tr, (r, t, X) = run_oracle(O, s, mode, od)
        ntr, nterm, nx = np_lm(s.uv, s.cam_idx, s.pt_idx, s.K, s.rot.copy(), s.t.copy(), s.X.copy(), mode, od)
        term = ["CONVERGENCE", "NO_CONVERGENCE", "FAILURE"][sm["termination_type"]]
        so, sn = seq_of(tr), seq_of(ntr)
        gauge = name.startswith("gauge")
        if gauge:
            # decisive prefix only (then rounding noise decides); the radius clamp must be reached
            k = L.decisive_prefix(tr)
            assert so[:k] == sn[:k], (name, so, sn)
            tr_c, ntr_c = tr[:k + 1], ntr[:k + 1]
        else:
            assert so == sn, (name, so, sn)
            assert term == nterm, (name, term, nterm)
            tr_c, ntr_c = tr, ntr
        cost_rel = max(abs(a["cost"] - b["cost"]) / b["cost"] for a, b in zip(tr_c, ntr_c))
        rad_rel = max(abs(a["trust_region_radius"] - b["trust_region_radius"]) / b["trust_region_radius"]
                      for a, b in zip(tr_c, ntr_c))
        final_rel = abs(tr[-1]["cost"] - ntr[-1]["cost"]) / ntr[-1]["cost"]
        C_, P_ = s.rot.shape[0], s.X.shape[0]
        nxc = nx[:6 * C_].reshape(C_, 6)
        res_fn = lambda *a: O.residuals_jacobians(*a, jacobian=False)[0]
        gi_res, gi_al = L.gauge_invariant_diff(res_fn, s, (r, t, X),
                                               (nxc[:, :3], nxc[:, 3:], nx[6 * C_:].reshape(P_, 3)))
        per_it = [abs(a["cost"] - b["cost"]) / b["cost"] for a, b in zip(tr_c, ntr_c)]
        C = s.rot.shape[0]
        xf = np.concatenate([np.hstack([r, t]).ravel(), X.ravel()])
        par_rel = float(np.max(np.abs(xf - nx) / np.maximum(np.abs(nx), 1e-3)))
        # decision margins of the oracle's trajectory (how far each rho is from the threshold)
        rhos = [it["relative_decrease"] for it in tr[1:-1] if it["step_is_valid"]]
        margin = min((abs(x - od["min_relative_decrease"]) for x in rhos), default=float("inf"))
        report.append(f"{name:18s} mode {mode} {term:14s} {so:28s} cost {cost_rel:.1e} final {final_rel:.1e} radius {rad_rel:.1e} "
                      f"params {par_rel:.1e} gauge-inv res {gi_res:.1e} aligned {gi_al:.1e} rho-margin {margin:.3f}")
        out[name] = dict(mode=mode, options=od, summary=sm, trace=tr, numpy_sequence=sn, numpy_termination=nterm,
                         numpy_costs=[it["cost"] for it in ntr], numpy_cost_rel_diff=per_it,
                         numpy_radius_rel_diff=[abs(a["trust_region_radius"] - b["trust_region_radius"]) /
                                                b["trust_region_radius"] for a, b in zip(tr_c, ntr_c)],
                         numpy_param_max_rel=par_rel, numpy_residual_max_abs=gi_res, numpy_aligned_max_rel=gi_al, numpy_final_cost=ntr[-1]["cost"],
                         decisive_prefix=L.decisive_prefix(tr) if gauge else len(tr) - 1,
                         n_obs=int(s.n_obs), n_cams=int(C), n_pts=int(s.X.shape[0]))
        arrays[f"{name}__rot"], arrays[f"{name}__t"], arrays[f"{name}__X"] = r, t, X
    with open(os.path.join(HERE, "lm_branches.json"), "w") as f:
        json.dump(out, f, indent=0)
    np.savez_compressed(os.path.join(HERE, "lm_branches.npz"), **arrays)
    print("\n".join(report))


if __name__ == "__main__":
    main()
