"""The pass schedules of k_pnp_epnp's 12x12 Jacobi SVD (sfm_amd/csrc/
svd_schedule.h, pnp_kernels.hip cv_svd12_lanes) restated in Python: the
kernel's control flow (head / tail+head / tail passes, the per-sweep
"turned" flags, the 30-sweep bound) run pass by pass gives bitwise the
sequential sweep order of OpenCV's JacobiSVDImpl_ (oracle/pnp_oracle.py
cv_svd with tree=True), on EPnP-like matrices and on edge cases (nothing to
rotate, only late pairs to rotate).  CPU only."""
import math
import os
import re
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import pnp_oracle as P  # noqa: E402  (the checker)
from tools import svd_schedule  # noqa: E402

HEADER = os.path.join(ROOT, "sfm_amd", "csrc", "svd_schedule.h")
EPS = P.DBL_EPS * 10


def _tables(prefix=""):
    text = open(HEADER).read()
    out = {}
    for name in ("Pro", "Per", "Epi"):
        n = [int(x) for x in re.search(rf"kSvd{prefix}{name}N\[\d+\] = \{{([^}}]*)\}}", text).group(1).split(",")]
        rows = {}
        for key in "IJT":
            body = re.search(rf"kSvd{prefix}{name}{key}\[\d+\]\[\d\] = \{{(.*)\}};", text).group(1)
            rows[key] = [[int(v) for v in grp.split(",")] for grp in re.findall(r"\{([^{}]*)\}", body)]
        out[name] = [(n[p], list(zip(rows["I"][p], rows["J"][p], rows["T"][p]))) for p in range(len(n))]
    return out


def _seq(vals):
    acc = 0.0
    for v in vals:
        acc += v
    return acc


def _rotate(At, W, i, j, ssum=P.tree16):
    """One rotation of JacobiSVDImpl_ on rows i, j (ssum: the kernel's sums --
    tree16 for the 12x12, sequential for cv::solve's); None if it is skipped."""
    a, b = W[i], W[j]
    p = ssum([x * y for x, y in zip(At[i], At[j])])
    if abs(p) <= EPS * math.sqrt(a * b):
        return None
    p *= 2
    beta = a - b
    gamma = math.sqrt(p * p + beta * beta)
    if beta < 0:
        s = math.sqrt(((gamma - beta) * 0.5) / gamma)
        c = p / (gamma * s * 2)
    else:
        c = math.sqrt((gamma + beta) / (gamma * 2))
        s = p / (gamma * c * 2)
    ri = [c * x + s * y for x, y in zip(At[i], At[j])]
    rj = [-s * x + c * y for x, y in zip(At[i], At[j])]
    return ri, rj, ssum([x * x for x in ri]), ssum([x * x for x in rj])


def sequential(A, ssum=P.tree16):
    nr = A.shape[1]
    At = [list(map(float, A[:, i])) for i in range(nr)]
    W = [ssum([x * x for x in r]) for r in At]
    sweeps = 0
    for _ in range(30):
        sweeps += 1
        changed = False
        for i in range(nr - 1):
            for j in range(i + 1, nr):
                r = _rotate(At, W, i, j, ssum)
                if r:
                    At[i], At[j], W[i], W[j] = r
                    changed = True
        if not changed:
            break
    return At, W, sweeps


def scheduled(A, tabs, ssum=P.tree16):
    nr = A.shape[1]
    At = [list(map(float, A[:, i])) for i in range(nr)]
    W = [ssum([x * x for x in r]) for r in At]
    ch = [False, False]

    def run(name):
        for n, slots in tabs[name]:
            res = [(i, j, t, _rotate(At, W, i, j, ssum)) for i, j, t in slots[:n]]  # disjoint rows: pre-pass values
            assert len({r for i, j, _, _ in res for r in (i, j)}) == 2 * n
            for i, j, t, r in res:
                if r:
                    At[i], At[j], W[i], W[j] = r
                    ch[t] = True

    s, head, sweeps = 0, True, 1
    while True:
        if head:
            run("Pro")
        head = False
        if ch[1] and s + 1 < 30:
            ch[0] = ch[1] = False
            run("Per")
            s += 1
            sweeps += 1
        else:
            turned = ch[1]
            ch[0] = False
            run("Epi")
            if not (turned or ch[0]):
                break
            s += 1
            if s >= 30:
                break
            sweeps += 1
            ch[1] = False
            head = True
    return At, W, sweeps


def test_header_is_generated():
    assert open(HEADER).read() == svd_schedule.header_text()


def test_schedules_cover_the_sweep_in_dependency_order():
    tabs = _tables()
    k = svd_schedule.K_HEAD
    pairs = svd_schedule.PAIRS
    for name, want in (("Pro", [(i, j, 1) for i, j in pairs[:k]]),
                       ("Epi", [(i, j, 0) for i, j in pairs[k:]]),
                       ("Per", [(i, j, 0) for i, j in pairs[k:]] + [(i, j, 1) for i, j in pairs[:k]])):
        seen = [s for n, slots in tabs[name] for s in slots[:n]]
        assert sorted(seen) == sorted(want)
        # every rotation after the latest earlier one on each of its rows
        when = {}
        for p, (n, slots) in enumerate(tabs[name]):
            for s in slots[:n]:
                when[s] = p
        last = {}
        for s in want:
            for r in s[:2]:
                if r in last:
                    assert when[last[r]] < when[s], (name, last[r], s)
            last[s[0]] = last[s[1]] = s
    assert len(tabs["Per"]) == 18 and len(tabs["Pro"]) + len(tabs["Epi"]) == 26


def _epnp_like(rng):
    M = rng.standard_normal((10, 12)) * rng.uniform(0.1, 10, 12)
    M[:, rng.integers(0, 12)] *= 1e-3
    return M.T @ M


@pytest.mark.parametrize("seed", range(6))
def test_scheduled_sweeps_bitwise_sequential(seed):
    rng = np.random.default_rng(seed)
    tabs = _tables()
    A = _epnp_like(rng)
    At0, W0, sw0 = sequential(A)
    At1, W1, sw1 = scheduled(A, tabs)
    assert At0 == At1 and W0 == W1 and sw0 == sw1


def test_edge_cases_nothing_to_turn_and_late_pairs_only():
    tabs = _tables()
    D = np.diag(np.arange(1.0, 13.0))           # orthogonal rows: one empty sweep
    assert sequential(D) == scheduled(D, tabs)
    L = np.diag(np.arange(1.0, 13.0))           # only pairs among rows 9..11 (all in the tail)
    L[9, 11] = L[11, 9] = 0.5
    L[10, 11] = L[11, 10] = 0.25
    a, b = sequential(L), scheduled(L, tabs)
    assert a == b and a[2] >= 2


@pytest.mark.parametrize("nr,prefix", [(4, "L4"), (5, "L5")])
def test_small_lane_schedules_bitwise_sequential(nr, prefix):
    """cv::solve's 6 x nr SVDs (EPnP beta cases) one row per lane
    (cv_linalg.h cv_svd_sweeps_lanes): schedule coverage and dependency
    order, then bitwise the sequential sweeps on random and EPnP-like L."""
    tabs = _tables(prefix)
    head = dict(svd_schedule.SMALL)[nr][1]
    pairs = [(i, j) for i in range(nr - 1) for j in range(i + 1, nr)]
    for name, want in (("Pro", [(i, j, 1) for i, j in pairs[:head]]),
                       ("Epi", [(i, j, 0) for i, j in pairs[head:]]),
                       ("Per", [(i, j, 0) for i, j in pairs[head:]] + [(i, j, 1) for i, j in pairs[:head]])):
        seen = [s for n, slots in tabs[name] for s in slots[:n]]
        assert sorted(seen) == sorted(want)
    rng = np.random.default_rng(nr)
    for trial in range(20):
        A = rng.standard_normal((6, nr)) * rng.uniform(0.01, 100, nr)
        if trial % 4 == 3:
            A[:, -1] = A[:, 0] * 0.5 + 1e-9 * rng.standard_normal(6)   # near rank-deficient
        assert sequential(A, _seq) == scheduled(A, tabs, _seq)
    E = np.zeros((6, nr))
    E[np.arange(nr), np.arange(nr)] = np.arange(1.0, nr + 1)            # orthogonal columns: nothing turns
    assert sequential(E, _seq) == scheduled(E, tabs, _seq)
