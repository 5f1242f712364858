"""GPU: the frame-resident HIP matcher (sfm_matcher_*, CTracker::matchFeatures
overloads, /root/reference/CTracker.cpp:114-149, 211-250, 368-417, 419-477)
against the oracle (oracle/match_oracle.cpp) and the pure-Python restatement
of the sequential loop (tests/golden/make_golden.py::py_match).  Indices must
be bit-exact, order included.

Cases that decide the indices: several queries competing for one train row
(the "better match replaces the slot's query" rule, first minimal query
wins, slot order = first accepted query), exact 2-NN distance ties (lower
train index first), f1 = 0 (0/0 ratio: rejected), fewer than 2 train rows,
the (0, _maxReprErr = 7) window of CSfM.cpp:208-210, 673, the index-subset
overload of the per-frame loop (CSfM.cpp:518) and the whole-frame member
overload on distorted positions (CSfM.cpp:823).
"""
import os
import sys

import numpy as np
import pytest

import sfm_amd
from sfm_amd.matcher import FeatureMatcher
from oracle import ffi as O

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, G)
from make_golden import py_match  # noqa: E402


def _eq(a, b):
    return np.array_equal(np.asarray(a, np.int64), np.asarray(b, np.int64))


def test_committed_matcher_fixture_through_hip():
    z = np.load(os.path.join(G, "matcher.npz"))
    n = len([k for k in z.files if k.endswith("_idx0")])
    tr = sfm_amd.CTracker()
    for ci in range(n):
        a, b = tr.matchFeatures(z[f"case{ci}_p0"], z[f"case{ci}_d0"], z[f"case{ci}_p1"], z[f"case{ci}_d1"])
        assert _eq(a, z[f"case{ci}_idx0"]) and _eq(b, z[f"case{ci}_idx1"]), ci


def _competing_case(rng, n0=300, n1=200, nbytes=64):
    """Queries built from a few train rows with controlled bit flips: many
    queries accept the same train row with equal and decreasing distances."""
    d1 = rng.integers(0, 256, (n1, nbytes), dtype=np.uint8)
    p1 = rng.uniform(100, 1100, (n1, 2))
    src = rng.integers(0, 8, n0)                       # 8 popular train rows
    nflip = rng.integers(0, 6, n0)                     # distance 0..5 (many exact ties)
    d0 = d1[src].copy()
    for i in range(n0):
        bits = rng.choice(8 * nbytes, nflip[i], replace=False)
        for bit in bits:
            d0[i, bit // 8] ^= np.uint8(1 << (bit % 8))
    p0 = p1[src] + rng.normal(0, 6, (n0, 2))
    # exact 2-NN ties: train rows 100 and 101 identical, 102 = 103
    d1[101] = d1[100]
    d1[103] = d1[102]
    d0[:5] = d1[100]
    p0[:5] = p1[100] + 3.0
    return p0, d0, p1, d1


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("window", [(1.5, 40.0), (0.0, 7.0)])
def test_competing_queries_ties_and_windows(seed, window):
    rng = np.random.default_rng(seed)
    p0, d0, p1, d1 = _competing_case(rng)
    with FeatureMatcher(64) as m:
        g0, g1 = m.match(p0, d0, p1, d1, 0.8, *window)
    o0, o1 = O.match_features(p0, d0, p1, d1, 0.8, *window)
    r0, r1 = py_match(p0, d0, p1, d1, 0.8, *window)
    assert _eq(o0, r0) and _eq(o1, r1)
    assert _eq(g0, o0) and _eq(g1, o1)
    # the replacement rule is exercised: fewer slots than accepted queries
    assert len(g0) > 0 and len(set(g1.tolist())) == len(g1)


def test_zero_second_distance_and_tiny_train_sets():
    rng = np.random.default_rng(5)
    d1 = rng.integers(0, 256, (6, 64), dtype=np.uint8)
    d1[1] = d1[0]                                      # query == rows 0 and 1: d0 = d1 = 0 -> 0/0
    p1 = rng.uniform(0, 1280, (6, 2))
    d0 = np.stack([d1[0], d1[2], d1[3]])
    p0 = p1[[0, 2, 3]] + 5.0
    with FeatureMatcher(64) as m:
        for n1 in (6, 2, 1, 0):
            g = m.match(p0, d0, p1[:n1], d1[:n1])
            o = O.match_features(p0, d0, p1[:n1], d1[:n1])
            assert _eq(g[0], o[0]) and _eq(g[1], o[1]), n1
            if n1 < 2:
                assert len(g[0]) == 0                    # reference UB: no matches
        g = m.match(p0[:0], d0[:0], p1, d1)
        assert len(g[0]) == 0
    assert 0 not in O.match_features(p0, d0, p1, d1)[0]  # the 0/0 query is rejected


@pytest.mark.parametrize("n0,n1", [(2000, 2000), (5000, 4000), (63, 65), (700, 129)])
def test_large_frames_match_oracle(n0, n1):
    rng = np.random.default_rng(n0 + n1)
    d0 = rng.integers(0, 256, (n0, 64), dtype=np.uint8)
    d1 = rng.integers(0, 256, (n1, 64), dtype=np.uint8)
    k = min(n0, n1) // 2
    d1[:k] = d0[:k]
    flips = rng.integers(0, 512, (k, 6))
    for r in range(k):
        for bit in flips[r]:
            d1[r, bit // 8] ^= np.uint8(1 << (bit % 8))
    p0 = rng.uniform(0, 1280, (n0, 2))
    p1 = rng.uniform(0, 1280, (n1, 2))
    p1[:k] = p0[:k] + rng.normal(0, 8, (k, 2))
    with FeatureMatcher(64) as m:
        g0, g1 = m.match(p0, d0, p1, d1)
        kg = m.knn2(d0, d1)
    o0, o1 = O.match_features(p0, d0, p1, d1)
    assert _eq(g0, o0) and _eq(g1, o1)
    for a, b in zip(kg, O.knn2(d0, d1)):
        assert _eq(a, b)


@pytest.mark.parametrize("nbytes", [32, 61, 64, 128])
def test_descriptor_widths(nbytes):
    rng = np.random.default_rng(nbytes)
    d0 = rng.integers(0, 256, (300, nbytes), dtype=np.uint8)
    d1 = d0[rng.permutation(300)].copy()
    d1[:, 0] ^= 3
    p0 = rng.uniform(0, 1280, (300, 2))
    p1 = rng.uniform(0, 1280, (300, 2))
    with FeatureMatcher(nbytes) as m:
        kg = m.knn2(d0, d1)
        g = m.match(p0, d0, p1, d1, 0.8, 0.0, 2000.0)
    for a, b in zip(kg, O.knn2(d0, d1)):
        assert _eq(a, b)
    o = O.match_features(p0, d0, p1, d1, 0.8, 0.0, 2000.0)
    assert _eq(g[0], o[0]) and _eq(g[1], o[1])


def _frame(rng, n, base=None, motion=6.0):
    if base is None:
        pts = rng.uniform(0, 1280, (n, 2))
        desc = rng.integers(0, 256, (n, 64), dtype=np.uint8)
    else:
        bp, bd = base
        pts = np.vstack([bp[: n // 2] + rng.normal(0, motion, (n // 2, 2)), rng.uniform(0, 1280, (n - n // 2, 2))])
        desc = np.vstack([bd[: n // 2], rng.integers(0, 256, (n - n // 2, 64), dtype=np.uint8)])
        desc[: n // 2, 3] ^= 16
        perm = rng.permutation(n)
        pts, desc = pts[perm], desc[perm]
    # "distorted" positions: any other coordinates work for the test; these
    # move some pairs across the (1.5, 40) px gates
    dist = pts + rng.normal(0, 15, pts.shape)
    return pts, desc, dist


def test_index_subset_overload_on_resident_frames():
    """CTracker::matchFeatures(prevFrameIdx, currFrameIdx, ...) as called
    every frame at CSfM.cpp:518: subsets of the two resident frames,
    undistorted positions, frame-global indices out."""
    rng = np.random.default_rng(11)
    tr = sfm_amd.CTracker()
    prev = _frame(rng, 1800)
    curr = _frame(rng, 1900, base=prev[:2])
    tr.setKeyPoints(prev[0], prev[1], prev[2])
    tr.setKeyPoints(curr[0], curr[1], curr[2])
    for trial in range(4):
        pi = np.sort(rng.choice(1800, rng.integers(800, 1800), replace=False)).astype(np.int32)
        ci = rng.permutation(1900)[: rng.integers(600, 1900)].astype(np.int32)
        if trial == 3:
            pi = np.concatenate([pi, pi[:10]])      # duplicated indices: queries competing for the same rows
        g0, g1 = tr.matchFeatures(pi, ci)
        a, b = O.match_features(prev[0][pi], prev[1][pi], curr[0][ci], curr[1][ci])
        assert _eq(g0, pi[a]) and _eq(g1, ci[b]), trial
        assert len(g0) > 100
    # empty / tiny subsets
    assert len(tr.matchFeatures(np.zeros(0, np.int32), np.arange(10, dtype=np.int32))[0]) == 0
    assert len(tr.matchFeatures(np.arange(10, dtype=np.int32), np.arange(1, dtype=np.int32))[0]) == 0
    with pytest.raises(sfm_amd.SfmError):
        tr.matchFeatures(np.array([1800], np.int32), np.arange(10, dtype=np.int32))   # out of range


def test_whole_frame_member_overload_uses_distorted_positions():
    """bool CTracker::matchFeatures() (CTracker.cpp:419-477, CSfM.cpp:823):
    both resident frames, getPointsDistorted positions; the bool is
    matchCount >= _minFeatures."""
    rng = np.random.default_rng(12)
    tr = sfm_amd.CTracker()
    prev = _frame(rng, 1500)
    curr = _frame(rng, 1400, base=prev[:2])
    tr.setKeyPoints(*prev[:2], pts_distorted=prev[2])
    tr.setKeyPoints(*curr[:2], pts_distorted=curr[2])
    ok = tr.matchFeatures()
    a, b = O.match_features(prev[2], prev[1], curr[2], curr[1])
    assert _eq(tr._prevIdx, a) and _eq(tr._currIdx, b)
    assert ok == (len(a) >= 5)
    u = O.match_features(prev[0], prev[1], curr[0], curr[1])
    assert not (_eq(u[0], a) and _eq(u[1], b))      # the positions matter (distorted != undistorted)


def test_frames_swap_like_the_reference():
    rng = np.random.default_rng(13)
    frames = [_frame(rng, 600)]
    for _ in range(3):
        frames.append(_frame(rng, 600, base=frames[-1][:2]))
    with FeatureMatcher(64) as m:
        m.push_frame(frames[0][0], frames[0][1])
        for f_prev, f_curr in zip(frames, frames[1:]):
            m.push_frame(f_curr[0], f_curr[1])
            idx = np.arange(600, dtype=np.int32)
            g = m.match_subset(idx, idx)
            o = O.match_features(f_prev[0], f_prev[1], f_curr[0], f_curr[1])
            assert _eq(g[0], o[0]) and _eq(g[1], o[1])
            knn_ms, total_ms = m.last_time_ms()
            assert 0 < knn_ms <= total_ms
