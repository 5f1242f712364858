"""GPU: the C++ drop-in (include/sfm_ctracker_compat.hpp) called the way the
reference's pipeline calls CTracker, through tests/compat/compat_gpu.cpp
(prebuilt by __graft_entry__.build() into tests/compat/bin/), against the
oracle:

  * CSfM::bundleAdjustment (CSfM.cpp:310-348): C1 gathered keyframe by
    keyframe in a shuffled per-frame (hash-bucket-like) order with one
    aliased double* per observation into the map storage; the solution is
    scattered back through those pointers (parameters 1e-6 relative, cost
    1e-9, same iteration count);
  * detectFeaturesOpticalFlow + computeOpticalFlow on two synthetic frames
    (bit-exact corners and index lists);
  * the frame-resident matcher drop-ins: matchFeatures(prevIdx, currIdx, ...)
    (CSfM.cpp:518), matchFeatures() (CSfM.cpp:823), the (0, 7) window
    (CSfM.cpp:673) and the one-shot member-window overload (bit-exact).
"""
import os
import subprocess

import numpy as np
import pytest

from oracle import ffi as O
from sfm_amd import scene
from sfm_amd.video import SyntheticVideo

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "compat", "bin", "compat_gpu")


def _run(mode, d):
    assert os.path.exists(EXE), f"{EXE} missing: __graft_entry__.build() compiles it"
    out = subprocess.run([EXE, mode, str(d)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert f"compat_gpu {mode} ok" in out.stdout


def _w(d, name, a):
    np.ascontiguousarray(a).tofile(os.path.join(d, name))


def _r(d, name, dtype):
    return np.fromfile(os.path.join(d, name), dtype=dtype)


def test_bundle_adjustment_drop_in_as_csfm_calls_it(tmp_path):
    s = scene.config("C1")
    C, P = s.n_cams, s.n_pts
    rng = np.random.default_rng(17)
    # each keyframe's 2-D points in a shuffled order; its map-point views in
    # another shuffled order (the multimap's bucket order is unspecified)
    kf_pts, kf_npts, view_off, view_pt, view_2d, obs_order = [], [], [0], [], [], []
    for c in range(C):
        obs = np.flatnonzero(s.cam_idx == c)
        obs = obs[rng.permutation(len(obs))]                    # 2-D point j of keyframe c = obs[j]
        kf_pts.append(s.uv[obs])
        kf_npts.append(len(obs))
        views = rng.permutation(len(obs))                       # getPointsInFrame_Mutable order
        view_pt.extend(s.pt_idx[obs[views]])
        view_2d.extend(views)
        obs_order.extend(obs[views])
        view_off.append(len(view_pt))
    _w(tmp_path, "meta.i32", np.array([C, P], np.int32))
    _w(tmp_path, "kf_K.f64", s.K.reshape(C, 9))
    _w(tmp_path, "kf_rot.f64", s.rot)
    _w(tmp_path, "kf_t.f64", s.t)
    _w(tmp_path, "kf_pts.f64", np.concatenate(kf_pts))
    _w(tmp_path, "kf_npts.i32", np.array(kf_npts, np.int32))
    _w(tmp_path, "view_off.i32", np.array(view_off, np.int32))
    _w(tmp_path, "view_pt.i32", np.array(view_pt, np.int32))
    _w(tmp_path, "view_2d.i32", np.array(view_2d, np.int32))
    _w(tmp_path, "map.f64", s.X)
    _run("ba", tmp_path)
    o = np.array(obs_order)
    r, t, X = s.copy_params()
    sm, _ = O.solve(s.uv[o], s.cam_idx[o], s.pt_idx[o], s.K, r, t, X)
    gr, gt, gX = (_r(tmp_path, f"out_{k}.f64", np.float64).reshape(-1, 3) for k in ("rot", "t", "X"))
    term, iters, c0, c1 = _r(tmp_path, "out_summary.f64", np.float64)
    assert int(term) == sm["termination_type"] and int(iters) == sm["num_iterations"]
    assert abs(c1 - sm["final_cost"]) <= 1e-9 * sm["final_cost"]
    for a, b in ((gr, r), (gt, t), (gX, X)):
        assert np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-3)) < 1e-6
    assert not np.array_equal(gX, s.X)                          # written back through the pointers


def test_optical_flow_drop_ins(tmp_path):
    v = SyntheticVideo()
    f0, f1 = v.frame(0), v.frame(1)
    _w(tmp_path, "meta.i32", np.array([v.w, v.h], np.int32))
    _w(tmp_path, "prev.u8", f0)
    _w(tmp_path, "curr.u8", f1)
    _run("flow", tmp_path)
    c0 = _r(tmp_path, "out_c0.f32", np.float32).reshape(-1, 2)
    c1 = _r(tmp_path, "out_c1.f32", np.float32).reshape(-1, 2)
    assert np.array_equal(c0, O.detect_features_of(f0))
    assert np.array_equal(c1, O.detect_features_of(f1))
    fl, st = O.calc_optical_flow_pyr_lk(f0, f1, c0.astype(np.float64))
    opi, oci = O.klt_associate(c0, fl, st, c1.astype(np.float64))
    assert np.array_equal(_r(tmp_path, "out_pi.i32", np.int32), opi)
    assert np.array_equal(_r(tmp_path, "out_ci.i32", np.int32), oci)
    assert _r(tmp_path, "out_ok.i32", np.int32)[0] == int(len(opi) >= 5)
    assert len(opi) > 100


def test_matcher_drop_ins(tmp_path):
    rng = np.random.default_rng(21)
    n0, n1, nb = 1500, 1600, 64
    p0 = rng.uniform(0, 1280, (n0, 2))
    d0 = rng.integers(0, 256, (n0, nb), dtype=np.uint8)
    k = 900
    src = rng.permutation(n0)[:k]
    p1 = rng.uniform(0, 1280, (n1, 2))
    d1 = rng.integers(0, 256, (n1, nb), dtype=np.uint8)
    dst = rng.permutation(n1)[:k]
    p1[dst] = p0[src] + rng.normal(0, 4, (k, 2))
    d1[dst] = d0[src]
    d1[dst, 5] ^= 8
    q0 = p0 * 1.0003 - 0.2                                   # distorted positions differ
    q1 = p1 * 1.0003 - 0.2
    s0 = np.sort(rng.permutation(n0)[:1200]).astype(np.int32)
    s1 = rng.permutation(n1)[:1300].astype(np.int32)
    _w(tmp_path, "meta.i32", np.array([n0, n1, nb], np.int32))
    for name, a in (("f0_pts.f64", p0), ("f0_dist.f64", q0), ("f1_pts.f64", p1), ("f1_dist.f64", q1),
                    ("f0_desc.u8", d0), ("f1_desc.u8", d1), ("sub0.i32", s0), ("sub1.i32", s1)):
        _w(tmp_path, name, a)
    _run("match", tmp_path)
    ri = lambda nm: _r(tmp_path, nm, np.int32)
    a, b = O.match_features(p0[s0], d0[s0], p1[s1], d1[s1])
    assert np.array_equal(ri("out_sub_a.i32"), s0[a]) and np.array_equal(ri("out_sub_b.i32"), s1[b])
    a, b = O.match_features(q0, d0, q1, d1)
    assert np.array_equal(ri("out_all_a.i32"), a) and np.array_equal(ri("out_all_b.i32"), b)
    assert ri("out_ok.i32")[0] == int(len(a) >= 5)
    a, b = O.match_features(p0, d0, p1, d1, 0.8, 0.0, 7.0)
    assert np.array_equal(ri("out_w7_a.i32"), a) and np.array_equal(ri("out_w7_b.i32"), b)
    a, b = O.match_features(p0, d0, p1, d1)
    assert np.array_equal(ri("out_free_a.i32"), a) and np.array_equal(ri("out_free_b.i32"), b)
    assert len(a) > 300
