"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes binding of liboracle.so (the CPU restatement of the reference path,
see ba_oracle.cpp / match_oracle.cpp headers).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
PARITY UNPINNED: no reference test or fixture pins these results.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_int, c_int32, c_int64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


class Options(ctypes.Structure):
    _fields_ = [("max_num_iterations", c_int32), ("max_num_consecutive_invalid_steps", c_int32),
                ("jacobi_scaling", c_int32), ("pad_", c_int32)] + [
        (n, c_double) for n in ("function_tolerance", "gradient_tolerance", "parameter_tolerance",
                                "initial_trust_region_radius", "max_trust_region_radius", "min_trust_region_radius",
                                "min_lm_diagonal", "max_lm_diagonal", "min_relative_decrease")]


class Summary(ctypes.Structure):
    _fields_ = [(n, c_int32) for n in ("termination_type", "num_iterations", "num_successful_steps",
                                       "num_unsuccessful_steps", "num_invalid_steps", "num_residual_evaluations",
                                       "num_jacobian_evaluations", "num_linear_solves")] + [
        (n, c_double) for n in ("initial_cost", "final_cost", "wall_time_s", "jacobian_time_s",
                                "linear_solver_time_s", "residual_time_s")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class Iteration(ctypes.Structure):
    _fields_ = [(n, c_int32) for n in ("iteration", "step_is_valid", "step_is_successful", "pad_")] + [
        (n, c_double) for n in ("cost", "cost_change", "gradient_max_norm", "step_norm", "relative_decrease",
                                "trust_region_radius")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_ if n != "pad_"}


_L = None


def lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_default_options.argtypes = [POINTER(Options)]
        L.oracle_default_options.restype = None
        L.oracle_ba_residuals_jacobians.argtypes = [c_int64] + [c_void_p] * 9
        L.oracle_ba_residuals_jacobians.restype = c_int
        L.oracle_ba_solve.argtypes = [POINTER(Options), c_int, c_int64, c_void_p, c_void_p, c_void_p, c_int32,
                                      c_void_p, c_void_p, c_void_p, c_int32, c_void_p, POINTER(Summary), c_void_p,
                                      c_int32, POINTER(c_int32)]
        L.oracle_ba_solve.restype = c_int
        L.oracle_set_threads.argtypes = [c_int]
        L.oracle_set_threads.restype = c_int
        L.oracle_set_order.argtypes = [c_int]
        L.oracle_set_order.restype = c_int
        L.oracle_knn2_hamming.argtypes = [c_void_p, c_int32, c_void_p, c_int32, c_int32] + [c_void_p] * 4
        L.oracle_knn2_hamming.restype = c_int
        L.oracle_match_features.argtypes = [c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_int32,
                                            c_double, c_double, c_double, c_void_p, c_void_p]
        L.oracle_match_features.restype = c_int
        L.oracle_ba_reduced_system.argtypes = [c_int64, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p,
                                               c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                               c_int32, c_void_p, c_void_p, c_void_p, c_void_p]
        L.oracle_ba_reduced_system.restype = c_int
        L.oracle_pyr_down.argtypes = [c_void_p, c_int32, c_int32, c_void_p]
        L.oracle_pyr_down.restype = None
        L.oracle_scharr.argtypes = [c_void_p, c_int32, c_int32, c_void_p]
        L.oracle_scharr.restype = None
        L.oracle_calc_optical_flow_pyr_lk.argtypes = [c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_int32,
                                                      c_void_p, c_void_p, c_int32, c_int32, c_int32, c_double,
                                                      c_double]
        L.oracle_calc_optical_flow_pyr_lk.restype = c_int
        L.oracle_representative_descriptors.argtypes = [c_void_p, c_void_p, c_int32, c_int32, c_void_p]
        L.oracle_representative_descriptors.restype = c_int
        L.oracle_min_eigen.argtypes = [c_void_p, c_int32, c_int32, c_void_p]
        L.oracle_min_eigen.restype = None
        L.oracle_good_features.argtypes = [c_void_p, c_int32, c_int32, c_int32, c_double, c_double, c_void_p]
        L.oracle_good_features.restype = c_int32
        L.oracle_corner_subpix.argtypes = [c_void_p, c_int32, c_int32, c_void_p, c_int32, c_int32, c_int32, c_double]
        L.oracle_corner_subpix.restype = None
        L.oracle_detect_features_of.argtypes = [c_void_p, c_int32, c_int32, c_int32, c_double, c_double, c_int32,
                                                c_int32, c_double, c_void_p]
        L.oracle_detect_features_of.restype = c_int32
        L.oracle_klt_associate.argtypes = [c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_int32, c_double,
                                           c_double, c_double, c_void_p, c_void_p]
        L.oracle_klt_associate.restype = c_int32
        _L = L
    return _L


def _p(a):
    return None if a is None else a.ctypes.data_as(c_void_p)


def default_options(**kw) -> Options:
    o = Options()
    lib().oracle_default_options(ctypes.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def residuals_jacobians(uv, cam_idx, pt_idx, K9, rot, t, X, jacobian=True):
    uv = np.ascontiguousarray(uv, np.float64)
    cam_idx = np.ascontiguousarray(cam_idx, np.int32)
    pt_idx = np.ascontiguousarray(pt_idx, np.int32)
    K9 = np.ascontiguousarray(K9, np.float64).reshape(-1, 9)
    rot, t, X = (np.ascontiguousarray(a, np.float64) for a in (rot, t, X))
    n = uv.shape[0]
    res = np.zeros((n, 2))
    jac = np.zeros((n, 2, 9)) if jacobian else None
    rc = lib().oracle_ba_residuals_jacobians(n, _p(uv), _p(cam_idx), _p(pt_idx), _p(K9), _p(rot), _p(t), _p(X),
                                             _p(res), _p(jac))
    assert rc == 0
    return res, jac


def solve(uv, cam_idx, pt_idx, K9, rot, t, X, mode=2, options: Options | None = None, trace_cap=128, threads=1,
          order=0):
    """rot, t, X are updated in place (float64, C-contiguous).  threads > 1
    runs the oracle's OpenMP loops (bitwise the 1-thread result).  order=1
    sums the reduced matrix's diagonal blocks in the device solver's
    association instead of Ceres' (oracle_set_order; tests only)."""
    uv = np.ascontiguousarray(uv, np.float64)
    cam_idx = np.ascontiguousarray(cam_idx, np.int32)
    pt_idx = np.ascontiguousarray(pt_idx, np.int32)
    K9 = np.ascontiguousarray(K9, np.float64).reshape(-1, 9)
    o = options if options is not None else default_options()
    sm = Summary()
    tr = (Iteration * trace_cap)()
    tl = c_int32(0)
    prev = lib().oracle_set_threads(int(threads))
    prev_order = lib().oracle_set_order(int(order))
    try:
        rc = lib().oracle_ba_solve(ctypes.byref(o), mode, uv.shape[0], _p(uv), _p(cam_idx), _p(pt_idx), rot.shape[0],
                                   _p(K9), _p(rot), _p(t), X.shape[0], _p(X), ctypes.byref(sm), tr, trace_cap,
                                   ctypes.byref(tl))
    finally:
        lib().oracle_set_threads(prev)
        lib().oracle_set_order(prev_order)
    if rc != 0:
        raise RuntimeError(f"oracle_ba_solve returned {rc}")
    return sm.as_dict(), [tr[i].as_dict() for i in range(tl.value)]


def knn2(desc0, desc1):
    desc0 = np.ascontiguousarray(desc0, np.uint8)
    desc1 = np.ascontiguousarray(desc1, np.uint8)
    n0, n1 = desc0.shape[0], desc1.shape[0]
    out = [np.zeros(n0, np.int32) for _ in range(4)]
    lib().oracle_knn2_hamming(_p(desc0), n0, _p(desc1), n1, desc0.shape[1], *map(_p, out))
    return tuple(out)


def match_features(pts0, desc0, pts1, desc1, ratio=0.8, min_distance=1.5, max_distance=40.0):
    pts0 = np.ascontiguousarray(pts0, np.float64).reshape(-1, 2)
    pts1 = np.ascontiguousarray(pts1, np.float64).reshape(-1, 2)
    desc0 = np.ascontiguousarray(desc0, np.uint8)
    desc1 = np.ascontiguousarray(desc1, np.uint8)
    n0, n1 = pts0.shape[0], pts1.shape[0]
    nb = desc0.shape[1] if n0 else 64
    cap = max(1, min(n0, n1))
    i0 = np.zeros(cap, np.int32)
    i1 = np.zeros(cap, np.int32)
    m = lib().oracle_match_features(_p(pts0), _p(desc0), n0, _p(pts1), _p(desc1), n1, nb, ratio, min_distance,
                                    max_distance, _p(i0), _p(i1))
    return i0[:m].copy(), i1[:m].copy()


def reduced_system(uv, cam_idx, pt_idx, K9, rot, t, X, scale_c, scale_p, D_c, D_p, add_cam_diag=True):
    """DENSE_SCHUR reduced camera system (S [6C][6C], rhs [6C]) plus unscaled
    squared column norms, for the sharding-decomposition tests."""
    uv = np.ascontiguousarray(uv, np.float64)
    cam_idx = np.ascontiguousarray(cam_idx, np.int32)
    pt_idx = np.ascontiguousarray(pt_idx, np.int32)
    K9 = np.ascontiguousarray(K9, np.float64).reshape(-1, 9)
    arrs = [np.ascontiguousarray(a, np.float64) for a in (rot, t, X, scale_c, scale_p, D_c, D_p)]
    C, P = arrs[0].shape[0], arrs[2].shape[0]
    S = np.zeros((6 * C, 6 * C))
    rhs = np.zeros(6 * C)
    cc = np.zeros((C, 6))
    cp = np.zeros((P, 3))
    rc = lib().oracle_ba_reduced_system(uv.shape[0], _p(uv), _p(cam_idx), _p(pt_idx), C, _p(K9), _p(arrs[0]),
                                        _p(arrs[1]), P, _p(arrs[2]), _p(arrs[3]), _p(arrs[4]), _p(arrs[5]),
                                        _p(arrs[6]), 1 if add_cam_diag else 0, _p(S), _p(rhs), _p(cc), _p(cp))
    if rc != 0:
        raise RuntimeError("oracle_ba_reduced_system failed")
    return S, rhs, cc, cp


# ---- optical-flow tracker (klt_oracle.cpp) --------------------------------
def pyr_down(img):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.zeros(((h + 1) // 2, (w + 1) // 2), np.uint8)
    lib().oracle_pyr_down(_p(img), w, h, _p(out))
    return out


def scharr(img):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.zeros((h, w, 2), np.int16)
    lib().oracle_scharr(_p(img), w, h, _p(out))
    return out


def calc_optical_flow_pyr_lk(prev, nxt, prev_pts, win=21, max_level=3, max_count=20, eps=0.03, min_eig=1e-3):
    """cv::calcOpticalFlowPyrLK restatement (CTracker.cpp:513 call)."""
    prev = np.ascontiguousarray(prev, np.uint8)
    nxt = np.ascontiguousarray(nxt, np.uint8)
    pts = np.ascontiguousarray(prev_pts, np.float32).reshape(-1, 2)
    h, w = prev.shape
    n = pts.shape[0]
    out = np.zeros((n, 2), np.float32)
    st = np.zeros(n, np.uint8)
    rc = lib().oracle_calc_optical_flow_pyr_lk(_p(prev), _p(nxt), w, h, _p(pts), n, _p(out), _p(st), win, max_level,
                                               max_count, eps, min_eig)
    if rc:
        raise ValueError(f"oracle_calc_optical_flow_pyr_lk: {rc}")
    return out, st


def klt_associate(prev_pts, flowed, status, curr_pts, max_match_distance=40.0, min_match_distance=1.5,
                  max_org_feat_dist=1.0):
    """CTracker::computeOpticalFlow association + gates (CTracker.cpp:515-545)."""
    prev_pts = np.ascontiguousarray(prev_pts, np.float32).reshape(-1, 2)
    flowed = np.ascontiguousarray(flowed, np.float32).reshape(-1, 2)
    status = np.ascontiguousarray(status, np.uint8)
    curr = np.ascontiguousarray(curr_pts, np.float64).reshape(-1, 2)
    n, m = prev_pts.shape[0], curr.shape[0]
    pi = np.zeros(max(1, n), np.int32)
    ci = np.zeros(max(1, n), np.int32)
    k = lib().oracle_klt_associate(_p(prev_pts), _p(flowed), _p(status), n, _p(curr), m, max_match_distance,
                                   min_match_distance, max_org_feat_dist, _p(pi), _p(ci))
    return pi[:k].copy(), ci[:k].copy()


def min_eigen(img):
    """cornerMinEigenVal(blockSize 3, ksize 3) restatement (gftt_oracle.cpp)."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.zeros((h, w), np.float32)
    lib().oracle_min_eigen(_p(img), w, h, _p(out))
    return out


def good_features(img, max_corners=500, quality=0.05, min_distance=10.0):
    """goodFeaturesToTrack restatement (CTracker.cpp:262 call): integer corners."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.zeros((max(1, max_corners), 2), np.float32)
    n = lib().oracle_good_features(_p(img), w, h, max_corners, quality, min_distance, _p(out))
    return out[:n].copy()


def corner_subpix(img, pts, win=5, max_iter=20, eps=0.03):
    """cornerSubPix restatement (CTracker.cpp:265 call)."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    p = np.ascontiguousarray(pts, np.float32).reshape(-1, 2).copy()
    lib().oracle_corner_subpix(_p(img), w, h, _p(p), p.shape[0], win, max_iter, eps)
    return p


def detect_features_of(img, max_corners=500, quality=0.05, min_distance=10.0, win=5, max_iter=20, eps=0.03):
    """CTracker::detectFeaturesOpticalFlow (CTracker.cpp:252-272) minus setPoints."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.zeros((max(1, max_corners), 2), np.float32)
    n = lib().oracle_detect_features_of(_p(img), w, h, max_corners, quality, min_distance, win, max_iter, eps,
                                        _p(out))
    return out[:n].copy()


def representative_descriptors(desc, row_off):
    """CMap::getRepresentativeDescriptors restatement -> best row per point."""
    desc = np.ascontiguousarray(desc, np.uint8)
    row_off = np.ascontiguousarray(row_off, np.int32)
    n = row_off.shape[0] - 1
    best = np.zeros(max(1, n), np.int32)
    rc = lib().oracle_representative_descriptors(_p(desc), _p(row_off), n, desc.shape[1], _p(best))
    if rc:
        raise ValueError("a point has no descriptor rows")
    return best[:n].copy()
