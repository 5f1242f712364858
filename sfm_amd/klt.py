"""Pyramidal Lucas-Kanade tracker on the device.

Host-side mirror of CTracker::computeOpticalFlow
(/root/reference/CTracker.cpp:480-562) and of the OpenCV call it makes,
cv::calcOpticalFlowPyrLK (CTracker.cpp:513), over the C ABI
(sfm_klt_* in include/sfm_amd.h).  Frames are pushed once; their pyramids
and Scharr derivatives stay resident in HBM, so each frame is uploaded and
pre-processed exactly once (as the previous frame of the next call it is
reused, like CTracker's _prevFrame/_currFrame swap, CSfM.cpp:626-629).
No CPU fallback: every call goes through libsfm_amd.so.
"""
from __future__ import annotations

import ctypes
from ctypes import c_int32, c_void_p

import numpy as np

from ._ffi import GFTTParams, KLTParams, check, default_gftt_params, default_klt_params, lib, ptr


def make_params(**kw) -> KLTParams:
    p = default_klt_params()
    for k, v in kw.items():
        if not hasattr(p, k):
            raise AttributeError(f"KLTParams has no field {k!r}")
        setattr(p, k, v)
    return p


def make_gftt_params(**kw) -> GFTTParams:
    p = default_gftt_params()
    for k, v in kw.items():
        if not hasattr(p, k):
            raise AttributeError(f"GFTTParams has no field {k!r}")
        setattr(p, k, v)
    return p


class KLTTracker:
    """Device-resident two-frame LK tracker for one frame size."""

    def __init__(self, width: int, height: int, device: int = 0, params: KLTParams | None = None, **kw):
        self.width, self.height, self.device = int(width), int(height), device
        self.params = params if params is not None else make_params(**kw)
        h = c_void_p()
        check(lib().sfm_klt_create(device, self.width, self.height, ctypes.byref(self.params), ctypes.byref(h)),
              "sfm_klt_create")
        self._h = h

    @property
    def num_levels(self) -> int:
        return int(lib().sfm_klt_num_levels(self._h))

    def push_frame(self, grey: np.ndarray) -> None:
        g = np.ascontiguousarray(grey, dtype=np.uint8)
        if g.shape != (self.height, self.width):
            raise ValueError(f"frame shape {g.shape} != {(self.height, self.width)}")
        check(lib().sfm_klt_push_frame(self._h, ptr(g), self.width), "sfm_klt_push_frame")

    def level(self, which: int, level: int):
        """(image u8 [h][w], derivatives int16 [h][w][2]) of a pyramid level of
        the previous (which=0) or current (which=1) frame."""
        w, h = c_int32(0), c_int32(0)
        check(lib().sfm_klt_get_level(self._h, which, level, None, None, ctypes.byref(w), ctypes.byref(h)),
              "sfm_klt_get_level")
        img = np.zeros((h.value, w.value), np.uint8)
        dxy = np.zeros((h.value, w.value, 2), np.int16)
        check(lib().sfm_klt_get_level(self._h, which, level, ptr(img), ptr(dxy), None, None), "sfm_klt_get_level")
        return img, dxy

    def calc_flow(self, prev_pts):
        """cv::calcOpticalFlowPyrLK(prev, curr, prev_pts) -> (next_pts float32 [n][2], status uint8 [n])."""
        pts = np.ascontiguousarray(prev_pts, dtype=np.float32).reshape(-1, 2)
        n = pts.shape[0]
        nxt = np.zeros((n, 2), np.float32)
        st = np.zeros(n, np.uint8)
        check(lib().sfm_klt_calc_flow(self._h, ptr(pts), n, ptr(nxt), ptr(st)), "sfm_klt_calc_flow")
        return nxt, st

    def compute_optical_flow(self, prev_pts_dist, curr_pts_dist, with_flow: bool = False):
        """CTracker::computeOpticalFlow body (CTracker.cpp:480-562): returns
        (prevIdx, currIdx) int32 arrays in the reference's slot order, plus
        (flowed, status) when with_flow."""
        prev = np.ascontiguousarray(prev_pts_dist, dtype=np.float64).reshape(-1, 2)
        curr = np.ascontiguousarray(curr_pts_dist, dtype=np.float64).reshape(-1, 2)
        n, m = prev.shape[0], curr.shape[0]
        pi = np.zeros(max(1, n), np.int32)
        ci = np.zeros(max(1, n), np.int32)
        nm = c_int32(0)
        flowed = np.zeros((max(1, n), 2), np.float32) if with_flow else None
        st = np.zeros(max(1, n), np.uint8) if with_flow else None
        check(lib().sfm_klt_compute_optical_flow(self._h, ptr(prev), n, ptr(curr), m, ptr(pi), ptr(ci),
                                                 ctypes.byref(nm), ptr(flowed), ptr(st)),
              "sfm_klt_compute_optical_flow")
        k = nm.value
        out = (pi[:k].copy(), ci[:k].copy())
        if with_flow:
            out = out + (flowed[:n].copy(), st[:n].copy())
        return out

    def detect_features(self, params: GFTTParams | None = None, **kw) -> np.ndarray:
        """CTracker::detectFeaturesOpticalFlow (CTracker.cpp:252-272) on the
        current frame: goodFeaturesToTrack(500, 0.05, 10) + cornerSubPix(5x5,
        20, 0.03) -> corners float32 [n][2] in response order (row T7)."""
        p = params if params is not None else make_gftt_params(**kw)
        cap = max(1, int(p.max_corners))
        out = np.zeros((cap, 2), np.float32)
        n = c_int32(0)
        check(lib().sfm_klt_detect_features(self._h, ctypes.byref(p), ptr(out), cap, ctypes.byref(n)),
              "sfm_klt_detect_features")
        return out[:n.value].copy()

    def detect_time_ms(self) -> float:
        ms = ctypes.c_double(0.0)
        check(lib().sfm_klt_detect_time(self._h, ctypes.byref(ms)), "sfm_klt_detect_time")
        return ms.value

    def phase_times(self) -> dict:
        ms = np.zeros(3)
        check(lib().sfm_klt_phase_times(self._h, ptr(ms)), "sfm_klt_phase_times")
        return {"pyramid": float(ms[0]), "lk": float(ms[1]), "associate": float(ms[2])}

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().sfm_klt_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def calc_optical_flow_pyr_lk(prev, nxt, prev_pts, device: int = 0, **kw):
    """One-shot cv::calcOpticalFlowPyrLK on two host frames."""
    prev = np.ascontiguousarray(prev, np.uint8)
    nxt = np.ascontiguousarray(nxt, np.uint8)
    pts = np.ascontiguousarray(prev_pts, np.float32).reshape(-1, 2)
    h, w = prev.shape
    n = pts.shape[0]
    out = np.zeros((n, 2), np.float32)
    st = np.zeros(n, np.uint8)
    p = make_params(**kw)
    check(lib().sfm_calc_optical_flow_pyr_lk(device, ptr(prev), ptr(nxt), w, h, ptr(pts), n, ptr(out), ptr(st),
                                             ctypes.byref(p)), "sfm_calc_optical_flow_pyr_lk")
    return out, st


def good_features_to_track(grey, device: int = 0, **kw) -> np.ndarray:
    """One-shot goodFeaturesToTrack + cornerSubPix (the row-T7 pair) on a host frame."""
    g = np.ascontiguousarray(grey, np.uint8)
    h, w = g.shape
    p = make_gftt_params(**kw)
    cap = max(1, int(p.max_corners))
    out = np.zeros((cap, 2), np.float32)
    n = c_int32(0)
    check(lib().sfm_good_features_to_track(device, ptr(g), w, h, w, ctypes.byref(p), ptr(out), cap, ctypes.byref(n)),
          "sfm_good_features_to_track")
    return out[:n.value].copy()
