"""Frame-resident descriptor matcher (sfm_matcher_* of include/sfm_amd.h).

The device side of CTracker's four matchFeatures overloads
(/root/reference/CTracker.cpp:114-149, 211-250, 368-417, 419-477): the last
two frames' keypoints and descriptors stay resident in HBM (one upload per
frame, the _prevFrame = _currFrame swap of CSfM.cpp:626-629); every call
runs on the device with pooled buffers.  No CPU fallback.
"""
from __future__ import annotations

import ctypes
from ctypes import c_double, c_int32, c_void_p

import numpy as np

from ._ffi import check, lib, ptr

RATIO_TEST = 0.8            # CTracker.cpp:27
MAX_MATCH_DISTANCE = 40.0   # CTracker.cpp:30
MIN_MATCH_DISTANCE = 1.5    # CTracker.cpp:31


def _pts(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64).reshape(-1, 2)


def _desc(a, nbytes: int) -> np.ndarray:
    d = np.ascontiguousarray(a, dtype=np.uint8)
    if d.size == 0:
        return d.reshape(0, nbytes)
    if d.ndim != 2 or d.shape[1] != nbytes:
        raise ValueError(f"descriptors must be (n, {nbytes}) uint8, got {d.shape}")
    return d


class FeatureMatcher:
    def __init__(self, desc_bytes: int = 64, device: int = 0):
        h = c_void_p()
        check(lib().sfm_matcher_create(device, desc_bytes, ctypes.byref(h)), "sfm_matcher_create")
        self._h = h
        self.desc_bytes = desc_bytes
        self.n = [0, 0]   # keypoints of [previous, current] frame

    def close(self) -> None:
        if self._h:
            lib().sfm_matcher_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def push_frame(self, pts, desc, pts_distorted=None) -> None:
        """New current frame: undistorted keypoints (CFrame::_pts), their
        descriptors and (optionally) the distorted positions."""
        p = _pts(pts)
        d = _desc(desc, self.desc_bytes)
        if d.shape[0] != p.shape[0]:
            raise ValueError("one descriptor row per keypoint")
        pd = None if pts_distorted is None else _pts(pts_distorted)
        if pd is not None and pd.shape != p.shape:
            raise ValueError("pts_distorted must match pts")
        check(lib().sfm_matcher_push_frame(self._h, ptr(p), ptr(pd), ptr(d), p.shape[0]), "sfm_matcher_push_frame")
        self.n = [self.n[1], p.shape[0]]

    def match_subset(self, prev_idx, curr_idx, ratio=RATIO_TEST, min_distance=MIN_MATCH_DISTANCE,
                     max_distance=MAX_MATCH_DISTANCE):
        """CTracker::matchFeatures(prevFrameIdx, currFrameIdx, ...) -> frame-global (prev, curr) indices."""
        a = np.ascontiguousarray(prev_idx, dtype=np.int32)
        b = np.ascontiguousarray(curr_idx, dtype=np.int32)
        cap = max(1, min(a.size, b.size))
        o0, o1, nm = np.zeros(cap, np.int32), np.zeros(cap, np.int32), c_int32(0)
        check(lib().sfm_matcher_match_subset(self._h, ptr(a), a.size, ptr(b), b.size, ratio, min_distance,
                                             max_distance, ptr(o0), ptr(o1), ctypes.byref(nm)),
              "sfm_matcher_match_subset")
        return o0[:nm.value].copy(), o1[:nm.value].copy()

    def store_keyframe(self, slot: int, pts, desc) -> None:
        """Keyframe slot `slot` resident on the device (pts [n][2], desc)."""
        p = _pts(pts)
        d = _desc(desc, self.desc_bytes)
        if d.shape[0] != p.shape[0]:
            raise ValueError("one descriptor row per keypoint")
        check(lib().sfm_matcher_store_keyframe(self._h, int(slot), ptr(p), ptr(d), p.shape[0]),
              "sfm_matcher_store_keyframe")

    def match_keyframes(self, q_slot: int, q_idx, t_slot: int, t_idx, q_pts=None, ratio=RATIO_TEST,
                        min_distance=MIN_MATCH_DISTANCE, max_distance=MAX_MATCH_DISTANCE):
        """match(pts0, desc0, pts1, desc1) on stored keyframe rows: query rows
        q_idx of q_slot (positions q_pts if given), train rows t_idx of
        t_slot -> subset-local (query, train) indices."""
        a = np.ascontiguousarray(np.asarray(q_idx).reshape(-1), dtype=np.int32)
        b = np.ascontiguousarray(np.asarray(t_idx).reshape(-1), dtype=np.int32)
        qp = None if q_pts is None else _pts(q_pts)
        if qp is not None and qp.shape[0] != a.size:
            raise ValueError("one query position per query row")
        cap = max(1, min(a.size, b.size))
        o0, o1, nm = np.zeros(cap, np.int32), np.zeros(cap, np.int32), c_int32(0)
        check(lib().sfm_matcher_match_keyframes(self._h, int(q_slot), ptr(a), a.size, ptr(qp), int(t_slot), ptr(b),
                                                b.size, ratio, min_distance, max_distance, ptr(o0), ptr(o1),
                                                ctypes.byref(nm)), "sfm_matcher_match_keyframes")
        return o0[:nm.value].copy(), o1[:nm.value].copy()

    def track_pnp(self, device_map, prev_pt3d, K, min_matches: int, iterations: int = 20, reproj_err: float = 7.0,
                  confidence: float = 0.99, ratio=RATIO_TEST, min_distance=MIN_MATCH_DISTANCE,
                  max_distance=MAX_MATCH_DISTANCE):
        """CSfM::tracking's pose step as one device call (sfm_track_pnp):
        matchFeatures(prevIdx, currIdx) of the previous frame's keypoints with
        a map point (prev_pt3d >= 0) against the whole current frame, then
        cv::solvePnPRansac on their map points.  -> (n_matches, found, rvec,
        tvec, inlier keypoints, their map points); no PnP below min_matches."""
        p3 = np.ascontiguousarray(np.asarray(prev_pt3d).reshape(-1), dtype=np.int32)
        K9 = np.ascontiguousarray(np.asarray(K, np.float64).reshape(9))
        cap = max(1, int((p3 >= 0).sum()))
        kp, pt = np.zeros(cap, np.int32), np.zeros(cap, np.int32)
        rvec, tvec = np.zeros(3), np.zeros(3)
        found, nm, ni = c_int32(0), c_int32(0), c_int32(0)
        check(lib().sfm_track_pnp(self._h, device_map._h, len(p3), ptr(p3), ratio, min_distance, max_distance,
                                  int(min_matches), ptr(K9), int(iterations), float(reproj_err), float(confidence),
                                  ptr(rvec), ptr(tvec), ctypes.byref(found), ctypes.byref(nm), cap, ptr(kp), ptr(pt),
                                  ctypes.byref(ni)), "sfm_track_pnp")
        return nm.value, bool(found.value), rvec, tvec, kp[:ni.value].copy(), pt[:ni.value].copy()

    def match_frames(self, distorted: bool = True, ratio=RATIO_TEST, min_distance=MIN_MATCH_DISTANCE,
                     max_distance=MAX_MATCH_DISTANCE):
        """bool CTracker::matchFeatures(): the whole frames (distorted positions) -> (_prevIdx, _currIdx)."""
        cap = max(1, min(self.n))
        o0, o1, nm = np.zeros(cap, np.int32), np.zeros(cap, np.int32), c_int32(0)
        check(lib().sfm_matcher_match_frames(self._h, 1 if distorted else 0, ratio, min_distance, max_distance,
                                             ptr(o0), ptr(o1), ctypes.byref(nm)), "sfm_matcher_match_frames")
        return o0[:nm.value].copy(), o1[:nm.value].copy()

    def match(self, pts0, desc0, pts1, desc1, ratio=RATIO_TEST, min_distance=MIN_MATCH_DISTANCE,
              max_distance=MAX_MATCH_DISTANCE):
        """The (pts0, desc0, pts1, desc1[, min, max]) overloads on host arrays."""
        p0, p1 = _pts(pts0), _pts(pts1)
        d0, d1 = _desc(desc0, self.desc_bytes), _desc(desc1, self.desc_bytes)
        if d0.shape[0] != p0.shape[0] or d1.shape[0] != p1.shape[0]:
            raise ValueError("one descriptor row per point")
        cap = max(1, min(p0.shape[0], p1.shape[0]))
        o0, o1, nm = np.zeros(cap, np.int32), np.zeros(cap, np.int32), c_int32(0)
        check(lib().sfm_matcher_match(self._h, ptr(p0), ptr(d0), p0.shape[0], ptr(p1), ptr(d1), p1.shape[0], ratio,
                                      min_distance, max_distance, ptr(o0), ptr(o1), ctypes.byref(nm)),
              "sfm_matcher_match")
        return o0[:nm.value].copy(), o1[:nm.value].copy()

    def knn2(self, desc0, desc1):
        d0, d1 = _desc(desc0, self.desc_bytes), _desc(desc1, self.desc_bytes)
        n0 = d0.shape[0]
        out = [np.zeros(n0, np.int32) for _ in range(4)]
        check(lib().sfm_matcher_knn2(self._h, ptr(d0), n0, ptr(d1), d1.shape[0], *map(ptr, out)),
              "sfm_matcher_knn2")
        return tuple(out)

    def last_time_ms(self):
        """(2-NN search, whole call) device time of the last match (HIP events)."""
        buf = np.zeros(2)
        check(lib().sfm_matcher_last_time(self._h, ptr(buf)), "sfm_matcher_last_time")
        return float(buf[0]), float(buf[1])
