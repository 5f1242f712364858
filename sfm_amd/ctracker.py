"""Host-side mirror of the reference's CTracker call surface for the hot path.

Mirrors /root/reference/CTracker.h:44-67 (same names, argument meaning and
behaviour) over the C ABI; OpenCV types are replaced by their memory layout
(Point2d -> float64 [n][2], Matx33d -> float64 [9] row-major, Mat of BRISK
descriptors -> uint8 [n][64]).

  bundleAdjustmentStructAndPose  CTracker.h:65,  CTracker.cpp:670-702
  matchFeatures (all overloads)  CTracker.h:53-58, CTracker.cpp:114-149,
                                 211-250, 368-417, 419-477 (frame-resident
                                 device matcher, sfm_amd/matcher.py)
  computeOpticalFlow             CTracker.h:60,  CTracker.cpp:480-562
  detectFeaturesOpticalFlow      CTracker.h:48,  CTracker.cpp:252-272

The reference passes parameter blocks as vector<double*> with one pointer
per observation (duplicates across observations, identity by address,
CSfM.cpp:321-340).  Python has no raw pointers; the mirror takes the
deduplicated form (`pts3d` [P][3] + per-observation `pt_idx`) and writes
results back in place, exactly as Ceres writes through the pointers.
"""
from __future__ import annotations

import ctypes
from ctypes import c_int32

import numpy as np

from . import ba as _ba
from ._ffi import check, lib, ptr

STRUCT_ONLY, POSE_ONLY, STRUCT_AND_POSE = _ba.STRUCT_ONLY, _ba.POSE_ONLY, _ba.STRUCT_AND_POSE


class CTracker:
    """Hot-path subset of CTracker (constructor constants: CTracker.cpp:25-49)."""

    def __init__(self, device: int = 0):
        self.device = device
        self._ratioTest = 0.8             # CTracker.cpp:27
        self._maxMatchDistance = 40.0     # CTracker.cpp:30
        self._minMatchDistance = 1.5      # CTracker.cpp:31
        self._minFeatures = 5             # CTracker.cpp:32
        self._maxOrgFeatDist = 1.0        # CTracker.cpp:33
        self.last_summary = None
        self.last_trace = None
        self._klt = None
        self._prevIdx = np.zeros(0, np.int32)
        self._currIdx = np.zeros(0, np.int32)
        self._matcher = None

    # ---- bundle adjustment (CTracker.cpp:670-702) --------------------------
    def bundleAdjustmentStructAndPose(self, observations, camIdx, K, R, t, pts3D, isStructOrPose, pt_idx=None,
                                      options=None):
        """observations [N][2]; camIdx [N]; K [C][9] (or [C][3][3]); R, t [C][3]
        (updated in place); pts3D [P][3] (updated in place) with pt_idx [N], or
        pts3D [N][3] one row per observation when pt_idx is None (then rows
        that are equal objects are NOT merged — pass pt_idx for shared points).
        Returns the Ceres-style summary the reference discards."""
        K9 = np.ascontiguousarray(np.asarray(K, dtype=np.float64).reshape(-1, 9))
        if pt_idx is None:
            pt_idx = np.arange(len(observations), dtype=np.int32)
        sm, tr = _ba.solve(observations, camIdx, pt_idx, K9, R, t, pts3D, options=options, mode=isStructOrPose)
        self.last_summary, self.last_trace = sm, tr
        return sm

    # ---- matching --------------------------------------------------------
    def _resident(self):
        """The frame-resident matcher (created by setKeyPoints); the
        resident-frame overloads use its own descriptor width."""
        if self._matcher is None:
            raise RuntimeError("matchFeatures: setKeyPoints() the previous and current frames first")
        return self._matcher

    def _m(self, nbytes: int):
        """A matcher of descriptor width `nbytes` for explicit-data calls: the
        resident one when the width agrees, else a separate one, so a call
        with another width never discards the resident frames."""
        from .matcher import FeatureMatcher
        if self._matcher is not None and self._matcher.desc_bytes == nbytes:
            return self._matcher
        if self._matcher is None:
            self._matcher = FeatureMatcher(nbytes, device=self.device)
            return self._matcher
        other = getattr(self, "_other", None)
        if other is None or other.desc_bytes != nbytes:
            if other is not None:
                other.close()
            self._other = other = FeatureMatcher(nbytes, device=self.device)
        return other

    @staticmethod
    def _nbytes(desc0, desc1) -> int:
        for d in (desc0, desc1):
            d = np.asarray(d)
            if d.ndim == 2 and d.shape[0]:
                return int(d.shape[1])
        return 64

    def _match(self, pts0, desc0, pts1, desc1, min_d, max_d):
        return self._m(self._nbytes(desc0, desc1)).match(pts0, desc0, pts1, desc1, self._ratioTest, float(min_d),
                                                         float(max_d))

    def setKeyPoints(self, pts, desc, pts_distorted=None) -> None:
        """The new current frame's keypoints (CFrame::setKeyPoints after
        detectFeatures, CTracker.cpp:275-287): undistorted positions,
        descriptors, distorted positions.  They stay resident on the device;
        the previous current frame becomes _prevFrame (CSfM.cpp:626-629)."""
        from .matcher import FeatureMatcher
        d = np.asarray(desc)
        nbytes = int(d.shape[1]) if d.ndim == 2 and d.shape[1] else 64
        if self._matcher is not None and self._matcher.desc_bytes != nbytes:
            self._matcher.close()        # a new descriptor width starts a new frame pair
            self._matcher = None
        if self._matcher is None:
            self._matcher = FeatureMatcher(nbytes, device=self.device)
        self._matcher.push_frame(pts, desc, pts_distorted)

    def matchFeatures(self, *args):
        """Overloads of CTracker::matchFeatures:
        ()                                                 CTracker.cpp:419-477
           the two resident frames (setKeyPoints), distorted positions;
           fills _prevIdx/_currIdx, returns matchCount >= _minFeatures
        (prevFrameIdx, currFrameIdx)                       CTracker.cpp:368-417
           index subsets of the resident frames, undistorted positions;
           returns frame-global (prevMatchIdx, currMatchIdx)
        (pts0, desc0, pts1, desc1)                         CTracker.cpp:114-149
        (pts0, desc0, pts1, desc1, minDist, maxDist)       CTracker.cpp:211-250
        (prevPts, prevDesc, currPts, currDesc, prevIdx, currIdx)   the
           index-subset rule on explicit frame data (no resident frames)."""
        if len(args) == 0:
            self._prevIdx, self._currIdx = self._resident().match_frames(True, self._ratioTest, self._minMatchDistance,
                                                                  self._maxMatchDistance)
            return len(self._prevIdx) >= self._minFeatures
        if len(args) == 2:
            return self._resident().match_subset(args[0], args[1], self._ratioTest, self._minMatchDistance,
                                          self._maxMatchDistance)
        if len(args) == 4:
            return self._match(*args, self._minMatchDistance, self._maxMatchDistance)
        if len(args) == 6 and np.isscalar(args[4]):
            return self._match(*args)
        if len(args) == 6:
            prevPts, prevDesc, currPts, currDesc, prevIdx, currIdx = args
            prevIdx = np.asarray(prevIdx, dtype=np.int64)
            currIdx = np.asarray(currIdx, dtype=np.int64)
            a, b = self._match(np.asarray(prevPts)[prevIdx], np.asarray(prevDesc)[prevIdx],
                               np.asarray(currPts)[currIdx], np.asarray(currDesc)[currIdx],
                               self._minMatchDistance, self._maxMatchDistance)
            return prevIdx[a].astype(np.int32), currIdx[b].astype(np.int32)
        raise TypeError("matchFeatures: unsupported overload")

    def knnMatch2(self, desc0, desc1):
        """The 2-NN Hamming search alone (brisk::BruteForceMatcher::knnMatch, k=2)."""
        return self._m(self._nbytes(desc0, desc1)).knn2(desc0, desc1)

    # ---- optical flow (CTracker.cpp:480-562) -------------------------------
    def pushFrame(self, grey) -> None:
        """Make `grey` (CFrame::getFrameGrey(), u8 [h][w]) the current frame;
        the previous current frame becomes _prevFrame (CSfM.cpp:626-629).
        Its pyramid is built once on the device and kept resident."""
        from .klt import KLTTracker, make_params
        g = np.asarray(grey)
        if self._klt is None or (self._klt.height, self._klt.width) != g.shape:
            if self._klt is not None:
                self._klt.close()
            self._klt = KLTTracker(g.shape[1], g.shape[0], device=self.device,
                                   params=make_params(max_match_distance=self._maxMatchDistance,
                                                      min_match_distance=self._minMatchDistance,
                                                      max_org_feat_dist=self._maxOrgFeatDist))
        self._klt.push_frame(g)

    def computeOpticalFlow(self, prevPtsDistorted, currPtsDistorted) -> bool:
        """LK flow of the previous frame's (distorted) points into the current
        frame, associated with the current frame's detected points; fills
        _prevIdx/_currIdx (CTracker.cpp:520-545) and returns
        matchCount >= _minFeatures (CTracker.cpp:558-561)."""
        if self._klt is None:
            raise RuntimeError("computeOpticalFlow: pushFrame() the previous and current frames first")
        self._prevIdx, self._currIdx = self._klt.compute_optical_flow(prevPtsDistorted, currPtsDistorted)
        return len(self._prevIdx) >= self._minFeatures

    def detectFeaturesOpticalFlow(self) -> bool:
        """goodFeaturesToTrack(500, 0.05, 10) + cornerSubPix(5x5, 20, 0.03) on
        the current frame (CTracker.cpp:252-272); the corners (float32 [n][2],
        what the reference hands to CFrame::setPoints) are kept in
        self.currPoints; returns n >= _minFeatures (CTracker.cpp:267)."""
        if self._klt is None:
            raise RuntimeError("detectFeaturesOpticalFlow: pushFrame() a frame first")
        from .klt import make_gftt_params
        self.currPoints = self._klt.detect_features(make_gftt_params(min_features=self._minFeatures))
        return len(self.currPoints) >= self._minFeatures
