"""Host-side mirror of the CMap member next to the BA/matcher hot path
(SURVEY.md §8f row 2): CMap::getRepresentativeDescriptors
(/root/reference/CMap.cpp:345-381) — for every requested map point, the
descriptor (one per observing keyframe) with the smallest sum of Hamming
distances to the point's other descriptors, first on ties.  These are the
map-point descriptors the guided matching of CSfM.cpp:673 and :208-210
feeds to CTracker::matchFeatures.  Runs on the device through the C ABI
(sfm_representative_descriptors); no CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._ffi import check, lib, ptr


def representative_descriptors(desc: np.ndarray, row_off: np.ndarray, device: int = 0):
    """desc uint8 [rows][bytes], row_off int32 [n+1] (point i = rows
    row_off[i]:row_off[i+1]) -> (best row per point int32 [n], descriptors
    uint8 [n][bytes])."""
    desc = np.ascontiguousarray(desc, np.uint8)
    row_off = np.ascontiguousarray(row_off, np.int32)
    n = int(row_off.shape[0]) - 1
    nbytes = int(desc.shape[1]) if desc.ndim == 2 else 64
    best = np.zeros(max(1, n), np.int32)
    out = np.zeros((max(1, n), nbytes), np.uint8)
    check(lib().sfm_representative_descriptors(device, ptr(desc), ptr(row_off), n, nbytes, ptr(best), ptr(out)),
          "sfm_representative_descriptors")
    return best[:n].copy(), out[:n].copy()


class CMap:
    """The descriptor store of CMap (CMap.h: `_descriptor`, one Mat of rows
    per map point) with getRepresentativeDescriptors."""

    def __init__(self, device: int = 0):
        self.device = device
        self._descriptor: list[np.ndarray] = []

    def addPoint(self, descriptors) -> int:
        d = np.ascontiguousarray(descriptors, np.uint8)
        self._descriptor.append(d.reshape(-1, d.shape[-1]))
        return len(self._descriptor) - 1

    def addDescriptor(self, pt_idx: int, descriptor) -> None:
        """A new keyframe observes the point: one more descriptor row."""
        d = np.ascontiguousarray(descriptor, np.uint8).reshape(1, -1)
        self._descriptor[pt_idx] = np.vstack([self._descriptor[pt_idx], d])

    def getRepresentativeDescriptors(self, pts3DIdx) -> np.ndarray:
        """uint8 [len(pts3DIdx)][bytes], in pts3DIdx order (CMap.cpp:345-381)."""
        idx = list(pts3DIdx)
        if not idx:
            return np.zeros((0, 64), np.uint8)
        mats = [self._descriptor[i] for i in idx]
        row_off = np.zeros(len(mats) + 1, np.int32)
        row_off[1:] = np.cumsum([m.shape[0] for m in mats])
        _, out = representative_descriptors(np.vstack(mats), row_off, self.device)
        return out


class DeviceMap:
    """CMap's observation store resident on the device (sfm_map_*, SURVEY.md
    §8f row 2): the multimap gathers of the tracking path (CMap.cpp:145-295,
    CSfM.cpp:648-669) as device queries, with CMap's method names."""

    def __init__(self, desc_bytes: int = 64, device: int = 0):
        self.desc_bytes = int(desc_bytes)
        h = ctypes.c_void_p()
        check(lib().sfm_map_create(device, self.desc_bytes, ctypes.byref(h)), "sfm_map_create")
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().sfm_map_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def size(self):
        n_pts, n_obs, n_rows = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64()
        check(lib().sfm_map_size(self._h, ctypes.byref(n_pts), ctypes.byref(n_obs), ctypes.byref(n_rows)),
              "sfm_map_size")
        return n_pts.value, n_obs.value, n_rows.value

    def addNewPoints(self, pts3D, pts2DIdx, frameNo) -> np.ndarray:
        """pts2DIdx [n_frames][n_pts] (the reference's vector<vector<int>>)."""
        X = np.ascontiguousarray(np.asarray(pts3D, np.float64).reshape(-1, 3))
        n = int(X.shape[0])
        fr = np.ascontiguousarray(np.asarray(frameNo, np.int32).reshape(-1))
        i2 = np.ascontiguousarray(np.asarray(pts2DIdx, np.int32).reshape(len(fr), n))
        out = np.zeros(max(1, n), np.int32)
        check(lib().sfm_map_add_new_points(self._h, n, ptr(X), len(fr), ptr(fr), ptr(i2), ptr(out)),
              "sfm_map_add_new_points")
        return out[:n].copy()

    def addPointMatches(self, pts3DIdx, pts2DIdx, frameNo: int) -> None:
        a = np.ascontiguousarray(np.asarray(pts3DIdx, np.int32).reshape(-1))
        b = np.ascontiguousarray(np.asarray(pts2DIdx, np.int32).reshape(-1))
        check(lib().sfm_map_add_point_matches(self._h, len(a), ptr(a), ptr(b), int(frameNo)),
              "sfm_map_add_point_matches")

    def addDescriptors(self, pts3DIdx, descriptors) -> None:
        a = np.ascontiguousarray(np.asarray(pts3DIdx, np.int32).reshape(-1))
        d = np.ascontiguousarray(np.asarray(descriptors, np.uint8).reshape(len(a), self.desc_bytes))
        check(lib().sfm_map_add_descriptors(self._h, len(a), ptr(a), ptr(d)), "sfm_map_add_descriptors")

    def getPointsAtIdx(self, pts3DIdx) -> np.ndarray:
        a = np.ascontiguousarray(np.asarray(pts3DIdx, np.int32).reshape(-1))
        X = np.zeros((max(1, len(a)), 3))
        check(lib().sfm_map_get_points(self._h, len(a), ptr(a), ptr(X)), "sfm_map_get_points")
        return X[:len(a)].copy()

    def setPointsAtIdx(self, pts3DIdx, pts3D) -> None:
        a = np.ascontiguousarray(np.asarray(pts3DIdx, np.int32).reshape(-1))
        X = np.ascontiguousarray(np.asarray(pts3D, np.float64).reshape(len(a), 3))
        check(lib().sfm_map_set_points(self._h, len(a), ptr(a), ptr(X)), "sfm_map_set_points")

    def getPointsInFrames(self, frameNo) -> np.ndarray:
        fr = np.ascontiguousarray(np.asarray(frameNo, np.int32).reshape(-1))
        cap = max(1, self.size()[0])
        out = np.zeros(cap, np.int32)
        n = ctypes.c_int32()
        check(lib().sfm_map_points_in_frames(self._h, len(fr), ptr(fr), cap, ptr(out), ctypes.byref(n)),
              "sfm_map_points_in_frames")
        return out[:n.value].copy()

    def getPointsInFrame(self, frameNo: int):
        """(pts3DIdx, pts2DIdx) of CMap::getPointsInFrame(pts3DIdx, pts2DIdx, frameNo)."""
        # The 2D list can outgrow the observation count: a point matched k
        # times in this frame emits k 2D indices per entry, k^2 in all
        # (CMap.cpp:225-240).  The call reports both counts before it rejects
        # a short buffer, so a second call with those sizes always fits.
        cap = max(1, self.size()[1])
        for _ in range(2):
            p3 = np.zeros(cap, np.int32)
            p2 = np.zeros(cap, np.int32)
            n3, n2 = ctypes.c_int32(), ctypes.c_int32()
            rc = lib().sfm_map_points_in_frame(self._h, int(frameNo), cap, ptr(p3), ctypes.byref(n3), ptr(p2),
                                               ctypes.byref(n2))
            need = max(n3.value, n2.value)
            if rc == 0 or need <= cap:
                break
            cap = need
        check(rc, "sfm_map_points_in_frame")
        return p3[:n3.value].copy(), p2[:n2.value].copy()

    def getPointsInFrameMulti(self, frameNo):
        """[(pts3DIdx, pts2DIdx) of getPointsInFrame(f) for f in frameNo], in
        one device query (the per-keyframe gather of CSfM::bundleAdjustment,
        CSfM.cpp:321-340)."""
        fr = np.ascontiguousarray(np.asarray(frameNo, np.int32).reshape(-1))
        nf = len(fr)
        off3 = np.zeros(nf + 1, np.int32)
        off2 = np.zeros(nf + 1, np.int32)
        cap = max(1, self.size()[1])
        for _ in range(2):
            p3 = np.zeros(cap, np.int32)
            p2 = np.zeros(cap, np.int32)
            rc = lib().sfm_map_points_in_frame_multi(self._h, nf, ptr(fr), cap, ptr(p3), ptr(off3), ptr(p2), ptr(off2))
            need = int(max(off3[-1], off2[-1]))
            if rc == 0 or need <= cap:
                break
            cap = need
        check(rc, "sfm_map_points_in_frame_multi")
        return [(p3[off3[i]:off3[i + 1]].copy(), p2[off2[i]:off2[i + 1]].copy()) for i in range(nf)]

    def matchFrame(self, matcher, frameNo, existing, R, t, K, train_idx, ratio: float = 0.8, min_distance: float = 0.0,
                   max_distance: float = 7.0):
        """CSfM::findMapPointsInCurrentFrame (CSfM.cpp:634-692) on the device
        (sfm_map_match_frame): the keyframes' points minus `existing`,
        projected with (R, t, K), their representative descriptors matched
        against the keypoints `train_idx` of the frame last pushed to
        `matcher`.  Returns (map point ids, frame-global keypoint ids)."""
        fr = np.ascontiguousarray(np.asarray(frameNo, np.int32).reshape(-1))
        ex = np.ascontiguousarray(np.asarray(existing, np.int32).reshape(-1))
        tr = np.ascontiguousarray(np.asarray(train_idx, np.int32).reshape(-1))
        R9 = np.ascontiguousarray(np.asarray(R, np.float64).reshape(9))
        t3 = np.ascontiguousarray(np.asarray(t, np.float64).reshape(3))
        K9 = np.ascontiguousarray(np.asarray(K, np.float64).reshape(9))
        cap = max(1, len(tr))
        pm = np.zeros(cap, np.int32)
        km = np.zeros(cap, np.int32)
        n = ctypes.c_int32(0)
        check(lib().sfm_map_match_frame(self._h, matcher._h, len(fr), ptr(fr), len(ex), ptr(ex), ptr(R9), ptr(t3),
                                        ptr(K9), len(tr), ptr(tr), float(ratio), float(min_distance),
                                        float(max_distance), cap, ptr(pm), ptr(km), ctypes.byref(n)),
              "sfm_map_match_frame")
        return pm[:n.value].copy(), km[:n.value].copy()

    def getRepresentativeDescriptors(self, pts3DIdx, return_best: bool = False):
        a = np.ascontiguousarray(np.asarray(pts3DIdx, np.int32).reshape(-1))
        out = np.zeros((max(1, len(a)), self.desc_bytes), np.uint8)
        best = np.zeros(max(1, len(a)), np.int32)
        if len(a):
            check(lib().sfm_map_representative_descriptors(self._h, len(a), ptr(a), ptr(out), ptr(best)),
                  "sfm_map_representative_descriptors")
        if return_best:
            return out[:len(a)].copy(), best[:len(a)].copy()
        return out[:len(a)].copy()
