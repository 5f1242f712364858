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
