"""CPU restatement of CMap's observation store (TEST INFRASTRUCTURE ONLY: the
checker of sfm_map_*, imported by tests/ and never by the product).

Follows /root/reference/CMap.cpp with the reference's containers made
explicit:

* addNewPoints (CMap.cpp:36-78): per new point i (in order), per frame j:
  _frameNo[p].push_back(frameNo[j]), _pts2DIdx[p].push_back(pts2DIdx[j][i]),
  _frameViewsPointIdx.emplace(frameNo[j], p);
* addPointMatches (CMap.cpp:118-132): the same three appends per match;
* addDescriptors (CMap.cpp:308-315): _descriptor[p].push_back(row);
* the reference's container is an std::unordered_multimap (CMap.h:96-97),
  whose equal_range order is implementation-defined: libc++ (the
  reference's Xcode toolchain) keeps equal keys in insertion order, while
  libstdc++ links a new equal key in next to its existing group rather than
  at its end, so it does not yield insertion order.  This restatement
  adopts insertion order (libc++); that order is the BA observation order
  of CSfM::bundleAdjustment, so the choice is part of the unpinned parity.
  The multimap is kept as the list of (frame, point) entries in emplace
  order;
* getPointsInFrames(pts3DIdx, frameNo) (CMap.cpp:277-295): the points of
  every frame's equal_range appended, then sort + unique;
* getPointsInFrame(pts3DIdx, pts2DIdx, frameNo) (CMap.cpp:225-240): per
  equal_range entry, push the point, then EVERY i with _frameNo[p][i] ==
  frameNo pushes _pts2DIdx[p][i];
* getRepresentativeDescriptors (CMap.cpp:345-381): the row with the
  smallest sum of Hamming distances to the point's rows, first on ties.

Parity anchor: the reference's own code paths above (no fixtures exist for
CMap); the tests pin this restatement on hand-checked cases.
"""
from __future__ import annotations

import numpy as np


class CMapOracle:
    def __init__(self, desc_bytes: int = 64):
        self.desc_bytes = desc_bytes
        self.pts3D: list[np.ndarray] = []
        self.frameNo: list[list[int]] = []
        self.pts2DIdx: list[list[int]] = []
        self.descriptor: list[list[np.ndarray]] = []
        self.mm: list[tuple[int, int]] = []  # _frameViewsPointIdx, emplace order

    def addNewPoints(self, pts3D, pts2DIdx, frameNo):
        """pts2DIdx[j][i]: frame j's 2D index of new point i (CMap.cpp:60-66)."""
        out = []
        for i in range(len(pts3D)):
            p = len(self.pts3D)
            self.pts3D.append(np.asarray(pts3D[i], np.float64).copy())
            self.frameNo.append([])
            self.pts2DIdx.append([])
            self.descriptor.append([])
            for j in range(len(pts2DIdx)):
                self.frameNo[p].append(int(frameNo[j]))
                self.pts2DIdx[p].append(int(pts2DIdx[j][i]))
                self.mm.append((int(frameNo[j]), p))
            out.append(p)
        return out

    def addPointMatches(self, pts3DIdx, pts2DIdx, frameNo):
        for idx, i2 in zip(pts3DIdx, pts2DIdx):
            self.pts2DIdx[idx].append(int(i2))
            self.frameNo[idx].append(int(frameNo))
            self.mm.append((int(frameNo), int(idx)))

    def addDescriptors(self, pts3DIdx, descriptors):
        for i, idx in enumerate(pts3DIdx):
            self.descriptor[idx].append(np.asarray(descriptors[i], np.uint8).copy())

    def equal_range(self, f):
        return [p for (k, p) in self.mm if k == f]

    def getPointsInFrames(self, frameNo):
        out = []
        for f in frameNo:
            out.extend(self.equal_range(f))
        return sorted(set(out))

    def getPointsInFrame(self, frameNo):
        p3, p2 = [], []
        for p in self.equal_range(frameNo):
            p3.append(p)
            for i in range(len(self.frameNo[p])):
                if self.frameNo[p][i] == frameNo:
                    p2.append(self.pts2DIdx[p][i])
        return p3, p2

    def getPointsAtIdx(self, idx):
        return np.array([self.pts3D[i] for i in idx]).reshape(-1, 3)

    def getRepresentativeDescriptors(self, pts3DIdx):
        rows, best = [], []
        for idx in pts3DIdx:
            d = self.descriptor[idx]
            sums = [sum(int(np.unpackbits(a ^ b).sum()) for b in d) for a in d]
            b = int(np.argmin(sums))  # first minimum
            best.append(b)
            rows.append(d[b])
        return np.array(best, np.int32), np.array(rows, np.uint8).reshape(-1, self.desc_bytes)
