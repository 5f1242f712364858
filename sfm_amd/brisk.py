"""BRISK on the device (sfm_brisk_*; CTracker::detectFeatures,
/root/reference/CTracker.cpp:275-287).  BRISK as published, in its reference
implementation's form (oracle/brisk_oracle.py); the reference's ethz-asl
BRISK 2 library is absent, so parity with it is unpinned.
No CPU fallback."""
from __future__ import annotations

import ctypes

import numpy as np

from ._ffi import check, lib, ptr

DESC_BYTES = 64


def describe(img, keypoints, device: int = 0):
    """img uint8 [h][w], keypoints [n][3] (x, y, size) -> (kept index [m],
    angle [m] degrees, descriptors uint8 [m][64]); keypoints too near the
    border for their scale are dropped, as the reference's compute does."""
    im = np.ascontiguousarray(img, np.uint8)
    if im.ndim != 2:
        raise ValueError("img must be 2-D 8-bit grey")
    kp = np.ascontiguousarray(np.asarray(keypoints, np.float32).reshape(-1, 3))
    n = int(kp.shape[0])
    kept = np.zeros(max(1, n), np.int32)
    ang = np.zeros(max(1, n), np.float32)
    desc = np.zeros((max(1, n), DESC_BYTES), np.uint8)
    m = ctypes.c_int32()
    check(lib().sfm_brisk_describe(device, ptr(im), im.shape[1], im.shape[0], ptr(kp), n, ptr(kept), ptr(ang),
                                   ptr(desc), ctypes.byref(m)), "sfm_brisk_describe")
    k = m.value
    return kept[:k].copy(), ang[:k].copy(), desc[:k].copy()
