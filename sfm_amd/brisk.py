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


def _detect_call(call, cap: int, describe: bool):
    for _ in range(2):  # the call reports the count before it rejects a short buffer
        kps = np.zeros((cap, 5), np.float32)
        lay = np.zeros(cap, np.int32)
        desc = np.zeros((cap, DESC_BYTES), np.uint8) if describe else None
        n = ctypes.c_int32()
        rc = call(cap, kps, lay, desc, n)
        if rc == 0 or n.value <= cap:
            break
        cap = n.value
    return rc, kps, lay, desc, n.value


def detect(img, threshold: int = 60, octaves: int = 6, describe: bool = True, device: int = 0):
    """CTracker::detectFeatures: BriskFeatureDetector(threshold, octaves,
    true) + the descriptor.  -> (keypoints [n][5] (x, y, size, angle,
    response) float32, layer [n], descriptors uint8 [n][64] or None)."""
    im = np.ascontiguousarray(img, np.uint8)
    if im.ndim != 2:
        raise ValueError("img must be 2-D 8-bit grey")
    rc, kps, lay, desc, k = _detect_call(
        lambda cap, kps, lay, desc, n: lib().sfm_brisk_detect_describe(
            device, ptr(im), im.shape[1], im.shape[0], int(threshold), int(octaves), cap, ptr(kps), ptr(lay),
            ptr(desc) if desc is not None else None, ctypes.byref(n)),
        max(1024, im.shape[0] * im.shape[1] // 64), describe)
    check(rc, "sfm_brisk_detect_describe")
    return kps[:k].copy(), lay[:k].copy(), (desc[:k].copy() if describe else None)


def detect_resident(klt, threshold: int = 60, octaves: int = 6, describe: bool = True):
    """detect() on the current frame of a KLTTracker (sfm_klt_brisk_detect_
    describe): the frame sfm_klt_push_frame uploaded, no second upload."""
    rc, kps, lay, desc, k = _detect_call(
        lambda cap, kps, lay, desc, n: lib().sfm_klt_brisk_detect_describe(
            klt._h, int(threshold), int(octaves), cap, ptr(kps), ptr(lay), ptr(desc) if desc is not None else None,
            ctypes.byref(n)),
        max(1024, klt.width * klt.height // 64), describe)
    check(rc, "sfm_klt_brisk_detect_describe")
    return kps[:k].copy(), lay[:k].copy(), (desc[:k].copy() if describe else None)
