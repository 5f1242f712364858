"""Per-frame pose: cv::solvePnPRansac as
CSfM::tracking calls it (/root/reference/CSfM.cpp:553-565), on the device
through the C ABI (sfm_pnp_ransac; pnp_kernels.hip).  OpenCV 3.0 semantics
(see oracle/pnp_oracle.py for the restatement and its caveats).  No CPU
fallback.
"""
from __future__ import annotations

import ctypes
from ctypes import c_int32

import numpy as np

from ._ffi import check, lib, ptr


def solvePnPRansac(objectPoints, imagePoints, cameraMatrix, iterationsCount: int = 20, reprojectionError: float = 7.0,
                   confidence: float = 0.99, device: int = 0):
    """-> (found, rvec [3], tvec [3], inliers int32 [k]).  Defaults are the
    reference's call (CSfM.cpp:553-560)."""
    obj = np.ascontiguousarray(np.asarray(objectPoints, np.float64).reshape(-1, 3))
    img = np.ascontiguousarray(np.asarray(imagePoints, np.float64).reshape(-1, 2))
    if obj.shape[0] != img.shape[0]:
        raise ValueError(f"{obj.shape[0]} object points but {img.shape[0]} image points")
    K = np.ascontiguousarray(np.asarray(cameraMatrix, np.float64).reshape(9))
    n = int(obj.shape[0])
    rvec, tvec = np.zeros(3), np.zeros(3)
    inl = np.zeros(max(1, n), np.int32)
    n_inl, found = c_int32(0), c_int32(0)
    check(lib().sfm_pnp_ransac(device, n, ptr(obj), ptr(img), ptr(K), int(iterationsCount), float(reprojectionError),
                               float(confidence), ptr(rvec), ptr(tvec), ptr(inl), ctypes.byref(n_inl),
                               ctypes.byref(found)), "sfm_pnp_ransac")
    return bool(found.value), rvec, tvec, inl[:n_inl.value].copy()
