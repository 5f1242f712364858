"""sfm_amd — MI355X-native bundle-adjustment + tracking core for hulop/SfM.

The compute path is libsfm_amd.so (hand-written HIP kernels for gfx950 + a
C++ LM driver behind the C ABI of include/sfm_amd.h).  This package is the
thin host-side mirror of the reference's CTracker surface; it never falls
back to CPU arithmetic.
"""
from ._ffi import (BAIteration, BAOptions, BASummary, SfmError, LIB_PATH, default_options, device_count,
                   exported_symbols, lib)
from .ba import BundleAdjuster, make_options, solve, STRUCT_ONLY, POSE_ONLY, STRUCT_AND_POSE
from .ctracker import CTracker
from . import scene, video
from .klt import KLTTracker, calc_optical_flow_pyr_lk
from .cmap import CMap, DeviceMap, representative_descriptors
from .pnp import solvePnPRansac

__all__ = ["BundleAdjuster", "CTracker", "CMap", "DeviceMap", "solvePnPRansac", "representative_descriptors", "KLTTracker", "calc_optical_flow_pyr_lk", "video", "BAOptions", "BASummary", "BAIteration", "SfmError", "make_options",
           "solve", "default_options", "device_count", "exported_symbols", "lib", "scene", "LIB_PATH",
           "STRUCT_ONLY", "POSE_ONLY", "STRUCT_AND_POSE"]
