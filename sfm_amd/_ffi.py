"""ctypes binding of include/sfm_amd.h (libsfm_amd.so, built in-tree).

The product path has no CPU fallback: if the HIP library is missing or a
call fails, an exception is raised.  Struct layouts mirror the header
field for field.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_int64, c_uint8, c_uint64, c_void_p

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SFM_AMD_LIB") or os.path.join(_HERE, "libsfm_amd.so")


class SfmError(RuntimeError):
    """A C-ABI call returned a negative errno-style code."""

    def __init__(self, code: int, what: str, msg: str):
        super().__init__(f"{what} failed with {code}: {msg}")
        self.code = code


class BAOptions(ctypes.Structure):
    _fields_ = [
        ("max_num_iterations", c_int32),
        ("max_num_consecutive_invalid_steps", c_int32),
        ("jacobi_scaling", c_int32),
        ("reserved0", c_int32),
        ("function_tolerance", c_double),
        ("gradient_tolerance", c_double),
        ("parameter_tolerance", c_double),
        ("initial_trust_region_radius", c_double),
        ("max_trust_region_radius", c_double),
        ("min_trust_region_radius", c_double),
        ("min_lm_diagonal", c_double),
        ("max_lm_diagonal", c_double),
        ("min_relative_decrease", c_double),
    ]


class BASummary(ctypes.Structure):
    _fields_ = [
        ("termination_type", c_int32),
        ("num_iterations", c_int32),
        ("num_successful_steps", c_int32),
        ("num_unsuccessful_steps", c_int32),
        ("num_invalid_steps", c_int32),
        ("num_residual_evaluations", c_int32),
        ("num_jacobian_evaluations", c_int32),
        ("num_linear_solves", c_int32),
        ("initial_cost", c_double),
        ("final_cost", c_double),
        ("wall_time_s", c_double),
        ("jacobian_time_s", c_double),
        ("linear_solver_time_s", c_double),
        ("residual_time_s", c_double),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class BAIteration(ctypes.Structure):
    _fields_ = [
        ("iteration", c_int32),
        ("step_is_valid", c_int32),
        ("step_is_successful", c_int32),
        ("reserved", c_int32),
        ("cost", c_double),
        ("cost_change", c_double),
        ("gradient_max_norm", c_double),
        ("step_norm", c_double),
        ("relative_decrease", c_double),
        ("trust_region_radius", c_double),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_ if name != "reserved"}


class KLTParams(ctypes.Structure):
    _fields_ = [
        ("win_size", c_int32),
        ("max_level", c_int32),
        ("max_count", c_int32),
        ("reserved", c_int32),
        ("epsilon", c_double),
        ("min_eig_threshold", c_double),
        ("max_match_distance", c_double),
        ("min_match_distance", c_double),
        ("max_org_feat_dist", c_double),
    ]


class GFTTParams(ctypes.Structure):
    _fields_ = [
        ("max_corners", c_int32),
        ("subpix_win", c_int32),
        ("subpix_max_iter", c_int32),
        ("min_features", c_int32),
        ("quality_level", c_double),
        ("min_distance", c_double),
        ("subpix_epsilon", c_double),
    ]


# name -> (restype, argtypes)
_SIGNATURES = {
    "sfm_abi_version": (c_int32, []),
    "sfm_last_error": (c_char_p, []),
    "sfm_ba_default_options": (None, [POINTER(BAOptions)]),
    "sfm_device_count": (c_int32, []),
    "sfm_ba_solve": (c_int, [POINTER(BAOptions), c_int32, c_int64, c_void_p, c_void_p, c_void_p, c_int32, c_void_p,
                             c_void_p, c_void_p, c_int32, c_void_p, POINTER(BASummary), c_void_p, c_int32,
                             POINTER(c_int32)]),
    "sfm_ba_create": (c_int, [c_int32, POINTER(c_void_p)]),
    "sfm_ba_destroy": (c_int, [c_void_p]),
    "sfm_ba_set_problem": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p,
                                   c_void_p, c_int32, c_void_p]),
    "sfm_ba_reset_parameters": (c_int, [c_void_p]),
    "sfm_ba_solve_resident": (c_int, [c_void_p, POINTER(BAOptions), c_int32, POINTER(BASummary), c_void_p, c_int32,
                                      POINTER(c_int32)]),
    "sfm_ba_get_parameters": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "sfm_ba_evaluate": (c_int, [c_void_p, POINTER(c_double), c_void_p, c_void_p]),
    "sfm_ba_bench_jacobian": (c_int, [c_void_p, c_int32, POINTER(c_double)]),
    "sfm_ba_phase_times": (c_int, [c_void_p, c_void_p]),
    "sfm_ba_set_profiling": (c_int, [c_void_p, c_int32]),
    "sfm_ba_sync": (c_int, [c_void_p]),
    "sfm_comm_unique_id": (c_int, [c_void_p]),
    "sfm_ba_set_comm": (c_int, [c_void_p, c_int32, c_int32, c_void_p]),
    "sfm_ba_set_host_comm": (c_int, [c_void_p, c_int32, c_int32, c_void_p, c_void_p]),
    "sfm_ba_set_host_collectives": (c_int, [c_void_p, c_int32, c_int32, c_void_p, c_void_p]),
    "sfm_ba_set_distributed_factor": (c_int, [c_void_p, c_int32]),
    "sfm_match_features": (c_int, [c_int32, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_int32,
                                   c_double, c_double, c_double, c_void_p, c_void_p, POINTER(c_int32)]),
    "sfm_knn2_hamming": (c_int, [c_int32, c_void_p, c_int32, c_void_p, c_int32, c_int32, c_void_p, c_void_p,
                                 c_void_p, c_void_p]),
    "sfm_matcher_create": (c_int, [c_int32, c_int32, POINTER(c_void_p)]),
    "sfm_matcher_destroy": (c_int, [c_void_p]),
    "sfm_matcher_push_frame": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32]),
    "sfm_matcher_match_subset": (c_int, [c_void_p, c_void_p, c_int32, c_void_p, c_int32, c_double, c_double, c_double,
                                         c_void_p, c_void_p, POINTER(c_int32)]),
    "sfm_matcher_match_frames": (c_int, [c_void_p, c_int32, c_double, c_double, c_double, c_void_p, c_void_p,
                                         POINTER(c_int32)]),
    "sfm_matcher_match": (c_int, [c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_double,
                                  c_double, c_double, c_void_p, c_void_p, POINTER(c_int32)]),
    "sfm_matcher_knn2": (c_int, [c_void_p, c_void_p, c_int32, c_void_p, c_int32, c_void_p, c_void_p, c_void_p,
                                 c_void_p]),
    "sfm_matcher_last_time": (c_int, [c_void_p, c_void_p]),
    "sfm_representative_descriptors": (c_int, [c_int32, c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p]),
    "sfm_brisk_describe": (c_int, [c_int32, c_void_p, c_int32, c_int32, c_void_p, c_int32, c_void_p, c_void_p,
                                   c_void_p, POINTER(c_int32)]),
    "sfm_klt_brisk_detect_describe": (c_int, [c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                              c_void_p]),
    "sfm_brisk_detect_describe": (c_int, [c_int32, c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32, c_void_p,
                                          c_void_p, c_void_p, POINTER(c_int32)]),
    "sfm_map_create": (c_int, [c_int32, c_int32, POINTER(c_void_p)]),
    "sfm_map_destroy": (c_int, [c_void_p]),
    "sfm_map_size": (c_int, [c_void_p, POINTER(c_int32), POINTER(c_int64), POINTER(c_int64)]),
    "sfm_map_add_new_points": (c_int, [c_void_p, c_int32, c_void_p, c_int32, c_void_p, c_void_p, c_void_p]),
    "sfm_map_add_point_matches": (c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_int32]),
    "sfm_map_add_descriptors": (c_int, [c_void_p, c_int32, c_void_p, c_void_p]),
    "sfm_map_get_points": (c_int, [c_void_p, c_int32, c_void_p, c_void_p]),
    "sfm_map_set_points": (c_int, [c_void_p, c_int32, c_void_p, c_void_p]),
    "sfm_map_points_in_frames": (c_int, [c_void_p, c_int32, c_void_p, c_int32, c_void_p, POINTER(c_int32)]),
    "sfm_map_points_in_frame": (c_int, [c_void_p, c_int32, c_int32, c_void_p, POINTER(c_int32), c_void_p,
                                        POINTER(c_int32)]),
    "sfm_map_points_in_frame_multi": (c_int, [c_void_p, c_int32, c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                                              c_void_p]),
    "sfm_map_representative_descriptors": (c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p]),
    "sfm_map_match_frame": (c_int, [c_void_p, c_void_p, c_int32, c_void_p, c_int32, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_int32, c_void_p, c_double, c_double, c_double, c_int32, c_void_p,
                                    c_void_p, POINTER(c_int32)]),
    "sfm_matcher_store_keyframe": (c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_int32]),
    "sfm_matcher_match_keyframes": (c_int, [c_void_p, c_int32, c_void_p, c_int32, c_void_p, c_int32, c_void_p,
                                            c_int32, c_double, c_double, c_double, c_void_p, c_void_p,
                                            POINTER(c_int32)]),
    "sfm_track_pnp": (c_int, [c_void_p, c_void_p, c_int32, c_void_p, c_double, c_double, c_double, c_int32,
                              c_void_p, c_int32, c_double, c_double, c_void_p, c_void_p, POINTER(c_int32),
                              POINTER(c_int32), c_int32, c_void_p, c_void_p, POINTER(c_int32)]),
    "sfm_pnp_ransac": (c_int, [c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_int32, c_double, c_double,
                               c_void_p, c_void_p, c_void_p, POINTER(c_int32), POINTER(c_int32)]),
    "sfm_triangulate_points": (c_int, [c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p,
                                       c_void_p]),
    "sfm_dense_spd_solve": (c_int, [c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_int32, POINTER(c_double),
                                    POINTER(c_int32)]),
    "sfm_bench_stream_copy": (c_int, [c_int32, c_int64, c_int32, POINTER(c_double)]),
    "sfm_dist_factor_profile": (c_int, [c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p]),
    "sfm_klt_default_params": (None, [POINTER(KLTParams)]),
    "sfm_klt_create": (c_int, [c_int32, c_int32, c_int32, POINTER(KLTParams), POINTER(c_void_p)]),
    "sfm_klt_destroy": (c_int, [c_void_p]),
    "sfm_klt_num_levels": (c_int32, [c_void_p]),
    "sfm_klt_push_frame": (c_int, [c_void_p, c_void_p, c_int32]),
    "sfm_klt_get_level": (c_int, [c_void_p, c_int32, c_int32, c_void_p, c_void_p, POINTER(c_int32),
                                  POINTER(c_int32)]),
    "sfm_klt_calc_flow": (c_int, [c_void_p, c_void_p, c_int32, c_void_p, c_void_p]),
    "sfm_klt_compute_optical_flow": (c_int, [c_void_p, c_void_p, c_int32, c_void_p, c_int32, c_void_p, c_void_p,
                                             POINTER(c_int32), c_void_p, c_void_p]),
    "sfm_klt_phase_times": (c_int, [c_void_p, c_void_p]),
    "sfm_calc_optical_flow_pyr_lk": (c_int, [c_int32, c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_int32,
                                             c_void_p, c_void_p, POINTER(KLTParams)]),
    "sfm_gftt_default_params": (None, [POINTER(GFTTParams)]),
    "sfm_klt_detect_features": (c_int, [c_void_p, POINTER(GFTTParams), c_void_p, c_int32, POINTER(c_int32)]),
    "sfm_klt_detect_time": (c_int, [c_void_p, POINTER(c_double)]),
    "sfm_good_features_to_track": (c_int, [c_int32, c_void_p, c_int32, c_int32, c_int32, POINTER(GFTTParams),
                                           c_void_p, c_int32, POINTER(c_int32)]),
    "sfm_scene_default_intrinsics": (None, [c_void_p]),
    "sfm_scene_generate": (c_int, [c_int32, c_int32, c_int32, c_int32, c_int32, c_uint64, c_double, c_double,
                                   c_double, c_double] + [c_void_p] * 10),
}

_LIB = None


def lib() -> ctypes.CDLL:
    """Load libsfm_amd.so once.  Raises if it has not been built."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(there is no CPU fallback for the HIP path)")
        L = ctypes.CDLL(LIB_PATH)
        # (an A/B build of an earlier revision, SFM_AMD_LIB, may lack newer
        # entry points: those stay unbound there; the in-tree library must
        # export every one, tests/test_abi.py)
        variant = "SFM_AMD_LIB" in os.environ
        for name, (res, args) in _SIGNATURES.items():
            if variant and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def exported_symbols() -> list[str]:
    return list(_SIGNATURES)


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise SfmError(rc, what, lib().sfm_last_error().decode(errors="replace"))


def ptr(a: np.ndarray | None) -> c_void_p | None:
    """The array's data address for a C-ABI call.

    Unlike ctypes' data_as, the returned c_void_p holds NO reference to the
    array: the caller must keep `a` alive (bound to a local name) until the
    call returns -- never pass a temporary such as
    ptr(np.ascontiguousarray(x)) straight into lib().fn(...)."""
    if a is None:
        return None
    assert a.flags.c_contiguous, "arrays passed to the C ABI must be C-contiguous"
    # (the array interface's address: ~1.4 us, where ctypes.data_as takes ~5 us
    # per array -- 20-30 us of every keyframe solve's call)
    return c_void_p(a.__array_interface__["data"][0])


def default_options() -> BAOptions:
    o = BAOptions()
    lib().sfm_ba_default_options(ctypes.byref(o))
    return o


def default_klt_params() -> KLTParams:
    p = KLTParams()
    lib().sfm_klt_default_params(ctypes.byref(p))
    return p


def default_gftt_params() -> GFTTParams:
    p = GFTTParams()
    lib().sfm_gftt_default_params(ctypes.byref(p))
    return p


def device_count() -> int:
    return int(lib().sfm_device_count())


__all__ = ["lib", "check", "ptr", "BAOptions", "BASummary", "BAIteration", "KLTParams", "GFTTParams", "SfmError",
           "default_options", "default_klt_params", "default_gftt_params",
           "device_count", "exported_symbols", "LIB_PATH", "c_uint8"]
