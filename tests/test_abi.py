"""CPU: the C-ABI library loads and exports every symbol include/sfm_amd.h
declares (no compute calls: there is no GPU in this container)."""
import ctypes
import os
import re

import numpy as np

import sfm_amd
from sfm_amd import scene

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "sfm_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sfm_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = ctypes.CDLL(sfm_amd.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # and the Python binding covers all of them
    assert set(names) <= set(sfm_amd.exported_symbols()), set(names) - set(sfm_amd.exported_symbols())


def test_abi_version_and_defaults():
    assert sfm_amd.lib().sfm_abi_version() == 1
    o = sfm_amd.default_options()
    assert o.max_num_iterations == 50 and o.jacobi_scaling == 1
    assert o.function_tolerance == 1e-6 and o.gradient_tolerance == 1e-10 and o.parameter_tolerance == 1e-8
    assert o.initial_trust_region_radius == 1e4 and o.max_trust_region_radius == 1e16
    assert o.min_lm_diagonal == 1e-6 and o.max_lm_diagonal == 1e32 and o.min_relative_decrease == 1e-3


def test_struct_layouts_match_header():
    assert ctypes.sizeof(sfm_amd.BAOptions) == 4 * 4 + 9 * 8
    assert ctypes.sizeof(sfm_amd.BASummary) == 8 * 4 + 6 * 8
    assert ctypes.sizeof(sfm_amd.BAIteration) == 4 * 4 + 6 * 8


def test_device_count_without_gpu_does_not_crash():
    assert sfm_amd.device_count() >= 0


def test_product_path_fails_loudly_without_device():
    if sfm_amd.device_count() > 0:
        return
    try:
        sfm_amd.BundleAdjuster()
    except sfm_amd.SfmError as e:
        assert e.code == -19
    else:
        raise AssertionError("expected ENODEV without a GPU")


def test_solve_rejects_bad_indices_before_touching_the_device():
    s = scene.generate(3, 10, views=2, seed=1)
    bad = s.cam_idx.copy()
    bad[0] = 99
    r, t, X = s.copy_params()
    try:
        sfm_amd.solve(s.uv, bad, s.pt_idx, s.K, r, t, X)
    except sfm_amd.SfmError as e:
        assert e.code in (-22, -19)
    else:
        raise AssertionError("expected an error")
