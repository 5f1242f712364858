"""Device bundle adjuster (resident-problem API of include/sfm_amd.h)."""
from __future__ import annotations

import ctypes
from ctypes import c_double, c_int32, c_void_p

import numpy as np

from ._ffi import BAIteration, BAOptions, BASummary, check, default_options, lib, ptr

STRUCT_ONLY, POSE_ONLY, STRUCT_AND_POSE = 0, 1, 2   # CTracker::BA_TYPE (CTracker.h:67)
TERMINATION = {0: "CONVERGENCE", 1: "NO_CONVERGENCE", 2: "FAILURE"}
PHASES = ["jacobian", "cam_reduce", "point_eval", "point_prep", "schur", "cholesky", "backsolve", "backsub", "other"]


def _f64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


def _i32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.int32)


def _check_shapes(uv, cam_idx, pt_idx, K9, rot, t, X) -> None:
    """Shapes the C ABI reads (it trusts n_obs / n_cams / n_pts): a short
    array would be an out-of-bounds host read, so refuse it here."""
    n = uv.shape[0] if uv.ndim == 2 else -1
    if uv.ndim != 2 or uv.shape[1] != 2:
        raise ValueError(f"uv must be (n, 2), got {uv.shape}")
    if cam_idx.shape != (n,) or pt_idx.shape != (n,):
        raise ValueError(f"cam_idx / pt_idx must be ({n},), got {cam_idx.shape} / {pt_idx.shape}")
    if rot.ndim != 2 or rot.shape[1] != 3 or t.shape != rot.shape:
        raise ValueError(f"rot and t must be (C, 3), got {rot.shape} / {t.shape}")
    C = rot.shape[0]
    if K9.size != 9 * C or not (K9.shape in ((C, 9), (C, 3, 3)) or (C == 1 and K9.shape in ((9,), (3, 3)))):
        raise ValueError(f"K must be (C, 9) or (C, 3, 3) with C = {C}, got {K9.shape}")
    if X.ndim != 2 or X.shape[1] != 3:
        raise ValueError(f"X must be (P, 3), got {X.shape}")


def make_options(**overrides) -> BAOptions:
    o = default_options()
    for k, v in overrides.items():
        if not hasattr(o, k):
            raise KeyError(k)
        setattr(o, k, v)
    return o


class BundleAdjuster:
    """A problem resident in HBM on one GPU (or one landmark shard of it)."""

    def __init__(self, device: int = 0):
        h = c_void_p()
        check(lib().sfm_ba_create(device, ctypes.byref(h)), "sfm_ba_create")
        self._h = h
        self.device = device
        self.n_obs = self.n_cams = self.n_pts = 0

    def close(self) -> None:
        if self._h:
            lib().sfm_ba_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- multi-GPU -------------------------------------------------------
    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_uint8 * 128)()
        check(lib().sfm_comm_unique_id(buf), "sfm_comm_unique_id")
        return bytes(buf)

    def set_comm(self, nranks: int, rank: int, uid: bytes) -> None:
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        check(lib().sfm_ba_set_comm(self._h, nranks, rank, buf), "sfm_ba_set_comm")

    # test hook: the sharded path with a host all-reduce (several ranks on ONE GPU)
    ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(c_double), ctypes.c_int64, ctypes.c_int32,
                                    c_void_p)

    def set_host_comm(self, nranks: int, rank: int, allreduce) -> None:
        """allreduce(array float64 view, op) with op 0 = sum, 1 = max, in place
        (e.g. torch.distributed over gloo); see sfm_ba_set_host_comm."""
        def _cb(buf, count, op, user):
            try:
                allreduce(np.ctypeslib.as_array(buf, (int(count),)), int(op))
                return 0
            except Exception:
                return 1
        self._host_cb = BundleAdjuster.ALLREDUCE_FN(_cb)  # kept alive with the handle
        check(lib().sfm_ba_set_host_comm(self._h, nranks, rank, ctypes.cast(self._host_cb, c_void_p), None),
              "sfm_ba_set_host_comm")

    COLLECTIVE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int32, ctypes.POINTER(c_double),
                                     ctypes.POINTER(c_double), ctypes.c_int64, ctypes.c_int32, c_void_p)

    def set_host_collectives(self, nranks: int, rank: int, allreduce, broadcast, reduce_scatter, reduce) -> None:
        """The host hook with the distributed factor's collectives as well
        (sfm_ba_set_host_collectives): allreduce(buf, op), broadcast(buf, root)
        and reduce(buf, root) in place on a float64 array; reduce_scatter(buf,
        out) with buf holding nranks segments of len(out), this rank's summed
        segment into out."""
        def _cb(kind, buf, out, count, arg, user):
            try:
                n = int(count)
                if kind == 3:
                    reduce(np.ctypeslib.as_array(buf, (n,)), int(arg))
                elif kind == 2:
                    reduce_scatter(np.ctypeslib.as_array(buf, (n * nranks,)), np.ctypeslib.as_array(out, (n,)))
                elif kind == 1:
                    broadcast(np.ctypeslib.as_array(buf, (n,)), int(arg))
                else:
                    allreduce(np.ctypeslib.as_array(buf, (n,)), int(arg))
                return 0
            except Exception:
                return 1
        self._host_cb = BundleAdjuster.COLLECTIVE_FN(_cb)  # kept alive with the handle
        check(lib().sfm_ba_set_host_collectives(self._h, nranks, rank, ctypes.cast(self._host_cb, c_void_p), None),
              "sfm_ba_set_host_collectives")

    def set_distributed_factor(self, panel_tiles: int) -> None:
        """0: replicated reduced-camera factor (all-reduce of the packed
        system); k > 0: 1-D block-cyclic panels of k 64-column tiles."""
        check(lib().sfm_ba_set_distributed_factor(self._h, int(panel_tiles)), "sfm_ba_set_distributed_factor")

    # ---- problem ---------------------------------------------------------
    def set_problem(self, uv, cam_idx, pt_idx, K9, rot, t, X) -> None:
        uv, K9, rot, t, X = _f64(uv), _f64(K9), _f64(rot), _f64(t), _f64(X)
        cam_idx, pt_idx = _i32(cam_idx), _i32(pt_idx)
        _check_shapes(uv, cam_idx, pt_idx, K9, rot, t, X)
        n = int(uv.shape[0])
        C, P = int(rot.shape[0]), int(X.shape[0])
        check(lib().sfm_ba_set_problem(self._h, n, ptr(uv), ptr(cam_idx), ptr(pt_idx), C, ptr(K9), ptr(rot),
                                       ptr(t), P, ptr(X)), "sfm_ba_set_problem")
        self.n_obs, self.n_cams, self.n_pts = n, C, P

    def reset(self) -> None:
        check(lib().sfm_ba_reset_parameters(self._h), "sfm_ba_reset_parameters")

    def solve(self, options: BAOptions | None = None, mode: int = STRUCT_AND_POSE, trace_cap: int = 128):
        opts = options if options is not None else default_options()
        sm = BASummary()
        tr = (BAIteration * trace_cap)()
        tl = c_int32(0)
        check(lib().sfm_ba_solve_resident(self._h, ctypes.byref(opts), mode, ctypes.byref(sm), tr, trace_cap,
                                          ctypes.byref(tl)), "sfm_ba_solve_resident")
        return sm, [tr[i].as_dict() for i in range(tl.value)]

    def parameters(self):
        rot = np.zeros((self.n_cams, 3))
        t = np.zeros((self.n_cams, 3))
        X = np.zeros((self.n_pts, 3))
        check(lib().sfm_ba_get_parameters(self._h, ptr(rot), ptr(t), ptr(X)), "sfm_ba_get_parameters")
        return rot, t, X

    def evaluate(self, want_jacobian: bool = True):
        cost = c_double(0.0)
        res = np.zeros((self.n_obs, 2))
        jac = np.zeros((self.n_obs, 2, 9)) if want_jacobian else None
        check(lib().sfm_ba_evaluate(self._h, ctypes.byref(cost), ptr(res), ptr(jac)), "sfm_ba_evaluate")
        return cost.value, res, jac

    def bench_jacobian(self, reps: int) -> float:
        ms = c_double(0.0)
        check(lib().sfm_ba_bench_jacobian(self._h, reps, ctypes.byref(ms)), "sfm_ba_bench_jacobian")
        return ms.value

    def set_profiling(self, on: bool) -> None:
        check(lib().sfm_ba_set_profiling(self._h, 1 if on else 0), "sfm_ba_set_profiling")

    def phase_times(self) -> dict:
        buf = np.zeros(2 * len(PHASES))
        check(lib().sfm_ba_phase_times(self._h, ptr(buf)), "sfm_ba_phase_times")
        return {p: {"ms": float(buf[i]), "count": int(buf[len(PHASES) + i])} for i, p in enumerate(PHASES)}

    def sync(self) -> None:
        check(lib().sfm_ba_sync(self._h), "sfm_ba_sync")


def solve(uv, cam_idx, pt_idx, K9, rot, t, X, options: BAOptions | None = None, mode: int = STRUCT_AND_POSE,
          trace_cap: int = 128):
    """One-shot drop-in solve (sfm_ba_solve): rot, t, X are updated in place."""
    for name, a in (("rot", rot), ("t", t), ("X", X)):
        if not (isinstance(a, np.ndarray) and a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]):
            raise TypeError(f"{name} must be a C-contiguous float64 array (updated in place)")
    uv, K9 = _f64(uv), _f64(K9)
    cam_idx, pt_idx = _i32(cam_idx), _i32(pt_idx)
    _check_shapes(uv, cam_idx, pt_idx, K9, rot, t, X)
    opts = options if options is not None else default_options()
    sm = BASummary()
    tr = (BAIteration * trace_cap)()
    tl = c_int32(0)
    check(lib().sfm_ba_solve(ctypes.byref(opts), mode, int(uv.shape[0]), ptr(uv), ptr(cam_idx), ptr(pt_idx),
                             int(rot.shape[0]), ptr(K9), ptr(rot), ptr(t), int(X.shape[0]), ptr(X),
                             ctypes.byref(sm), tr, trace_cap, ctypes.byref(tl)), "sfm_ba_solve")
    return sm, [tr[i].as_dict() for i in range(tl.value)]


def dense_spd_solve(A, b, device: int = 0, reps: int = 1):
    """Testing hook: y = A^-1 b with the device Cholesky used for the reduced
    camera system.  Returns (y, ms_per_solve, chol_fail)."""
    A = _f64(A)
    b = _f64(b)
    n = int(A.shape[0])
    y = np.zeros(n)
    ms = c_double(0.0)
    fl = c_int32(0)
    check(lib().sfm_dense_spd_solve(device, n, ptr(A), ptr(b), ptr(y), reps, ctypes.byref(ms), ctypes.byref(fl)),
          "sfm_dense_spd_solve")
    return y, ms.value, fl.value
