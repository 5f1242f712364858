"""One-shot sfm_ba_solve at C3, four times, through the C ABI (SFM_TIMING=1
adds the host phase breakdown of set_problem and the solve on stderr):
  SFM_TIMING=1 python tools/c3_oneshot_timing.py"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from sfm_amd import ba as B  # noqa: E402
from sfm_amd import scene as S  # noqa: E402

sc = S.config("C3")
L = B.lib()
opts, sm = B.default_options(), B.BASummary()
tr, tl = (B.BAIteration * 128)(), ctypes.c_int32(0)
r, t, X = sc.rot.copy(), sc.t.copy(), sc.X.copy()
uv, ci, pi, K = B._f64(sc.uv), B._i32(sc.cam_idx), B._i32(sc.pt_idx), B._f64(sc.K)
args = (ctypes.byref(opts), B.STRUCT_AND_POSE, int(uv.shape[0]), B.ptr(uv), B.ptr(ci), B.ptr(pi), int(r.shape[0]),
        B.ptr(K), B.ptr(r), B.ptr(t), int(X.shape[0]), B.ptr(X), ctypes.byref(sm), tr, 128, ctypes.byref(tl))
for k in range(4):
    r[:] = sc.rot; t[:] = sc.t; X[:] = sc.X
    t0 = time.perf_counter()
    assert L.sfm_ba_solve(*args) == 0
    print("one-shot ms", round((time.perf_counter() - t0) * 1e3, 3), "iterations", sm.num_iterations, flush=True)
