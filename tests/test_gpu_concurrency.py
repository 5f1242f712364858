"""GPU: the persistent grids of the solve (k_chol_fused, k_backsolve) beside
other device work.

Both kernels hand tiles between their workgroups and used to take their
roles from the workgroup index, which needs the whole grid resident at once.
Roles now go by start order (the first workgroup to run walks the diagonal /
takes the first back-substitution row), so a grid that only partly fits
beside other streams' kernels runs slower but finishes.  Checked here by
running work on other streams while C3 solves run:

* BRISK detection and the frame-resident matcher in two threads (each handle
  has its own stream; ctypes releases the GIL), a C3 solve in the main
  thread: it must succeed, equal the same solve run alone bitwise, and
  match the oracle (/root/reference/CTracker.cpp:670-702);
* two C3 solves at once on two handles (two persistent grids competing for
  the CUs): both must equal the solo solve bitwise.
"""
import threading

import numpy as np
import pytest

import sfm_amd
from sfm_amd import scene
from oracle import ffi as O

pytestmark = pytest.mark.gpu


def _solo(s):
    with sfm_amd.BundleAdjuster() as ba:
        ba.set_problem(s.uv, s.cam_idx, s.pt_idx, s.K, s.rot, s.t, s.X)
        sm, tr = ba.solve()
        return sm, tr, ba.parameters()


def _rel(a, b, floor=1e-3):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b)) / np.maximum(np.abs(np.asarray(b)), floor)))


def _background(stop, errors):
    """BRISK + matcher calls on their own streams until `stop` is set."""
    from sfm_amd import brisk
    from sfm_amd.matcher import FeatureMatcher
    from sfm_amd.video import SyntheticVideo

    def brisk_loop():
        try:
            v = SyntheticVideo(speed=2.0)
            frames = [v.frame(k) for k in range(3)]
            k = 0
            while not stop.is_set():
                brisk.detect(frames[k % 3])
                k += 1
        except Exception as e:  # reported by the test
            errors.append(e)

    def match_loop():
        try:
            rng = np.random.default_rng(3)
            n = 4000
            d = rng.integers(0, 256, (n, 64), dtype=np.uint8)
            p = rng.uniform(0, [1280, 720], (n, 2))
            idx = np.arange(n, dtype=np.int32)
            with FeatureMatcher(64) as m:
                m.push_frame(p, d)
                while not stop.is_set():
                    m.push_frame(p + 1.0, d)
                    m.match_subset(idx, idx)
        except Exception as e:
            errors.append(e)

    th = [threading.Thread(target=brisk_loop), threading.Thread(target=match_loop)]
    for t in th:
        t.start()
    return th


@pytest.mark.timeout(300)
def test_c3_solve_beside_brisk_and_matcher_streams():
    s = scene.config("C3")
    sm0, tr0, p0 = _solo(s)
    stop, errors = threading.Event(), []
    th = _background(stop, errors)
    try:
        got = []
        for _ in range(3):  # several solves, so some overlap the background work
            r, t, X = s.copy_params()
            sm, tr = sfm_amd.solve(s.uv, s.cam_idx, s.pt_idx, s.K, r, t, X)
            got.append((sm, tr, (r, t, X)))
    finally:
        stop.set()
        for t_ in th:
            t_.join()
    assert not errors, errors
    for sm, tr, p in got:
        assert tr == tr0 and sm.final_cost == sm0.final_cost
        for a, b in zip(p, p0):
            assert np.array_equal(a, b)
    # and the oracle (8 threads: bitwise its serial solve)
    r, t, X = s.copy_params()
    sm_o, tr_o = O.solve(s.uv, s.cam_idx, s.pt_idx, s.K, r, t, X, threads=8)
    sm, tr, (rg, tg, Xg) = got[-1]
    assert sm.num_iterations == sm_o["num_iterations"]
    assert [it["step_is_successful"] for it in tr] == [it["step_is_successful"] for it in tr_o]
    assert abs(sm.final_cost - sm_o["final_cost"]) <= 1e-9 * sm_o["final_cost"]
    assert _rel(Xg, X) < 1e-6 and _rel(tg, t) < 1e-6 and _rel(rg, r) < 1e-6


@pytest.mark.timeout(300)
def test_two_concurrent_c3_solves():
    s = scene.config("C3")
    sm0, tr0, p0 = _solo(s)
    out, errors = [None, None], []

    def run(i):
        try:
            with sfm_amd.BundleAdjuster() as ba:
                ba.set_problem(s.uv, s.cam_idx, s.pt_idx, s.K, s.rot, s.t, s.X)
                res = []
                for _ in range(3):
                    ba.reset()
                    sm, tr = ba.solve()
                    res.append((sm, tr, ba.parameters()))
                out[i] = res
        except Exception as e:
            errors.append(e)

    th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    for res in out:
        for sm, tr, p in res:
            assert tr == tr0 and sm.final_cost == sm0.final_cost
            for a, b in zip(p, p0):
                assert np.array_equal(a, b)
