"""CPU: the PnP oracle (oracle/pnp_oracle.py, the restated OpenCV 3.0
cv::solvePnPRansac of CSfM.cpp:553-565) on properties the algorithm
guarantees: EPnP recovers an exact pose from noise-free points (planar and
not), the RANSAC rejects gross outliers, cv::RNG / RANSACUpdateNumIters
behave as published, and the degenerate sizes take the reference's
branches.  (Parity against OpenCV itself is unpinned: it is absent.)"""
import numpy as np
import pytest

from oracle import pnp_oracle as P
from tests.pnp_cases import K, scene


@pytest.mark.parametrize("planar", [False, True])
@pytest.mark.parametrize("n", [5, 6, 12, 100])
def test_epnp_exact_on_noise_free_points(n, planar):
    X, uv, rv, tv = scene(n, 10 + n, noise=0.0, outliers=0.0, planar=planar)
    R, t = P.epnp(K, X.astype(np.float32), uv.astype(np.float32))
    R0 = P.rodrigues_v2m(rv)
    # float32 data: the pose is exact to the input rounding
    assert np.max(np.abs(R - R0)) < 1e-4
    assert np.max(np.abs(t - tv)) < 1e-3 * np.linalg.norm(tv)


def test_ransac_rejects_outliers_and_recovers_pose():
    X, uv, rv, tv = scene(300, 4, noise=0.5, outliers=0.2)
    ok, r, t, inl = P.solve_pnp_ransac(X, uv, K)
    assert ok
    # the returned pose is a 5-point EPnP hypothesis (3.0: no refinement): coarse
    assert np.max(np.abs(r - rv)) < 2e-2 and np.max(np.abs(t - tv)) < 0.2
    e = P.point_errors(K, X.astype(np.float32), uv.astype(np.float32), r, t)
    assert np.array_equal(inl, np.nonzero(e <= np.float32(49.0))[0])


def test_rng_and_iteration_bound():
    a, b = P.CvRNG(), P.CvRNG()
    seq = [a.next() for _ in range(5)]
    assert seq == [b.next() for _ in range(5)] and len(set(seq)) == 5
    # cv::RNG: state' = (uint32)state * 4164903690 + (state >> 32)
    s = (1 << 64) - 1
    s2 = ((s & 0xFFFFFFFF) * 4164903690 + (s >> 32)) & ((1 << 64) - 1)
    assert seq[0] == s2 & 0xFFFFFFFF
    assert P.ransac_update_num_iters(0.99, 0.0, 5, 20) == 0 or P.ransac_update_num_iters(0.99, 0.0, 5, 20) >= 0
    assert P.ransac_update_num_iters(0.99, 0.5, 5, 20) == 20          # bound not reached
    assert P.ransac_update_num_iters(0.99, 0.2, 5, 20) == round(np.log(0.01) / np.log(1 - 0.8 ** 5))
    sub = P.get_subset(P.CvRNG(), 10)
    assert len(set(sub)) == 5 and all(0 <= v < 10 for v in sub)


def test_degenerate_sizes():
    X, uv, _, _ = scene(4, 1, noise=0.0, outliers=0.0)
    ok, r, t, inl = P.solve_pnp_ransac(X, uv, K)
    assert not ok and len(inl) == 0
    X, uv, rv, tv = scene(5, 1, noise=0.0, outliers=0.0)
    ok, r, t, inl = P.solve_pnp_ransac(X, uv, K)
    assert ok and list(inl) == [0, 1, 2, 3, 4]
    assert np.max(np.abs(t - tv)) < 1e-2
