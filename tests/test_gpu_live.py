"""GPU: the live tracking path (sfm_amd.live.LiveSfM; CSfM::tracking +
CSfM::mapping, /root/reference/CSfM.cpp:109-261, 500-692) driven through
the device matcher (frame-to-frame subset overload and the (0, 7) window),
PnP, the device map store and the BA, on synthetic detector output.

* every keyframe's BA is re-solved by the oracle on the exact problem the
  driver gathered through the device map store (same LM path, parameters
  1e-6 relative, cost 1e-9);
* the map store's associations equal the keyframes' own (what
  getPointsInFrame returns is what the driver recorded);
* keypoint -> map point associations hit the right landmark, and the
  adjusted keyframe poses and map points match the stream's ground truth
  after a similarity alignment (the reference's BA holds no block constant,
  CTracker.cpp:670-702, so the gauge floats)."""
import json
import os

import numpy as np
import pytest

import lm_cases as L
from oracle import ffi as O
from sfm_amd.live import KeypointStream, LiveSfM, _project
from sfm_amd.mapping import _rodrigues

pytestmark = pytest.mark.gpu
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")


def _residuals(uv, cam_idx, pt_idx, K, rot, t, X):
    return O.residuals_jacobians(uv, cam_idx, pt_idx, K, rot, t, X, jacobian=False)[0]


def _rel(a, b, floor=1e-3):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b)) / np.maximum(np.abs(np.asarray(b)), floor)))


def _umeyama(A, B):
    """s, R, t minimising |s R A + t - B| (rows are points)."""
    ma, mb = A.mean(0), B.mean(0)
    a, b = A - ma, B - mb
    U, S, Vt = np.linalg.svd(b.T @ a / len(A))
    D = np.eye(3)
    D[2, 2] = np.sign(np.linalg.det(U @ Vt))
    R = U @ D @ Vt
    s = np.trace(np.diag(S) @ D) / (a ** 2).sum(1).mean()
    return s, R, mb - s * R @ ma


@pytest.fixture(scope="module")
def run80():
    s = LiveSfM(KeypointStream())
    s.run(80)
    yield s
    s.close()


def test_live_path_tracks_every_frame_and_grows_the_map(run80):
    s = run80
    assert s.lost == 0
    assert s.stats["tracked"] == 80 - 5 - 1        # every frame after the initial pair
    assert [f.no for f in s.kfs][:3] == [0, 5, 15]
    assert len(s.kfs) >= 7
    n_pts, n_obs, n_rows = s.map.size()
    assert n_pts >= 1500 and n_obs >= 3 * n_pts
    assert s.stats["map_matches"] > 0              # the (0, 7) window re-finds map points
    assert len(s.ba_log) == len(s.kfs) - 1


class _BothFinds(LiveSfM):
    """findMapPointsInCurrentFrame both ways on every tracked frame's state:
    the fused device call (sfm_map_match_frame) and the composed map /
    matcher calls; the composed result is the one kept."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.cmp = []

    def _find_map_points(self, cur):
        base = cur.pt3d.copy()
        self.fused_find = True
        super()._find_map_points(cur)
        fused = cur.pt3d.copy()
        cur.pt3d[:] = base
        self.fused_find = False
        super()._find_map_points(cur)
        self.cmp.append((cur.no, fused, cur.pt3d.copy()))


def test_fused_find_map_points_equals_the_composed_calls():
    s = _BothFinds(KeypointStream())
    try:
        s.run(45)
        assert len(s.cmp) >= 35
        found = 0
        for no, fused, comp in s.cmp:
            assert np.array_equal(fused, comp), f"frame {no}: {np.flatnonzero(fused != comp)[:10]}"
            found += int((comp >= 0).sum())
        assert found > 0
    finally:
        s.close()


def test_fused_tracking_equals_the_composed_calls():
    """sfm_track_pnp (matchFeatures + getPointsAtIdx + solvePnPRansac in one
    device call) and the mapping's matches on the matcher's keyframe store
    (sfm_matcher_match_keyframes) against the calls they replace: the same
    keyframes, poses, associations, statistics and map, bitwise."""
    runs = []
    for fused in (True, False):
        s = LiveSfM(KeypointStream())
        s.fused_track = fused
        s.resident_kf = fused
        try:
            s.run(60)
            runs.append(([f.no for f in s.kfs], [(f.rot.copy(), f.t.copy(), f.pt3d.copy()) for f in s.kfs],
                         dict(s.stats), s.map.size(), s.prev.rot.copy(), s.prev.t.copy(), s.prev.pt3d.copy()))
        finally:
            s.close()
    a, b = runs
    assert a[0] == b[0] and len(a[0]) >= 3
    for (r1, t1, p1), (r2, t2, p2) in zip(a[1], b[1]):
        assert np.array_equal(r1, r2) and np.array_equal(t1, t2) and np.array_equal(p1, p2)
    assert a[2] == b[2] and a[2]["tracked"] > 40
    assert a[3] == b[3]
    for x, y in zip(a[4:], b[4:]):
        assert np.array_equal(x, y)


def test_every_keyframe_ba_matches_oracle(run80):
    for rec in run80.ba_log:
        r, t, X = rec["rot"].copy(), rec["t"].copy(), rec["X"].copy()
        sm_o, tr_o = O.solve(rec["uv"], rec["cam_idx"], rec["pt_idx"], rec["K"], r, t, X)
        sm_g, tr_g = rec["summary"], rec["trace"]
        assert sm_g.termination_type == sm_o["termination_type"]
        assert sm_g.num_iterations == sm_o["num_iterations"]
        assert [x["step_is_successful"] for x in tr_g] == [x["step_is_successful"] for x in tr_o]
        assert abs(sm_g.final_cost - sm_o["final_cost"]) <= 1e-9 * max(sm_o["final_cost"], 1e-300)
        assert _rel(rec["X_out"], X) < 1e-6
        assert _rel(rec["t_out"], t) < 1e-6
        assert _rel(rec["rot_out"], r, floor=1e-2) < 1e-6


def test_map_store_associations_equal_the_keyframes(run80):
    s = run80
    for kf in s.kfs:
        p3, p2 = s.map.getPointsInFrame(kf.no)
        assert len(p3) == len(p2) == kf.n_matched()
        assert (kf.pt3d[p2] == p3).all()
    cov = s.map.getPointsInFrames([f.no for f in s.kfs])
    assert cov.tolist() == list(range(s.map.size()[0]))   # every point has a keyframe observation


def test_associations_and_geometry_match_ground_truth(run80):
    s = run80
    st = s.stream
    # landmark of every keyframe observation of every map point
    votes = {}
    for kf in s.kfs:
        lid = st.frame(kf.no)[2]
        for j in np.flatnonzero(kf.pt3d >= 0):
            votes.setdefault(int(kf.pt3d[j]), []).append(int(lid[j]))
    good = sum(1 for v in votes.values() if len(set(v)) == 1 and v[0] >= 0)
    assert good >= 0.97 * len(votes)
    # similarity alignment on the map points (the keyframe path is nearly a
    # line, so centres alone leave the roll about it undetermined)
    ids = np.array([k for k, v in votes.items() if len(set(v)) == 1 and v[0] >= 0])
    lm = np.array([votes[k][0] for k in ids])
    X = s.map.getPointsAtIdx(ids)
    sc, R, t = _umeyama(X, st.L[lm])
    d = np.linalg.norm((sc * X @ R.T + t) - st.L[lm], axis=1)
    C = np.array([-_rodrigues(f.rot).T @ f.t for f in s.kfs])
    Cg = np.array([-_rodrigues(st.pose(f.no)[0]).T @ st.pose(f.no)[1] for f in s.kfs])
    err = np.linalg.norm((sc * C @ R.T + t) - Cg, axis=1)
    print("point error median / p90", np.median(d), np.percentile(d, 90), "centre error max", err.max(), "scale", sc)
    # depth 8-14 units from keyframe baselines of 0.2-2 units at 0.3 px
    # (measured on MI355X: median 0.059, centres 0.035-0.037 -- a common
    # offset, ~0.3% of the depth, from the short-baseline triangulations)
    assert np.median(d) < 0.1
    assert err.max() < 0.06
    # keyframe-to-keyframe motion, free of that offset: within 5% of the
    # ground truth's 0.2-unit steps
    dm = np.linalg.norm(np.diff(sc * C @ R.T, axis=0), axis=1)
    dg = np.linalg.norm(np.diff(Cg, axis=0), axis=1)
    assert np.max(np.abs(dm - dg) / dg) < 0.05


@pytest.fixture(scope="module")
def run_brisk():
    from sfm_amd.live import BriskVideoStream
    st = BriskVideoStream()
    s = LiveSfM(st)
    s.run(40)
    yield s
    s.close()


def test_live_path_on_device_brisk_detections(run_brisk):
    """The live loop fed by the device BRISK (row T8) on the rendered video:
    every frame tracked, keyframes every 10 frames, each keyframe BA equal to
    the oracle's, and the adjusted map + poses reproducing the video's true
    image motion."""
    s = run_brisk
    st = s.stream
    assert s.lost == 0 and s.stats["tracked"] == 40 - 5 - 1
    assert [f.no for f in s.kfs][:4] == [0, 5, 15, 25]
    assert s.map.size()[0] > 1000
    rng = np.random.default_rng(0)
    table = []
    for k, rec in enumerate(s.ba_log):
        r, t, X = rec["rot"].copy(), rec["t"].copy(), rec["X"].copy()
        sm_o, _ = O.solve(rec["uv"], rec["cam_idx"], rec["pt_idx"], rec["K"], r, t, X)
        sc_ = type("S", (), dict(uv=rec["uv"], cam_idx=rec["cam_idx"], pt_idx=rec["pt_idx"], K=rec["K"]))
        # the rounding sensitivity of this problem: the oracle again from the
        # same start perturbed by ~2 ulp, three times, the largest spread (the
        # gauge of the whole map is free, as in CSfM::bundleAdjustment, and
        # the BRISK scale-space keypoints are clustered, so some keyframe BAs
        # amplify rounding far more than the synthetic scenes' 1e-9; one
        # perturbation under-reads a chaotic run by 10x, measured)
        sens = sens_x = sens_res = sens_al = 0.0
        for _ in range(3):
            rp, tp, Xp = (a * (1 + 4.4e-16 * rng.choice([-1.0, 1.0], a.shape)) for a in
                          (rec["rot"], rec["t"], rec["X"]))
            sm_p, _ = O.solve(rec["uv"], rec["cam_idx"], rec["pt_idx"], rec["K"], rp, tp, Xp)
            sens = max(sens, abs(sm_p["final_cost"] - sm_o["final_cost"]) / sm_o["final_cost"])
            sens_x = max(sens_x, _rel(Xp, X))
            pr, pa = L.gauge_invariant_diff(_residuals, sc_, (rp, tp, Xp), (r, t, X), extent=True)
            sens_res, sens_al = max(sens_res, pr), max(sens_al, pa)
        d = abs(rec["summary"].final_cost - sm_o["final_cost"]) / sm_o["final_cost"]
        dx = _rel(rec["X_out"], X)
        # gauge-invariant distances of the two solutions (SURVEY.md §7 hard
        # part 2): per-observation residuals (px) and camera centres + points
        # after a Sim(3) alignment, over the scene radius
        res, al = L.gauge_invariant_diff(_residuals, sc_, (rec["rot_out"], rec["t_out"], rec["X_out"]), (r, t, X),
                                         extent=True)
        row = dict(ba=k, obs=len(rec["uv"]), iterations=sm_o["num_iterations"],
                   gpu_iterations=rec["summary"].num_iterations,
                   termination=sm_o["termination_type"], cost_rel=d, cost_sensitivity=sens, X_rel=dx,
                   X_sensitivity=sens_x, residual_max_px=res, residual_sensitivity_px=sens_res,
                   sim3_aligned_rel=al, sim3_aligned_sensitivity=sens_al)
        if sm_o["termination_type"] == 1:
            # the oracle in the device solver's association of the reduced
            # matrix's diagonal blocks (oracle order=1: the same arithmetic,
            # U_c summed first, then + D^2, then the outer products)
            r1, t1, X1 = rec["rot"].copy(), rec["t"].copy(), rec["X"].copy()
            sm_1, _ = O.solve(rec["uv"], rec["cam_idx"], rec["pt_idx"], rec["K"], r1, t1, X1, order=1)
            res1, al1 = L.gauge_invariant_diff(_residuals, sc_, (rec["rot_out"], rec["t_out"], rec["X_out"]),
                                               (r1, t1, X1), extent=True)
            row.update(order1_iterations=sm_1["num_iterations"],
                       order1_cost_rel=abs(rec["summary"].final_cost - sm_1["final_cost"]) / sm_1["final_cost"],
                       order1_X_rel=_rel(rec["X_out"], X1), order1_residual_max_px=res1, order1_sim3_aligned_rel=al1)
        table.append(row)
        print(f"keyframe BA {k}: {len(rec['uv'])} obs, iterations {sm_o['num_iterations']} "
              f"({sm_o['termination_type']}), cost rel diff {d:.2e} (oracle rounding sensitivity {sens:.2e}), "
              f"X rel diff {dx:.2e} (sensitivity {sens_x:.2e}), residuals {res:.1e} px, Sim(3)-aligned {al:.1e} "
              f"(sensitivity {sens_res:.1e} px, {sens_al:.1e})"
              + ("" if "order1_X_rel" not in row else
                 f"; vs the oracle in the device association: cost {row['order1_cost_rel']:.2e}, X "
                 f"{row['order1_X_rel']:.2e}, residuals {row['order1_residual_max_px']:.1e} px, aligned "
                 f"{row['order1_sim3_aligned_rel']:.1e}"))
    # the per-keyframe table (committed as profiles/r05_live_brisk_ba_parity.json)
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "live_brisk_ba_parity.json"), "w") as f:
        json.dump(table, f, indent=1)
    # Converged runs (Ceres' function tolerance): the north-star tolerance
    # flat -- cost, raw X and the Sim(3)-aligned distance (over the scene
    # radius) within 1e-6 relative, residuals within 1e-6 px (measured round
    # 5: X 6.9e-7, aligned 8.4e-11, residuals 3.1e-9 px at most).
    # A run stopped by the 50-iteration cap (NO_CONVERGENCE, termination 1)
    # ends at an arbitrary point of a slow drift along the free 7-DoF gauge,
    # where the reference algorithm itself moves by its own rounding: 2 ulp
    # of start perturbation move the oracle's end point (BA 3 of this stream)
    # by 2e-3 in raw X and 4e-4 of the radius after alignment.  There the
    # GPU's end point must lie within TWICE that spread of the oracle's in
    # every quantity (cost also <= 1e-6), both in Ceres' summation order and
    # in the device's association of the diagonal blocks (oracle order=1).
    for row in table:
        assert row["gpu_iterations"] == row["iterations"], row
        if row["termination"] != 1:
            assert row["cost_rel"] <= 1e-6, row
            assert row["X_rel"] <= 1e-6, row
            assert row["sim3_aligned_rel"] <= 1e-6, row
            assert row["residual_max_px"] <= 1e-6, row
            continue
        assert row["order1_iterations"] == row["iterations"], row
        for pre in ("", "order1_"):
            assert row[pre + "cost_rel"] <= min(1e-6, max(1e-9, 2 * row["cost_sensitivity"])), row
            assert row[pre + "X_rel"] <= max(1e-6, 2 * row["X_sensitivity"]), row
            assert row[pre + "sim3_aligned_rel"] <= max(1e-9, 2 * row["sim3_aligned_sensitivity"]), row
            assert row[pre + "residual_max_px"] <= max(1e-8, 2 * row["residual_sensitivity_px"]), row
    # The scene is one textured plane at depth 10 seen over 0.1-0.3-unit
    # baselines, where a lateral translation and a small rotation move the
    # image almost alike: the camera centres alone are weakly determined
    # (measured: one keyframe of the five trades 0.08 units of translation
    # for rotation, identically in the oracle's solve).  What the images
    # determine is the image motion: the map points of keyframe 0 projected
    # with each keyframe's adjusted pose must land where the video's true
    # similarity carries their keyframe-0 keypoints.
    kf0 = s.kfs[0]
    have = np.flatnonzero(kf0.pt3d >= 0)
    X = s.map.getPointsAtIdx(kf0.pt3d[have].astype(np.int32))
    for f in s.kfs[1:]:
        uv, z = _project(s.K, f.rot, f.t, X)
        truth = st.video.map_points(kf0.no, f.no, kf0.pts[have])
        inside = (z > 0) & (truth[:, 0] > 0) & (truth[:, 0] < st.video.w) & (truth[:, 1] > 0) & \
            (truth[:, 1] < st.video.h)
        e = np.linalg.norm(uv[inside] - truth[inside], axis=1)
        print(f"brisk live: keyframe {f.no}: {inside.sum()} points of keyframe 0, image motion error median "
              f"{np.median(e):.3f} px, p90 {np.percentile(e, 90):.3f} px")
        assert np.median(e) < 1.0 and np.percentile(e, 90) < 3.0
