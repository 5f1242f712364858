#!/usr/bin/env python3
"""Benchmark: landmark-sharded bundle adjustment on MI355X (BASELINE.json metric
"BA iterations/sec + residual-evals/sec (cams x pts x obs); 1/2/4/8 GPU").

A step is one complete BA solve -- CTracker::bundleAdjustmentStructAndPose
(/root/reference/CTracker.cpp:670-702) with the reference's Ceres options --
over a synthetic scene resident in HBM: parameters are reset on the device
(inside the timed region), then the LM loop runs to Ceres' own termination.

Workload per GPU: BASELINE config C3 (500 cameras, 200k points, 2M
observations, fp64).  With N GPUs the scene has N x 200k points sharded by
landmark (weak scaling; cameras replicated, RCCL all-reduce of the reduced
camera system every LM iteration).  `value` = residual-only evaluations x
observations (whole job) per second (the Jacobian evaluations,
which also evaluate the residual vector, are counted separately and reported
beside it as `jacobian_evals_per_s`); LM iterations/s is reported beside it.

Also reported: the one-shot C3 wall-clock (host arrays in, problem setup +
solve + download, sfm_ba_solve -- the reference rebuilds its ceres::Problem
per call, CTracker.cpp:672), a measured STREAM-copy bandwidth next to the
8 TB/s peak, the frame-resident matcher (CTracker::matchFeatures, 2k x 2k
64-B descriptors), the C5 tracker, the keyframe-sized solve, the per-frame
PnP and the C5 pipeline end to end (KLT + PnP + triangulation + BA after
every keyframe).

Launch:  python bench.py [--gpus N --steps K --warmup W]
   N>1:  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
F64_MFMA_PEAK_TFS = 78.6   # MI355X fp64 matrix spec
CAMS, PTS_PER_GPU, VIEWS = 500, 200_000, 10
C4 = (2000, 1_000_000)     # BASELINE config 4 (cams, points)
SEED = 0x5F3D2017 + 3      # config C3 (sfm_amd.scene.config); C4 is SEED + 1


def jacobian_bytes(n_obs: int, n_cams: int, n_pts: int) -> int:
    # record-writing variant (evaluate API): per observation point index 4 +
    # uv 16 + record 160 (r 16 + J 144) (k_jacobian); per
    # camera: pose 48 + K 40; per point: X 24.
    return 180 * n_obs + 88 * n_cams + 24 * n_pts


def jacobian_bytes_solve(n_obs_pad: int, n_cams: int, n_pts: int) -> int:
    # the solve's record-free pass: per (padded) observation slot point index
    # 4 + uv 16 streamed; X read once per point (24 B); per camera pose 48 +
    # K 40; out: 27 U_c / b_c partial sums (216 B) per 64-observation chunk.
    return 20 * n_obs_pad + 24 * n_pts + 88 * n_cams + 216 * (n_obs_pad // 64)


def jacobian_flops_solve(n_obs: int) -> float:
    # per observation: rotation applied (R from the per-camera
    # constants: 15), projection + residual (~12), the 2x9 Jacobian from the
    # rotated point (~60), Jacobi scaling (18), U_c (21 entries x 2 rows x 2)
    # + b_c (6 x 2 x 2) partial products (108), cost (4): ~217 fp64 flops.
    return 217.0 * n_obs


F64_VALU_PEAK_TFS = 78.6   # MI355X fp64 vector (MI355X_MICROARCH.md)


def cholesky_flops(n: int) -> float:
    return n ** 3 / 3.0


def host_info() -> dict:
    """nproc / CPU model of the machine running the CPU legs (BASELINE.md
    timing protocol)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return {"nproc": avail, "cpu_count": os.cpu_count(), "model": model}


def cpu_threads() -> int:
    """Threads for the all-cores CPU figure: the cores this process may use,
    capped at the box's CPU share (16 per GPU on the MI355X pool)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return max(1, min(16, avail))


def cpu_baseline(scene, reps: int = 3) -> dict:
    """Oracle (the C++ restatement of the reference's Ceres path) on the same
    C3 scene: BASELINE.md protocol -- one warm-up, then the median of `reps`
    complete solves (problem setup included, as the reference rebuilds its
    ceres::Problem per call), single-threaded (the reference's Ceres default
    num_threads = 1); the all-cores OpenMP figure is timed beside it."""
    from oracle import ffi as O

    def run(threads):
        walls = []
        sm = None
        for k in range(reps + 1):
            r, t, X = scene.copy_params()
            t0 = time.perf_counter()
            sm, _ = O.solve(scene.uv, scene.cam_idx, scene.pt_idx, scene.K, r, t, X, threads=threads)
            if k > 0:
                walls.append(time.perf_counter() - t0)
        return float(np.median(walls)), walls, sm

    wall, walls, sm = run(1)
    res_only = sm["num_residual_evaluations"] - sm["num_jacobian_evaluations"]
    nthr = cpu_threads()
    wall_mt, walls_mt, _ = run(nthr)
    return {
        "value": scene.n_obs * res_only / wall,
        "unit": "residual-evals/s (obs x residual-only evaluations)",
        "cores": 1,
        "kind": "port",
        "sample": (f"complete C3 solves ({scene.n_cams} cams / {scene.n_pts} pts / {scene.n_obs} obs, setup "
                   f"included): {sm['num_iterations']} LM iterations, {res_only} residual-only + "
                   f"{sm['num_jacobian_evaluations']} Jacobian evaluations; median of {reps} after 1 warm-up: "
                   f"{wall:.2f} s (oracle/ba_oracle.cpp, Ceres-1.12-equivalent restatement, 1 thread)"),
        "lm_iterations_per_s": sm["num_iterations"] / wall,
        "solve_s": wall,
        "solve_s_runs": walls,
        "multi_thread": {"threads": nthr, "host_threads_visible": host_info()["nproc"],
                         "solve_s": wall_mt, "solve_s_runs": walls_mt,
                         "value": scene.n_obs * res_only / wall_mt,
                         "lm_iterations_per_s": sm["num_iterations"] / wall_mt,
                         "note": (f"OpenMP oracle (Jacobian pass, Schur elimination, dense LLT in parallel) on "
                                  f"{nthr} threads: the box's CPU share per GPU is 16 threads, although the host "
                                  f"shows more")},
        "host": host_info(),
    }


def tracker_leg(device: int, steps: int, cpu: bool) -> dict:
    """Config C5 tracker leg (SURVEY.md §8a rows T7 + T6): one step = one
    1280x720 grey frame through the reference's optical-flow loop:
    push_frame (upload + pyramid + Scharr derivatives, resident in HBM),
    CTracker::detectFeaturesOpticalFlow (goodFeaturesToTrack 500 / 0.05 / 10
    + cornerSubPix 5x5 / 20 / 0.03) and CTracker::computeOpticalFlow of the
    previous frame's corners into this frame's (calcOpticalFlowPyrLK 21x21 /
    4 levels / <= 20 its + nearest-corner association).  Frames cycle over 3
    rendered synthetic frames."""
    from sfm_amd import klt
    from sfm_amd.video import SyntheticVideo
    v = SyntheticVideo()
    frames = [v.frame(k) for k in range(3)]
    tr = klt.KLTTracker(v.w, v.h, device=device)
    tr.push_frame(frames[0])
    prev = tr.detect_features()
    ph = {"pyramid": 0.0, "detect": 0.0, "lk": 0.0, "associate": 0.0}
    warm = 5
    matches = corners = 0
    for it in range(steps + warm):
        if it == warm:
            t0 = time.perf_counter()
            ph = {k: 0.0 for k in ph}
        k = (it + 1) % 3
        tr.push_frame(frames[k])
        cur = tr.detect_features()
        pi, _ = tr.compute_optical_flow(prev, cur)
        prev = cur
        matches, corners = len(pi), len(cur)
        for a, b in tr.phase_times().items():
            ph[a] += b
        ph["detect"] += tr.detect_time_ms()
    wall = (time.perf_counter() - t0) / steps
    out = {"workload": "C5 tracker: 1280x720 grey synthetic video, per frame push_frame + detectFeaturesOpticalFlow "
                       "(GFTT 500/0.05/10 + cornerSubPix) + computeOpticalFlow (calcOpticalFlowPyrLK 21x21, 4 levels, "
                       "<=20 its, eps 0.03) + association",
           "frames_per_s": 1.0 / wall, "ms_per_frame": wall * 1e3, "corners_per_frame": corners,
           "matches_per_frame": matches, "levels": tr.num_levels,
           "device_ms_per_frame": {a: round(b / steps, 4) for a, b in ph.items()},
           "cpu_baseline": None}
    tr.close()
    if cpu:
        from oracle import ffi as O
        reps = 10
        t0 = time.perf_counter()
        c_prev = O.detect_features_of(frames[0])
        for r in range(reps):
            k = (r + 1) % 3
            c = O.detect_features_of(frames[k])
            nx, st = O.calc_optical_flow_pyr_lk(frames[(k - 1) % 3], frames[k], c_prev)
            O.klt_associate(c_prev, nx, st, c)
            c_prev = c
        cw = (time.perf_counter() - t0) / reps
        out["cpu_baseline"] = {"frames_per_s": 1.0 / cw, "ms_per_frame": cw * 1e3, "cores": 1, "kind": "port",
                               "sample": f"{reps} frames of the same work (detection + both pyramids + LK + "
                                         "association) on oracle/gftt_oracle.cpp + klt_oracle.cpp, 1 thread"}
    return out


def incremental_ba_leg(device: int, cpu: bool) -> dict:
    """Keyframe-sized solves (the incremental BA CSfM::bundleAdjustment runs
    after each new keyframe, CSfM.cpp:259/970): BASELINE config C1 (20 cams /
    2k points / 20k obs), a complete LM solve per call, problem upload
    included (sfm_ba_solve one-shot, as the drop-in is called)."""
    import sfm_amd
    from sfm_amd import scene as S
    sc = S.config("C1")
    reps = 20
    for it in range(reps + 3):
        if it == 3:
            t0 = time.perf_counter()
        r, t, X = sc.copy_params()
        sm, _ = sfm_amd.solve(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, r, t, X)
    wall = (time.perf_counter() - t0) / reps
    # the same one-shot call through the C ABI alone (arguments prepared once,
    # the parameters reset outside the clock): the latency a C++ caller of the
    # drop-in sees, without the Python mirror's argument handling
    import ctypes
    from sfm_amd import ba as B
    L = B.lib()
    opts, smr = B.default_options(), B.BASummary()
    tr, tl = (B.BAIteration * 128)(), ctypes.c_int32(0)
    r, t, X = sc.copy_params()
    uv, ci, pi, K = B._f64(sc.uv), B._i32(sc.cam_idx), B._i32(sc.pt_idx), B._f64(sc.K)
    args = (ctypes.byref(opts), B.STRUCT_AND_POSE, int(uv.shape[0]), B.ptr(uv), B.ptr(ci), B.ptr(pi), int(r.shape[0]), B.ptr(K),
            B.ptr(r), B.ptr(t), int(X.shape[0]), B.ptr(X), ctypes.byref(smr), tr, 128, ctypes.byref(tl))
    raw = []
    for it in range(reps + 3):
        np.copyto(r, sc.rot), np.copyto(t, sc.t), np.copyto(X, sc.X)
        t1 = time.perf_counter()
        rc = L.sfm_ba_solve(*args)
        if it >= 3:
            raw.append(time.perf_counter() - t1)
        if rc != 0 or smr.num_iterations != sm.num_iterations:
            raise RuntimeError(f"sfm_ba_solve: rc {rc}, {smr.num_iterations} iterations")
    out = {"workload": "C1 keyframe BA: 20 cams / 2000 pts / 20000 obs, one-shot sfm_ba_solve (upload + LM + download)",
           "ms_per_solve": wall * 1e3, "c_abi_ms_per_solve": float(np.median(raw)) * 1e3,
           "c_abi_ms_per_solve_min": float(np.min(raw)) * 1e3, "lm_iterations": sm.num_iterations,
           "residual_evals_per_s": sc.n_obs * sm.num_residual_evaluations / wall, "cpu_baseline": None,
           "note": "ms_per_solve: sfm_amd.solve (Python mirror) per call, parameters copied in the loop; "
                   "c_abi_ms_per_solve: median of the bare sfm_ba_solve C call"}
    if cpu:
        from oracle import ffi as O
        t0 = time.perf_counter()
        for _ in range(3):
            r, t, X = sc.copy_params()
            smo, _ = O.solve(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, r, t, X)
        cw = (time.perf_counter() - t0) / 3
        out["cpu_baseline"] = {"ms_per_solve": cw * 1e3, "cores": 1, "kind": "port",
                               "sample": "3 C1 solves on oracle/ba_oracle.cpp, 1 thread"}
    return out


def pnp_leg(device: int, cpu: bool, steps: int = 50) -> dict:
    """Per-frame pose of CSfM::tracking: solvePnPRansac (20 iterations, 7 px,
    0.99; CSfM.cpp:553-565) on 500 map-point matches with 30 % outliers."""
    import sfm_amd
    from tests.pnp_cases import K, scene
    X, uv, _, _ = scene(500, 77, noise=0.5, outliers=0.3)
    for _ in range(5):
        sfm_amd.solvePnPRansac(X, uv, K, device=device)
    t0 = time.perf_counter()
    for _ in range(steps):
        found, r, t, inl = sfm_amd.solvePnPRansac(X, uv, K, device=device)
    wall = (time.perf_counter() - t0) / steps
    out = {"workload": "solvePnPRansac: 500 matches, 30% outliers, 20 iterations, 7 px, 0.99 (one call per frame)",
           "ms_per_call": wall * 1e3, "inliers": int(len(inl)), "cpu_baseline": None}
    if cpu:
        from oracle import pnp_oracle as P
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            P.solve_pnp_ransac(X, uv, K)
        cw = (time.perf_counter() - t0) / reps
        out["cpu_baseline"] = {"ms_per_call": cw * 1e3, "cores": 1, "kind": "port",
                               "sample": f"{reps} calls of oracle/pnp_oracle.py (Python restatement: not a speed "
                                         "reference for OpenCV's C++)"}
    return out


def c5_pipeline_leg(device: int, cpu: bool, n_frames: int = 300) -> dict:
    """BASELINE config C5 end to end (sfm_amd.mapping.IncrementalMapper): the
    300-frame 1280x720 synthetic video through per-frame KLT + PnP, a keyframe
    every 10 frames (corners, triangulation, BA over ALL keyframes, as
    CSfM::mapping does after each keyframe).  Frames are rendered before the
    timed region; everything after the frame upload is inside it."""
    from sfm_amd.mapping import IncrementalMapper
    from sfm_amd.video import SyntheticVideo
    v = SyntheticVideo()
    frames = [v.frame(k) for k in range(n_frames)]
    warm = IncrementalMapper(v, device=device)  # first-use costs (module load, caches)
    for f in frames[:21]:
        warm.process_frame(f)
    warm.close()
    m = IncrementalMapper(v, device=device)
    t0 = time.perf_counter()
    for f in frames:
        m.process_frame(f)
    wall = time.perf_counter() - t0
    last = m.ba_log[-1] if m.ba_log else None
    out = {"workload": f"C5 pipeline: {n_frames} frames 1280x720, per-frame LK + PnP, keyframe every 10 frames "
                       "(GFTT replenish, triangulation, BA over all keyframes, one-shot sfm_ba_solve)",
           "frames_per_s": n_frames / wall, "ms_per_frame": wall / n_frames * 1e3, "keyframes": len(m.kf_frames),
           "map_points": int(m.X.shape[0]), "pnp_frames": m.pnp_frames,
           "last_ba": None if last is None else {"cams": int(last["rot"].shape[0]), "points": int(last["X"].shape[0]),
                                                  "obs": int(len(last["uv"])),
                                                  "lm_iterations": last["summary"].num_iterations},
           "host_s": {k: round(val, 4) for k, val in m.times.items()}, "cpu_baseline": None}
    if cpu and m.ba_log:
        from oracle import ffi as O
        t0 = time.perf_counter()
        for rec in m.ba_log:
            r, t, X = rec["rot"].copy(), rec["t"].copy(), rec["X"].copy()
            O.solve(rec["uv"], rec["cam_idx"], rec["pt_idx"], rec["K"], r, t, X)
        cw = time.perf_counter() - t0
        out["cpu_baseline"] = {"ba_s_all_keyframes": cw, "gpu_ba_s_all_keyframes": m.times["ba"], "cores": 1,
                               "kind": "port", "sample": f"the {len(m.ba_log)} keyframe BA problems of this run "
                                                         "re-solved by oracle/ba_oracle.cpp, 1 thread"}
    m.close()
    return out


def live_path_leg(device: int, cpu: bool, n_frames: int = 300) -> dict:
    """The reference's live tracking path (sfm_amd.live.LiveSfM: CSfM::tracking
    + CSfM::mapping) on synthetic detector output (~1100 keypoints, 64-B
    descriptors per frame; the device BRISK leg is timed separately): per frame
    matchFeatures(prevIdx, currIdx) + PnP + map-point re-finding through the
    device map store, per keyframe KF-pair matching, triangulation and BA over
    all keyframes.  Keypoint frames are generated before the timed region."""
    from sfm_amd.live import KeypointStream, LiveSfM
    st = KeypointStream()
    frames = [st.frame(k)[:2] for k in range(n_frames)]
    warm = LiveSfM(st, device=device)
    for k in range(25):
        warm.process(k, *frames[k])
    warm.close()
    s = LiveSfM(st, device=device)
    t0 = time.perf_counter()
    for k in range(n_frames):
        s.process(k, *frames[k])
    wall = time.perf_counter() - t0
    last = s.ba_log[-1] if s.ba_log else None
    n_pts, n_obs, _ = s.map.size()
    out = {"workload": f"live path: {n_frames} frames of synthetic detector output (~1100 keypoints, 64-B descriptors), "
                       "matchFeatures(prevIdx, currIdx) + solvePnPRansac + findMapPointsInCurrentFrame per frame, "
                       "mapping + BA over all keyframes per keyframe",
           "frames_per_s": n_frames / wall, "ms_per_frame": wall / n_frames * 1e3, "keyframes": len(s.kfs),
           "map_points": int(n_pts), "map_observations": int(n_obs), "tracked_frames": s.stats["tracked"],
           "last_ba": None if last is None else {"cams": int(last["rot"].shape[0]), "points": int(last["X"].shape[0]),
                                                  "obs": int(len(last["uv"])),
                                                  "lm_iterations": last["summary"].num_iterations},
           "host_s": {k: round(val, 4) for k, val in s.times.items() if k != "stream"},
           "ba_solves": len(s.ba_log), "ba_lm_iterations": int(s.stats.get("ba_iterations", 0)), "cpu_baseline": None}
    if cpu and s.ba_log:
        from oracle import ffi as O
        t0 = time.perf_counter()
        for rec in s.ba_log:
            r, t, X = rec["rot"].copy(), rec["t"].copy(), rec["X"].copy()
            O.solve(rec["uv"], rec["cam_idx"], rec["pt_idx"], rec["K"], r, t, X)
        cw = time.perf_counter() - t0
        out["cpu_baseline"] = {"ba_s_all_keyframes": cw, "gpu_ba_s_all_keyframes": s.times["ba"], "cores": 1,
                               "kind": "port", "sample": f"the {len(s.ba_log)} keyframe BA problems of this run "
                                                         "re-solved by oracle/ba_oracle.cpp, 1 thread"}
    s.close()
    return out


def brisk_leg(device: int, cpu: bool, n_frames: int = 20) -> dict:
    """CTracker::detectFeatures on the device (sfm_brisk_detect_describe:
    BRISK threshold 60, 6 octaves, 64-B descriptors) on rendered 1280x720
    frames of the synthetic video (rendered before the timed region)."""
    from sfm_amd import brisk
    from sfm_amd.video import SyntheticVideo
    v = SyntheticVideo(speed=2.0)
    frames = [v.frame(k) for k in range(n_frames)]
    brisk.detect(frames[0])  # pattern upload, workspace
    t0 = time.perf_counter()
    nk = 0
    for f in frames:
        kp, _, _ = brisk.detect(f)
        nk += len(kp)
    wall = time.perf_counter() - t0
    out = {"workload": f"BRISK detect + describe (threshold 60, 6 octaves) on {n_frames} rendered 1280x720 frames, "
                       "host image in, keypoints + 64-B descriptors out",
           "ms_per_frame": wall / n_frames * 1e3, "keypoints_per_frame": nk / n_frames, "cpu_baseline": None}
    # one upload per frame: the KLT handle's push (pyramid + derivatives)
    # then BRISK on its resident frame (sfm_klt_brisk_detect_describe)
    from sfm_amd.klt import KLTTracker
    klt = KLTTracker(frames[0].shape[1], frames[0].shape[0], device=device)
    try:
        klt.push_frame(frames[0])
        brisk.detect_resident(klt)
        t0 = time.perf_counter()
        for f in frames:
            klt.push_frame(f)
            brisk.detect_resident(klt)
        wall_r = time.perf_counter() - t0
    finally:
        klt.close()
    out["resident_klt_frame"] = {"ms_per_frame": wall_r / n_frames * 1e3,
                                 "workload": "per frame: sfm_klt_push_frame (the one upload: pyramid + Scharr "
                                             "derivatives) + BRISK detect + describe on the resident frame"}
    if cpu:
        from oracle import brisk_oracle as B
        t0 = time.perf_counter()
        B.detect(frames[0])
        out["cpu_baseline"] = {"detect_ms_one_frame": (time.perf_counter() - t0) * 1e3, "cores": 1, "kind": "port",
                               "sample": "detection only on one frame by oracle/brisk_oracle.py (numpy restatement: "
                                         "not a speed reference for the reference's C++ library)"}
    return out


def oneshot_leg(sc, reps: int = 3) -> dict:
    """One-shot C3 solve as the drop-in is called: host arrays in,
    sfm_ba_solve (problem setup + upload + LM + download) -- the reference
    rebuilds its ceres::Problem on every call (CTracker.cpp:672).  One
    warm-up, then the median of `reps` (BASELINE.md timing protocol)."""
    import sfm_amd
    walls = []
    sm = None
    for k in range(reps + 1):
        r, t, X = sc.copy_params()
        t0 = time.perf_counter()
        sm, _ = sfm_amd.solve(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, r, t, X)
        if k > 0:
            walls.append(time.perf_counter() - t0)
    wall = float(np.median(walls))
    return {"workload": f"C3 one-shot sfm_ba_solve ({sc.n_cams} cams / {sc.n_pts} pts / {sc.n_obs} obs): host "
                        "arrays in, setup + upload + LM + download", "ms_per_solve": wall * 1e3,
            "ms_runs": [w * 1e3 for w in walls], "lm_iterations": sm.num_iterations,
            "lm_iterations_per_s": sm.num_iterations / wall}


def stream_copy_gbs(device: int) -> float:
    """Measured device-to-device copy bandwidth (STREAM copy: read + write
    bytes / time) of a 4 GiB buffer with 16-B accesses (sfm_bench_stream_copy:
    the best of a few grid / unroll shapes, 5 timed launches each), beside the
    8 TB/s spec; MI355X_MICROARCH.md measures 6.29 TB/s this way."""
    import ctypes
    import sfm_amd
    from sfm_amd._ffi import check
    gbs = ctypes.c_double(0.0)
    check(sfm_amd.lib().sfm_bench_stream_copy(device, 1 << 32, 5, ctypes.byref(gbs)), "sfm_bench_stream_copy")
    return gbs.value


def stream_copy_sizes(device: int) -> dict:
    """The same copy at several buffer sizes: below ~256 MiB the Infinity
    Cache (MALL) holds part of the working set, so only the 4-GiB figure is
    the HBM one."""
    import ctypes
    import sfm_amd
    from sfm_amd._ffi import check
    out = {}
    for mib in (64, 256, 1024, 4096):
        gbs = ctypes.c_double(0.0)
        check(sfm_amd.lib().sfm_bench_stream_copy(device, mib << 20, 5, ctypes.byref(gbs)), "sfm_bench_stream_copy")
        out[f"{mib}MiB"] = round(gbs.value, 1)
    return out


def matcher_leg(device: int, steps: int, cpu: bool) -> dict:
    """The per-frame matcher of CSfM::tracking (CSfM.cpp:518 ->
    CTracker::matchFeatures(prevIdx, currIdx, ...), CTracker.cpp:368-417):
    2000 keypoints per frame with 64-B (512-bit) descriptors; one step =
    push_frame (upload of the new frame's keypoints + descriptors, the
    _prevFrame = _currFrame swap) + the 2-NN Hamming search + the ratio /
    window / better-match-replaces rules over all keypoints of both frames.
    Frames cycle over 3 synthetic frames (descriptors re-observed with bit
    noise, keypoints moved a few pixels)."""
    from sfm_amd.matcher import FeatureMatcher
    rng = np.random.default_rng(11)
    n = 2000
    base_d = rng.integers(0, 256, (n, 64), dtype=np.uint8)
    base_p = rng.uniform(0, [1280, 720], (n, 2))
    frames = []
    for k in range(3):
        d = base_d.copy()
        flips = rng.integers(0, 512, (n, 24))
        for j in range(24):
            d[np.arange(n), flips[:, j] // 8] ^= (1 << (flips[:, j] % 8)).astype(np.uint8)
        p = base_p + rng.normal(0, 4, (n, 2)) + 3 * k
        perm = rng.permutation(n)
        frames.append((p[perm].copy(), d[perm].copy()))
    idx = np.arange(n, dtype=np.int32)
    m = FeatureMatcher(64, device=device)
    m.push_frame(*frames[0])
    warm = 5
    knn_ms = call_ms = 0.0
    nmatch = 0
    for it in range(steps + warm):
        if it == warm:
            t0 = time.perf_counter()
            knn_ms = call_ms = 0.0
        m.push_frame(*frames[(it + 1) % 3])
        a, b = m.match_subset(idx, idx)
        nmatch = len(a)
        k_ms, c_ms = m.last_time_ms()
        knn_ms += k_ms
        call_ms += c_ms
    wall = (time.perf_counter() - t0) / steps
    m.close()
    pairs = n * n
    out = {"workload": "C5 matcher: CTracker::matchFeatures(prevIdx, currIdx, ...) per frame, 2000 x 2000 keypoints, "
                       "64-B descriptors (push_frame + 2-NN Hamming + ratio 0.8 / window (1.5, 40) / replacement)",
           "frames_per_s": 1.0 / wall, "ms_per_frame": wall * 1e3, "matches_per_frame": nmatch,
           "device_ms_per_frame": {"knn2": round(knn_ms / steps, 4), "match_call": round(call_ms / steps, 4)},
           "hamming_pairs_per_s": pairs / (knn_ms / steps * 1e-3) if knn_ms > 0 else None,
           "cpu_baseline": None}
    if cpu:
        from oracle import ffi as O
        reps = 5
        t0 = time.perf_counter()
        for r in range(reps):
            (p0, d0), (p1, d1) = frames[r % 3], frames[(r + 1) % 3]
            O.match_features(p0, d0, p1, d1)
        cw = (time.perf_counter() - t0) / reps
        out["cpu_baseline"] = {"frames_per_s": 1.0 / cw, "ms_per_frame": cw * 1e3, "cores": 1, "kind": "port",
                               "sample": f"{reps} frame pairs of the same match on oracle/match_oracle.cpp, 1 thread"}
    return out


def self_launch(argv) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: start the N
    ranks through torch.distributed.run (one process per GPU, rendezvous on
    127.0.0.1) BEFORE anything touches the GPU, as a child process, and exit
    with its code (never an exec from a process that could have initialised
    the GPU)."""
    import socket
    import subprocess
    n = None
    for i, a in enumerate(argv):
        if a == "--gpus" and i + 1 < len(argv):
            n = int(argv[i + 1])
        elif a.startswith("--gpus="):
            n = int(a.split("=", 1)[1])
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def factor_layout(args, world: int, strong: bool) -> int:
    """Panel width (64-column tiles) of the distributed reduced-camera factor,
    0 = replicated (sfm_ba_set_distributed_factor).  Auto: the distributed
    factor with 8-tile panels for the strong-scaling C4 headline, which the
    model built on this GPU's measured parts predicts ahead of the replicated
    factor at every N > 1 (tools/dist_factor_model.py);
    replicated for the weak C3-per-GPU line (a 3000^2 system: one 36-MB
    all-reduce per LM iteration)."""
    if args.dist_pt >= 0:
        return args.dist_pt
    return 8 if (world > 1 and strong) else 0


def measure_ba(cams: int, P_total: int, p_begin: int, p_end: int, seed: int, strong: bool, args, world: int,
               rank: int, local_rank: int, dist, comm: bool) -> dict:
    """One BA workload: the scene's landmark shard [p_begin, p_end) set up
    resident, W untimed solves, then K timed solves (device reset + LM to
    Ceres' termination) between barriers, max over ranks; then a profiled
    pass of the same solves for the phase times."""
    import torch
    import sfm_amd
    from sfm_amd import scene as S
    sc = S.generate(cams, P_total, seed=seed, p_begin=p_begin, p_end=p_end)
    if rank == 0:
        print(f"[bench] {cams} cams / {P_total} pts: scene ready ({sc.n_obs} obs on rank 0)", file=sys.stderr, flush=True)
    ba = sfm_amd.BundleAdjuster(device=local_rank)
    if world > 1:
        uid = [sfm_amd.BundleAdjuster.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ba.set_comm(world, rank, uid[0])
    elif comm:
        ba.set_comm(1, 0, sfm_amd.BundleAdjuster.unique_id())
    dist_pt = factor_layout(args, world, strong) if (world > 1 or comm) else 0
    if dist_pt:
        ba.set_distributed_factor(dist_pt)
    t0 = time.perf_counter()
    ba.set_problem(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, sc.rot, sc.t, sc.X)
    ba.sync()
    setup_s = time.perf_counter() - t0
    opts = sfm_amd.default_options()

    def barrier():
        ba.sync()
        torch.cuda.synchronize(local_rank)
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        ba.reset()
        ba.solve(opts)
    barrier()
    if rank == 0:
        print(f"[bench] set_problem {setup_s:.2f} s, warm-up done", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    iters = evals = jevals = 0
    last = None
    for _ in range(args.steps):
        ba.reset()
        sm, _ = ba.solve(opts)
        iters += sm.num_iterations
        evals += sm.num_residual_evaluations
        jevals += sm.num_jacobian_evaluations
        last = sm
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        print(f"[bench] timed: {elapsed / max(1, args.steps) * 1e3:.3f} ms per solve", file=sys.stderr, flush=True)
    # phase breakdown from a separate pass of the same solves (the HIP events
    # it records stay out of the timed region above).  That pass runs the
    # host-driven LM loop (the same kernels): the device-driven loop also
    # enqueues phases that its flags then skip, which would count as launches
    prev_host_lm = os.environ.get("SFM_HOST_LM")
    os.environ["SFM_HOST_LM"] = "1"
    ba.set_profiling(True)
    for _ in range(args.steps):
        ba.reset()
        ba.solve(opts)
    ba.sync()
    phases = ba.phase_times()
    ba.set_profiling(False)
    if prev_host_lm is None:
        del os.environ["SFM_HOST_LM"]
    else:
        os.environ["SFM_HOST_LM"] = prev_host_lm
    n_obs_total = VIEWS * P_total   # every point has VIEWS observations
    res_only = evals - jevals       # residual-only (candidate) evaluations
    return {"ba": ba, "sc": sc, "elapsed": elapsed, "iters": iters, "evals": evals, "jevals": jevals, "last": last,
            "phases": phases, "setup_s": setup_s, "n_obs_total": n_obs_total, "n_pts_total": P_total,
            "res_only": res_only, "value": n_obs_total * res_only / elapsed, "strong": strong, "dist_pt": dist_pt}


def ba_summary(m: dict, args, world: int) -> dict:
    """The per-workload fields of a bench line."""
    sc, phases, last = m["sc"], m["phases"], m["last"]
    elapsed = m["elapsed"]
    return {
        "value": m["value"],
        "ms_per_step": elapsed / args.steps * 1e3,
        "scaling": "strong" if m["strong"] else "weak",
        "lm_iterations_per_s": m["iters"] / elapsed,
        "jacobian_evals_per_s": m["n_obs_total"] * m["jevals"] / elapsed,
        "lm_iterations_per_solve": m["iters"] / args.steps,
        "residual_only_evals_per_solve": m["res_only"] / args.steps,
        "jacobian_evals_per_solve": m["jevals"] / args.steps,
        "final_cost": last.final_cost if last else None,
        "set_problem_s": round(m["setup_s"], 4),
        "phase_ms_per_solve": {k: round(v["ms"] / args.steps, 4) for k, v in phases.items()},
        "workload": {"cams": sc.n_cams, "points": m["n_pts_total"], "observations": m["n_obs_total"],
                     "points_per_gpu": sc.n_pts, "obs_per_gpu": sc.n_obs, "views_per_point": VIEWS,
                     "parallelism": f"landmark-sharded x{world}" if world > 1 else "single GPU",
                     "reduced_camera_factor": (f"distributed: 1-D block-cyclic panels of {m['dist_pt']} tiles"
                                               if m["dist_pt"] else
                                               ("replicated (all-reduce of the packed system)" if world > 1
                                                else "single GPU"))},
    }


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pts-per-gpu", type=int, default=0,
                    help="weak scaling: this many points per rank (default at N=1: C3's 200k)")
    ap.add_argument("--cams", type=int, default=0, help="cameras (default: C3's 500, or C4's 2000 at N>1)")
    ap.add_argument("--total-pts", type=int, default=0,
                    help="strong scaling: this many points in total, split into landmark shards over the ranks "
                         "(BASELINE config C4: --cams 2000 --total-pts 1000000; the default headline at N>1)")
    ap.add_argument("--phases", action="store_true", help="print the per-phase breakdown to stderr")
    ap.add_argument("--no-tracker", action="store_true", help="skip the C5 tracker / matcher / keyframe legs")
    ap.add_argument("--no-oneshot", action="store_true", help="skip the one-shot C3 leg")
    ap.add_argument("--no-stream-copy", action="store_true",
                    help="skip the STREAM-copy reference (kernel traces of the BA kernels alone)")
    ap.add_argument("--c4-n1", action="store_true",
                    help="N=1: also measure BASELINE C4 on this GPU (the N=1 point of the strong-scaling curve the "
                         "N>1 lines report; off by default so that a kernel trace of the default command holds the "
                         "C3 headline's kernels only)")
    ap.add_argument("--dist-pt", type=int, default=-1,
                    help="reduced-camera factor at N>1: 0 replicated, k>0 distributed panels of k 64-column tiles, "
                         "-1 auto (8-tile panels for the C4 headline)")
    ap.add_argument("--comm", action="store_true",
                    help="use an RCCL communicator even at N=1 (exercises the sharded path's collectives)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check: ranks rendezvous and report the world, no GPU call")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(sys.argv[1:])

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE", file=sys.stderr)

    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        world = dist.get_world_size()   # n_gpus: the communicator's rank count
    if args.dry_run:
        t = torch.tensor([1.0])
        if world > 1:
            dist.all_reduce(t)
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_reporting": int(t.item()),
                              "local_rank": local_rank}))
        if world > 1:
            dist.destroy_process_group()
        return 0

    # headline workload: C3 at N=1 (BASELINE's single-GPU full-solve config);
    # at N>1 BASELINE C4 (2000 cams / 1M points / 10M obs) landmark-sharded
    # over the ranks (strong scaling), with C3-per-GPU weak scaling beside it
    explicit = args.total_pts > 0 or args.pts_per_gpu > 0
    if args.total_pts > 0:
        strong, cams, P_total = True, args.cams or CAMS, args.total_pts
        seed = SEED + 1 if (cams, P_total) == C4 else SEED
    elif args.pts_per_gpu > 0:
        strong, cams, P_total, seed = False, args.cams or CAMS, args.pts_per_gpu * world, SEED
    elif world > 1:
        strong, (cams, P_total), seed = True, C4, SEED + 1
    else:
        strong, cams, P_total, seed = False, args.cams or CAMS, PTS_PER_GPU, SEED
    if strong:
        p_begin, p_end = rank * P_total // world, (rank + 1) * P_total // world
    else:
        per = P_total // world
        p_begin, p_end = rank * per, (rank + 1) * per
    m = measure_ba(cams, P_total, p_begin, p_end, seed, strong, args, world, rank, local_rank, dist, args.comm)
    ba, sc, phases = m["ba"], m["sc"], m["phases"]
    head = ba_summary(m, args, world)

    jac = phases["jacobian"]
    # The solve's Jacobian pass is record-free (cost + U_c/b_c partials only;
    # the later passes recompute residuals and Jacobians)
    jac_solve_ms = jac["ms"] / max(1, jac["count"])
    cnt = np.bincount(sc.cam_idx, minlength=sc.n_cams)
    n_pad = int(((cnt + 63) // 64 * 64).sum())   # camera-major slots, runs padded to 64
    jac_bytes_s = jacobian_bytes_solve(n_pad, sc.n_cams, sc.n_pts)
    jac_gbs_s = jac_bytes_s / (jac_solve_ms * 1e-3) / 1e9
    jac_tfs_s = jacobian_flops_solve(sc.n_obs) / (jac_solve_ms * 1e-3) / 1e12
    jac_ms = ba.bench_jacobian(10)
    jac_bytes = jacobian_bytes(sc.n_obs, sc.n_cams, sc.n_pts)
    jac_gbs = jac_bytes / (jac_ms * 1e-3) / 1e9
    chol = phases["cholesky"]
    chol_ms = chol["ms"] / max(1, chol["count"])
    n_sys = 6 * sc.n_cams
    chol_tfs = cholesky_flops(n_sys) / (chol_ms * 1e-3) / 1e12
    dominant = max(phases, key=lambda k: phases[k]["ms"])

    # HBM bytes per launch from the committed PMC passes (tools/pmc_traffic.sh
    # -> tools/pmc_json.py -> profiles/pmc_c3.json; FETCH_SIZE/WRITE_SIZE in
    # separate passes, corrected per MI355X_MICROARCH.md "HBM").  Only valid
    # for the workload they were collected on (C3).
    pmc = {}
    prof = os.path.join(ROOT, "profiles", "pmc_c3.json")
    if os.path.exists(prof):
        try:
            with open(prof) as f:
                pm = json.load(f)
            if pm.get("n_obs") == sc.n_obs:
                pmc = pm.get("kernels", {})
        except (OSError, ValueError):
            pmc = {}

    mfma = {}
    prof2 = os.path.join(ROOT, "profiles", "pmc_mfma_c3.json")
    if os.path.exists(prof2) and pmc:
        try:
            with open(prof2) as f:
                mfma = json.load(f).get("kernels", {})
        except (OSError, ValueError):
            mfma = {}

    def traffic(kernel):
        e = pmc.get(kernel) or pmc.get(kernel + "<false>") or {}
        v = e.get("hbm_bytes_per_launch")
        return None if v is None else int(v)

    # the production pass of the solve (record-free): HIP events on the
    # solver stream over the profiled pass of the same solves
    roof_jac = {"kernel": "k_jacobian (residual + 2x9 Jacobian pass, record-free, as run inside the solve)",
                "bound": "hbm", "achieved": round(jac_gbs_s, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(jac_gbs_s / HBM_PEAK_GBS, 4), "traffic": traffic("k_jacobian"),
                "algorithmic_bytes": jac_bytes_s, "avg_launch_ms": round(jac_solve_ms, 5),
                "valu": {"achieved_tflops": round(jac_tfs_s, 3), "peak_tflops": F64_VALU_PEAK_TFS,
                         "frac": round(jac_tfs_s / F64_VALU_PEAK_TFS, 4),
                         "algorithmic_flops": jacobian_flops_solve(sc.n_obs)},
                "note": "latency-bound (X gathers, the 27 U_c/b_c wave reductions); traffic: PMC of the "
                        "record-free launches only (profiles/pmc_c3.json)"}
    roof_jac_rec = {"kernel": "k_jacobian_rec (record-writing variant, evaluate API; not run by the solve)",
                    "bound": "hbm", "achieved": round(jac_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(jac_gbs / HBM_PEAK_GBS, 4), "traffic": traffic("k_jacobian_rec"),
                    "algorithmic_bytes": jac_bytes, "avg_launch_ms": round(jac_ms, 5),
                    "variant": "timed back to back by sfm_ba_bench_jacobian (warm caches)"}
    roof_chol = {"kernel": "k_chol_fused (dense reduced-camera Cholesky, one persistent launch, f64 MFMA)", "bound": "mfma",
                 "achieved": round(chol_tfs, 3), "peak": F64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                 "frac": round(chol_tfs / F64_MFMA_PEAK_TFS, 4), "traffic": traffic("k_chol_fused"),
                 "algorithmic_flops": cholesky_flops(n_sys), "avg_ms": round(chol_ms, 4),
                 "mfma_busy_frac_pmc": (mfma.get("k_chol_fused<false>") or mfma.get("k_chol_fused") or {}).get(
                     "mfma_busy_frac")}
    roofline = roof_chol if dominant == "cholesky" else roof_jac

    wl = head.pop("workload")
    if strong:
        wname = (f"{cams} cams / {P_total} points / {m['n_obs_total']} obs in total"
                 + (" (BASELINE C4)" if (cams, P_total) == C4 else "")
                 + ", landmark-sharded over the ranks (strong scaling): full BA solve (LM + DENSE_SCHUR, "
                   "Ceres default options)")
    else:
        wname = ("C3 per GPU" if (cams, P_total // world) == (CAMS, PTS_PER_GPU) else
                 f"{cams} cams / {P_total // world} points per GPU") + \
                ": full BA solve (LM + DENSE_SCHUR, Ceres default options)"
    out = {
        "metric": "BA iterations/sec + residual-evals/sec (cams x pts x obs); 1/2/4/8 GPU",
        "value": head.pop("value"),
        "unit": "residual-evals/s (obs x evaluations)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": head.pop("ms_per_step"),
        "higher_is_better": True,
        "scaling": head.pop("scaling"),
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded object-scanning scene, SURVEY.md §8d; K from main/main.cpp:47-50)",
        "config": dict({"workload": wname}, **wl),
    }
    out.update(head)
    out.update({"roofline": roofline, "roofline_jacobian": roof_jac, "roofline_jacobian_records": roof_jac_rec,
                "roofline_cholesky": roof_chol})
    if world > 1 and not explicit:
        # weak scaling beside the strong headline: C3 per rank
        ba.close()
        mw = measure_ba(CAMS, PTS_PER_GPU * world, rank * PTS_PER_GPU, (rank + 1) * PTS_PER_GPU, SEED, False,
                        args, world, rank, local_rank, dist, False)
        wk = ba_summary(mw, args, world)
        wk["workload"] = dict({"workload": "C3 per GPU (weak scaling): full BA solve"}, **wk["workload"])
        out["weak_c3_per_gpu"] = wk
        mw["ba"].close()
        ba = None
    if rank == 0 and world == 1 and not args.no_stream_copy:
        out["stream_copy_gbs"] = round(stream_copy_gbs(local_rank), 1)
        out["stream_copy_gbs_by_buffer"] = stream_copy_sizes(local_rank)
    if rank == 0 and world == 1 and not args.no_oneshot:
        ba.close()  # the one-shot path keeps its own cached handle
        out["oneshot"] = oneshot_leg(sc)
    if world == 1 and not explicit and args.c4_n1:
        # the N = 1 point of the C4 strong-scaling curve (N > 1 lines report C4)
        if ba is not None:
            ba.close()
        m4 = measure_ba(C4[0], C4[1], 0, C4[1], SEED + 1, True, args, 1, 0, local_rank, dist, False)
        c4 = ba_summary(m4, args, 1)
        c4["workload"] = dict({"workload": "BASELINE C4 on one GPU (the N=1 point of the strong-scaling curve)"},
                              **c4["workload"])
        ph = m4["phases"]["cholesky"]
        c4_chol_ms = ph["ms"] / max(1, ph["count"])
        c4["cholesky_tflops"] = round(cholesky_flops(6 * C4[0]) / (c4_chol_ms * 1e-3) / 1e12, 2)
        out["c4_strong_n1"] = c4
        m4["ba"].close()
        ba = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # bounded: the oracle's C3 solve takes ~11 s per run on one core; a
        # larger explicit workload (C4: minutes per oracle solve) is sampled
        # by the C3 problem, whose residual-eval rate the line then reports
        big = sc.n_obs > 2_500_000
        print(f"[bench] cpu baseline ({'C3 sample' if big else 'same workload'})", file=sys.stderr, flush=True)
        from sfm_amd import scene as S
        cpu = cpu_baseline(S.config("C3") if big else sc)
        if big:
            cpu["sample"] = "C3 sample of the larger workload: " + cpu["sample"]
        out["cpu_baseline"] = cpu
        out["speedup_vs_cpu"] = out["value"] / cpu["value"]
        if "oneshot" in out:
            out["speedup_vs_cpu_oneshot"] = cpu["solve_s"] * 1e3 / out["oneshot"]["ms_per_solve"]
            out["speedup_vs_cpu_oneshot_multi_thread"] = cpu["multi_thread"]["solve_s"] * 1e3 / out["oneshot"]["ms_per_solve"]
    else:
        out["cpu_baseline"] = None
    if rank == 0 and world == 1 and not args.no_tracker:
        cb = not args.no_cpu_baseline
        for name, leg in (("tracker", lambda: tracker_leg(local_rank, 50, cb)),
                          ("matcher", lambda: matcher_leg(local_rank, 50, cb)),
                          ("incremental_ba", lambda: incremental_ba_leg(local_rank, cb)),
                          ("pnp", lambda: pnp_leg(local_rank, cb)),
                          ("c5_pipeline", lambda: c5_pipeline_leg(local_rank, cb)),
                          ("live_path", lambda: live_path_leg(local_rank, cb)),
                          ("brisk", lambda: brisk_leg(local_rank, cb))):
            print(f"[bench] leg {name}", file=sys.stderr, flush=True)
            out[name] = leg()
    if args.phases and rank == 0:
        print(json.dumps(phases, indent=1), file=sys.stderr)
    if rank == 0:
        print(json.dumps(out))
    if ba is not None:
        ba.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
