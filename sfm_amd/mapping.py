"""Config C5 end to end: per-frame KLT tracking on the device + incremental
bundle adjustment over all keyframes (BASELINE.json configs[4]; SURVEY.md
§8d "C5"), chained the way CSfM drives the reference's hot path:

* every frame (CSfM::tracking, /root/reference/CSfM.cpp:500-631): the frame
  goes up once (pyramids + Scharr derivatives resident, KLTTracker), the
  live tracks are flowed by calcOpticalFlowPyrLK (T6), and the frame's pose
  comes from solvePnPRansac over the tracks that carry map points
  (CSfM.cpp:553-565; sfm_pnp_ransac, 20 iterations, 7 px, 0.99);
* every `kf_every` frames (CSfM.cpp:44: keyframes at least 10 frames apart)
  a keyframe (CSfM.cpp:595-619): its tracked points become observations,
  new corners are detected (goodFeaturesToTrack + cornerSubPix, T7) to
  replenish the tracks, tracks seen by two keyframes without a map point
  are triangulated (GeometryUtils::triangulatePoints, CSfM.cpp:156:
  sfm_triangulate_points) and kept when in front of both cameras and within
  _maxReprErr = 7 px (CSfM.cpp:165), and bundle adjustment runs over ALL
  keyframes (CSfM::mapping -> bundleAdjustment, CSfM.cpp:252-259,
  STRUCT_AND_POSE) on a fresh problem gathered frame-major as
  CSfM::bundleAdjustment does (CSfM.cpp:310-348; one-shot sfm_ba_solve).

Scope notes: the map is bootstrapped from the video's known
relative pose of the first keyframe pair (the reference's initialisation,
CSfM::init with findHomography / findFundamentalMat, is OpenCV's and out
of scope); tracks follow the flowed LK positions (the association step of
computeOpticalFlow re-anchors points to fresh detections, which ends most
tracks within a few frames -- row T6 keeps it bit-exact on its own); the
reprojection re-finding of CSfM.cpp:190-221 is not restated (tracks already
carry the multi-keyframe observations).

The synthetic video is a textured plane under similarity motion
(sfm_amd.video): with fx = fy = f and the principal point at the image
centre it is exactly a pinhole camera rolling about its optical axis and
translating, the plane at depth `depth` in the first camera's frame, so
every frame has a closed-form ground-truth pose (gt_pose).
"""
from __future__ import annotations

import time

import numpy as np

from . import ba as _ba
from .klt import KLTTracker
from .pnp import solvePnPRansac
from ._ffi import check, lib, ptr
from .video import SyntheticVideo

F_PIX = 1072.606693272117800  # main/main.cpp:47 fx


def triangulate_points(cam0, cam1, uv0, uv1, P, device: int = 0) -> np.ndarray:
    """Device cv::triangulatePoints per point on P [C][3][4] (sfm_triangulate_points)."""
    cam0 = np.ascontiguousarray(cam0, np.int32)
    cam1 = np.ascontiguousarray(cam1, np.int32)
    uv0 = np.ascontiguousarray(np.asarray(uv0, np.float64).reshape(-1, 2))
    uv1 = np.ascontiguousarray(np.asarray(uv1, np.float64).reshape(-1, 2))
    P = np.ascontiguousarray(np.asarray(P, np.float64).reshape(-1, 12))
    n = int(cam0.shape[0])
    X = np.zeros((max(1, n), 3))
    check(lib().sfm_triangulate_points(device, n, ptr(cam0), ptr(cam1), ptr(uv0), ptr(uv1), int(P.shape[0]), ptr(P),
                                       ptr(X)), "sfm_triangulate_points")
    return X[:n].copy()


def video_gt_pose(video, k: int, depth: float = 10.0):
    """(rvec, t) of frame k of sfm_amd.video.SyntheticVideo relative to frame 0:
    a pinhole camera rolling about its optical axis and translating over the
    textured plane at `depth` (closed form of the video's similarity)."""
    s0, th0, t0 = video.pose(0)
    sk, thk, tk = video.pose(k)
    s, th = sk / s0, thk - th0
    B = s * np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
    d = tk - B @ t0
    tz = depth / s - depth
    t = np.array([d[0] * depth / (s * F_PIX), d[1] * depth / (s * F_PIX), tz])
    return np.array([0.0, 0.0, th]), t


def _rodrigues(r):
    r = np.asarray(r, np.float64)
    th = float(np.sqrt(r @ r))
    if th < np.finfo(float).eps:
        return np.eye(3)
    u = r / th
    c, s = np.cos(th), np.sin(th)
    return c * np.eye(3) + (1 - c) * np.outer(u, u) + s * np.array([[0, -u[2], u[1]], [u[2], 0, -u[0]],
                                                                    [-u[1], u[0], 0]])


class IncrementalMapper:
    def __init__(self, video: SyntheticVideo | None = None, device: int = 0, kf_every: int = 10,
                 depth: float = 10.0, max_tracks: int = 500, min_track_dist: float = 10.0):
        self.video = video if video is not None else SyntheticVideo()
        self.device = device
        self.kf_every = int(kf_every)
        self.depth = float(depth)
        self.max_tracks = int(max_tracks)
        self.min_track_dist = float(min_track_dist)
        w, h = self.video.w, self.video.h
        self.K = np.array([[F_PIX, 0.0, self.video.c[0]], [0.0, F_PIX, self.video.c[1]], [0.0, 0.0, 1.0]])
        self.tracker = KLTTracker(w, h, device=device)
        self.frame_no = -1
        self.tr_uv = np.zeros((0, 2), np.float32)   # live tracks: current position
        self.tr_id = np.zeros(0, np.int64)          # ... and track id
        self.next_id = 0
        # keyframe observations in append (= keyframe-major) order
        self.obs_kf = np.zeros(0, np.int32)
        self.obs_tid = np.zeros(0, np.int64)
        self.obs_uv = np.zeros((0, 2), np.float64)
        # per track id: map point (-1: none), first keyframe observation, count
        self.pt_of = np.zeros(0, np.int64)
        self.first_kf = np.zeros(0, np.int32)
        self.first_uv = np.zeros((0, 2), np.float64)
        self.nobs = np.zeros(0, np.int32)
        self.X = np.zeros((0, 3))
        self.kf_frames: list[int] = []
        self.kf_rot: list[np.ndarray] = []
        self.kf_t: list[np.ndarray] = []
        self.pose = (np.zeros(3), np.zeros(3))      # current frame's pose (rvec, t)
        self.ba_log: list[dict] = []
        self.times = {"render": 0.0, "track": 0.0, "pnp": 0.0, "keyframe": 0.0, "ba": 0.0}
        self.pnp_frames = 0

    # ---- ground truth of the synthetic video --------------------------------
    def gt_pose(self, k: int):
        return video_gt_pose(self.video, k, self.depth)

    # ---- per frame ----------------------------------------------------------------
    def process_frame(self, grey: np.ndarray) -> None:
        self.frame_no += 1
        k = self.frame_no
        t0 = time.perf_counter()
        self.tracker.push_frame(grey)
        if k > 0 and len(self.tr_uv):
            nxt, st = self.tracker.calc_flow(self.tr_uv)
            w, h = self.video.w, self.video.h
            keep = (st != 0) & (nxt[:, 0] >= 0) & (nxt[:, 1] >= 0) & (nxt[:, 0] <= w - 1) & (nxt[:, 1] <= h - 1)
            self.tr_uv, self.tr_id = nxt[keep], self.tr_id[keep]
        t1 = time.perf_counter()
        self.times["track"] += t1 - t0
        if k > 0 and self.X.shape[0]:
            pid = self.pt_of[self.tr_id]
            has = pid >= 0
            if has.sum() >= 5:
                obj = self.X[pid[has]]
                found, r, t, inl = solvePnPRansac(obj, self.tr_uv[has].astype(np.float64), self.K,
                                                  device=self.device)
                if found:
                    self.pose = (r, t)
                    self.pnp_frames += 1
        self.times["pnp"] += time.perf_counter() - t1
        if k % self.kf_every == 0:
            t2 = time.perf_counter()
            self._keyframe(k)
            self.times["keyframe"] += time.perf_counter() - t2

    def _keyframe(self, k: int) -> None:
        j = len(self.kf_frames)
        if j == 0:
            rot, t = np.zeros(3), np.zeros(3)         # CFrame.cpp:229-235: first keyframe at the origin
        elif j == 1:
            rot, t = self.gt_pose(k)                  # bootstrap (CSfM::init is out of scope)
        else:
            rot, t = self.pose[0].copy(), self.pose[1].copy()
        self.kf_frames.append(k)
        self.kf_rot.append(np.asarray(rot, np.float64))
        self.kf_t.append(np.asarray(t, np.float64))
        n_live = len(self.tr_id)
        if n_live:
            self.obs_kf = np.concatenate([self.obs_kf, np.full(n_live, j, np.int32)])
            self.obs_tid = np.concatenate([self.obs_tid, self.tr_id])
            self.obs_uv = np.vstack([self.obs_uv, self.tr_uv.astype(np.float64)])
            self.nobs[self.tr_id] += 1
        # new map points: live tracks seen by two keyframes without one
        cand = self.tr_id[(self.nobs[self.tr_id] >= 2) & (self.pt_of[self.tr_id] < 0)] if n_live else self.tr_id
        if len(cand) and j >= 1:
            P = np.stack([self.K @ np.hstack([_rodrigues(r), tt.reshape(3, 1)]) for r, tt in zip(self.kf_rot, self.kf_t)])
            c0 = self.first_kf[cand]
            c1 = np.full(len(cand), j, np.int32)
            uv0 = self.first_uv[cand]
            uv1 = self.tr_uv[(self.nobs[self.tr_id] >= 2) & (self.pt_of[self.tr_id] < 0)].astype(np.float64)
            Xn = triangulate_points(c0, c1, uv0, uv1, P, device=self.device)
            ok = np.ones(len(cand), bool)
            for cam, uvs in ((c0, uv0), (c1, uv1)):
                Rm = np.stack([_rodrigues(self.kf_rot[c]) for c in range(len(self.kf_rot))])[cam]
                Tm = np.stack(self.kf_t)[cam]
                Xc = np.einsum("nij,nj->ni", Rm, Xn) + Tm
                proj = Xc[:, :2] / Xc[:, 2:] * F_PIX + self.video.c
                err = np.linalg.norm(proj - uvs, axis=1)
                ok &= (Xc[:, 2] > 0) & (err <= 7.0) & np.isfinite(err)
            new = cand[ok]
            self.pt_of[new] = self.X.shape[0] + np.arange(len(new))
            self.X = np.vstack([self.X, Xn[ok]])
        # replenish: new corners away from the live tracks
        corners = self.tracker.detect_features()
        if len(corners) and len(self.tr_uv) < self.max_tracks:
            if len(self.tr_uv):
                d2 = ((corners[:, None, :] - self.tr_uv[None, :, :]) ** 2).sum(-1).min(axis=1)
                corners = corners[d2 >= self.min_track_dist ** 2]
            corners = corners[: self.max_tracks - len(self.tr_uv)]
            ids = np.arange(self.next_id, self.next_id + len(corners))
            self.next_id += len(corners)
            # a new track's first keyframe observation is this keyframe
            self.pt_of = np.concatenate([self.pt_of, np.full(len(ids), -1, np.int64)])
            self.first_kf = np.concatenate([self.first_kf, np.full(len(ids), j, np.int32)])
            self.first_uv = np.vstack([self.first_uv, corners.astype(np.float64)])
            self.nobs = np.concatenate([self.nobs, np.ones(len(ids), np.int32)])
            self.obs_kf = np.concatenate([self.obs_kf, np.full(len(ids), j, np.int32)])
            self.obs_tid = np.concatenate([self.obs_tid, ids])
            self.obs_uv = np.vstack([self.obs_uv, corners.astype(np.float64)])
            self.tr_uv = np.vstack([self.tr_uv, corners]).astype(np.float32)
            self.tr_id = np.concatenate([self.tr_id, ids])
        if j >= 1 and self.X.shape[0]:
            t3 = time.perf_counter()
            self._bundle_adjust()
            self.times["ba"] += time.perf_counter() - t3

    def _bundle_adjust(self) -> None:
        """CSfM::bundleAdjustment over every keyframe (frame-major gather)."""
        # observations are appended keyframe by keyframe: the mask keeps the
        # frame-major order of CSfM::bundleAdjustment's gather
        pid = self.pt_of[self.obs_tid]
        m = pid >= 0
        uv = np.ascontiguousarray(self.obs_uv[m])
        cam = np.ascontiguousarray(self.obs_kf[m])
        pt = np.ascontiguousarray(pid[m].astype(np.int32))
        C = len(self.kf_frames)
        K9 = np.tile(self.K.reshape(1, 9), (C, 1))
        rot = np.stack(self.kf_rot)
        t = np.stack(self.kf_t)
        X = self.X.copy()
        rec = {"uv": uv, "cam_idx": cam, "pt_idx": pt, "K": K9, "rot": rot.copy(), "t": t.copy(), "X": X.copy()}
        sm, tr = _ba.solve(uv, cam, pt, K9, rot, t, X)
        rec.update({"summary": sm, "trace": tr, "rot_out": rot.copy(), "t_out": t.copy(), "X_out": X.copy()})
        self.ba_log.append(rec)
        self.kf_rot = [r.copy() for r in rot]
        self.kf_t = [x.copy() for x in t]
        self.X = X
        # the next frames' PnP continues from the adjusted last keyframe
        # (CSfM.cpp:261: _prevFrame.setPose of the last keyframe)
        self.pose = (rot[-1].copy(), t[-1].copy())

    def close(self) -> None:
        self.tracker.close()
