"""GPU: the device map store (sfm_map_*, map_store.hip) against the CMap
restatement (oracle/cmap_oracle.py) on seeded histories shaped like the
tracking path's: keyframes adding new points seen by 2 frames, point
matches (some points matched twice in one frame, the multimap quirk),
descriptor rows per keyframe; every query compared exactly."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.cmap_oracle import CMapOracle  # noqa: E402

pytestmark = pytest.mark.gpu


def _history(seed, n_kf=12, desc_bytes=64, new_per_kf=300, dup=True):
    import sfm_amd
    rng = np.random.default_rng(seed)
    dm = sfm_amd.DeviceMap(desc_bytes)
    om = CMapOracle(desc_bytes)
    frames = []
    for k in range(n_kf):
        f = 10 * k + 3
        frames.append(f)
        n_pts = len(om.pts3D)
        if k >= 1:
            # new points triangulated between the previous and this keyframe
            X = rng.normal(size=(new_per_kf, 3))
            i2 = rng.integers(0, 2000, size=(2, new_per_kf)).astype(np.int32)
            fr = [frames[-2], f]
            a = dm.addNewPoints(X, i2, fr)
            b = om.addNewPoints(X, i2, fr)
            assert a.tolist() == b
            d = rng.integers(0, 256, size=(new_per_kf, desc_bytes), dtype=np.uint8)
            dm.addDescriptors(a, d)
            om.addDescriptors(b, d)
            d2 = d.copy()
            flips = rng.integers(0, desc_bytes, size=new_per_kf)
            d2[np.arange(new_per_kf), flips] ^= 0x5A
            dm.addDescriptors(a, d2)
            om.addDescriptors(b, d2)
        if n_pts:
            # matches of existing points in this keyframe (random subset,
            # random order), a few matched twice
            m = int(min(n_pts, 200))
            idx = rng.choice(n_pts, size=m, replace=False).astype(np.int32)
            if dup and m > 4:
                idx = np.concatenate([idx, idx[:3]])
            i2 = rng.integers(0, 2000, size=len(idx)).astype(np.int32)
            dm.addPointMatches(idx, i2, f)
            om.addPointMatches(idx, i2, f)
            d = rng.integers(0, 256, size=(len(idx), desc_bytes), dtype=np.uint8)
            dm.addDescriptors(idx, d)
            om.addDescriptors(idx, d)
    return dm, om, frames


@pytest.mark.parametrize("seed", [0, 1])
def test_map_queries_match_the_cmap_restatement(seed):
    dm, om, frames = _history(seed)
    try:
        n_pts, n_obs, n_rows = dm.size()
        assert n_pts == len(om.pts3D) and n_obs == len(om.mm)
        for f in frames + [999]:
            p3, p2 = dm.getPointsInFrame(f)
            q3, q2 = om.getPointsInFrame(f)
            assert p3.tolist() == q3 and p2.tolist() == q2, f
        rng = np.random.default_rng(seed + 100)
        for _ in range(5):
            sel = rng.choice(frames, size=rng.integers(1, len(frames)), replace=False).tolist() + [12345]
            assert dm.getPointsInFrames(sel).tolist() == om.getPointsInFrames(sel)
        allp = np.arange(n_pts, dtype=np.int32)
        q = rng.permutation(allp)[: min(500, n_pts)]
        rows, best = dm.getRepresentativeDescriptors(q, return_best=True)
        ob, orows = om.getRepresentativeDescriptors(q.tolist())
        assert best.tolist() == ob.tolist()
        assert (rows == orows).all()
        np.testing.assert_array_equal(dm.getPointsAtIdx(q), om.getPointsAtIdx(q.tolist()))
    finally:
        dm.close()


def test_duplicate_match_quirk_on_the_device():
    import sfm_amd
    dm = sfm_amd.DeviceMap(64)
    try:
        dm.addNewPoints(np.zeros((3, 3)), [[5, 6, 7], [8, 9, 10]], [10, 20])
        dm.addPointMatches([1, 1, 0], [40, 41, 42], 30)
        p3, p2 = dm.getPointsInFrame(30)
        assert p3.tolist() == [1, 1, 0] and p2.tolist() == [40, 41, 40, 41, 42]
        assert dm.getPointsInFrames([30]).tolist() == [0, 1]
        p3, p2 = dm.getPointsInFrame(20)
        assert p3.tolist() == [0, 1, 2] and p2.tolist() == [8, 9, 10]
    finally:
        dm.close()


def test_points_in_frame_when_2d_list_outgrows_observations():
    """n2 = sum of k^2 over a frame's points can exceed n_obs."""
    import sfm_amd
    from oracle.cmap_oracle import CMapOracle
    dm = sfm_amd.DeviceMap(64)
    om = CMapOracle()
    try:
        for m in (dm, om):
            m.addNewPoints(np.zeros((1, 3)), [[5], [6]], [10, 20])
            m.addPointMatches([0, 0, 0], [40, 41, 42], 30)
        assert dm.size()[1] == 5
        p3, p2 = dm.getPointsInFrame(30)
        o3, o2 = om.getPointsInFrame(30)
        assert p3.tolist() == list(o3) == [0, 0, 0]
        assert p2.tolist() == list(o2) == [40, 41, 42] * 3
    finally:
        dm.close()


def test_points_in_frame_multi_equals_per_frame_queries():
    """The one-call BA gather (sfm_map_points_in_frame_multi) against one
    getPointsInFrame per frame and the oracle, duplicates included."""
    import sfm_amd
    from oracle.cmap_oracle import CMapOracle
    rng = np.random.default_rng(3)
    dm = sfm_amd.DeviceMap(64)
    om = CMapOracle()
    try:
        pts, p2d = rng.normal(0, 1, (40, 3)), rng.integers(0, 500, (2, 40))
        for m in (dm, om):
            m.addNewPoints(pts, p2d, [0, 10])
        for f in (20, 30):
            idx = rng.choice(40, 25, replace=False)
            p2 = rng.integers(0, 500, 25)
            for m in (dm, om):
                m.addPointMatches(idx, p2, f)
        for m in (dm, om):
            m.addPointMatches([3, 3, 7], [1, 2, 3], 30)
        frames = [30, 0, 20, 10, 99]
        multi = dm.getPointsInFrameMulti(frames)
        for f, (a3, a2) in zip(frames, multi):
            b3, b2 = dm.getPointsInFrame(f)
            o3, o2 = om.getPointsInFrame(f)
            assert a3.tolist() == b3.tolist() == list(o3)
            assert a2.tolist() == b2.tolist() == list(o2)
        assert len(multi[-1][0]) == 0
        with pytest.raises(Exception):
            dm.getPointsInFrameMulti([10, 10])
    finally:
        dm.close()


def test_set_points_round_trip_and_errors():
    import sfm_amd
    dm = sfm_amd.DeviceMap(64)
    try:
        dm.addNewPoints(np.arange(12, dtype=float).reshape(4, 3), [[0, 1, 2, 3]], [7])
        dm.setPointsAtIdx([2], [[9.0, 8.0, 7.0]])
        np.testing.assert_array_equal(dm.getPointsAtIdx([2, 0]), [[9, 8, 7], [0, 1, 2]])
        with pytest.raises(Exception):
            dm.addPointMatches([4], [0], 8)           # no point 4
        with pytest.raises(Exception):
            dm.getRepresentativeDescriptors([1])      # no descriptor row yet
        assert dm.getPointsInFrames([]).tolist() == []
    finally:
        dm.close()
