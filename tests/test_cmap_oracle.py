"""CPU: the CMap restatement (oracle/cmap_oracle.py) on hand-checked cases of
the reference's container semantics (/root/reference/CMap.cpp:36-132,
225-295, 308-381), and the map store's C ABI on the no-device path."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.cmap_oracle import CMapOracle  # noqa: E402


def _map():
    m = CMapOracle(desc_bytes=8)
    # two new points seen by frames 10 and 20 (2D indices per frame)
    m.addNewPoints([[0, 0, 1], [1, 0, 1]], [[5, 6], [7, 8]], [10, 20])
    # a third point seen by frame 20 only
    m.addNewPoints([[2, 0, 1]], [[9]], [20])
    return m


def test_emplace_order_is_point_major():
    m = _map()
    # CMap.cpp:50-66: point 0 (frames 10, 20), point 1 (10, 20), point 2 (20)
    assert m.mm == [(10, 0), (20, 0), (10, 1), (20, 1), (20, 2)]
    assert m.frameNo[0] == [10, 20] and m.pts2DIdx[0] == [5, 7]
    assert m.frameNo[1] == [10, 20] and m.pts2DIdx[1] == [6, 8]


def test_points_in_frame_keeps_equal_range_order():
    m = _map()
    m.addPointMatches([2, 0], [11, 12], 30)
    assert m.getPointsInFrame(20) == ([0, 1, 2], [7, 8, 9])
    assert m.getPointsInFrame(30) == ([2, 0], [11, 12])   # insertion order, not sorted
    assert m.getPointsInFrame(99) == ([], [])


def test_point_matched_twice_in_a_frame_pushes_every_2d_index_per_entry():
    m = _map()
    m.addPointMatches([1, 1], [40, 41], 30)
    # two equal_range entries for point 1, each pushing both 2D indices
    assert m.getPointsInFrame(30) == ([1, 1], [40, 41, 40, 41])


def test_points_in_frames_sorted_unique():
    m = _map()
    m.addPointMatches([2, 0], [11, 12], 30)
    assert m.getPointsInFrames([30, 10]) == [0, 1, 2]
    assert m.getPointsInFrames([30]) == [0, 2]
    assert m.getPointsInFrames([]) == []


def test_representative_descriptor_first_minimum():
    m = _map()
    a = np.zeros(8, np.uint8)
    b = np.zeros(8, np.uint8); b[0] = 0b11
    c = np.zeros(8, np.uint8); c[0] = 0b01
    m.addDescriptors([0, 0, 0], [a, b, c])
    # sums: a: 0+2+1 = 3, b: 2+0+1 = 3, c: 1+1+0 = 2 -> c
    best, rows = m.getRepresentativeDescriptors([0])
    assert best.tolist() == [2] and (rows[0] == c).all()
    m.addDescriptors([1, 1], [a, b])  # tie (2, 2): the first row
    best, _ = m.getRepresentativeDescriptors([1])
    assert best.tolist() == [0]


def test_map_store_fails_loudly_without_a_device():
    import sfm_amd
    if sfm_amd.device_count() > 0:
        pytest.skip("a device is present")
    with pytest.raises(Exception):
        sfm_amd.DeviceMap(64)
