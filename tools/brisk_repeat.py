"""Repeatability of the device BRISK keypoints on the rendered video: the
keypoints of frame k0 mapped into frame k1 by the video's true similarity,
against the nearest keypoint detected in k1, per pyramid layer.
    python tools/brisk_repeat.py [k0 k1 threshold]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from sfm_amd import brisk
from sfm_amd.video import SyntheticVideo


def main():
    k0, k1, thr = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (0, 5, 60)))
    v = SyntheticVideo(speed=2.0)
    a, la, _ = brisk.detect(v.frame(k0), thr, 6)
    b, lb, _ = brisk.detect(v.frame(k1), thr, 6)
    pa = v.map_points(k0, k1, a[:, :2].astype(np.float64))
    inside = (pa[:, 0] > 20) & (pa[:, 0] < v.w - 20) & (pa[:, 1] > 20) & (pa[:, 1] < v.h - 20)
    print(f"frames {k0}->{k1} thr {thr}: {len(a)} / {len(b)} keypoints")
    for layer in range(12):
        sel = inside & (la == layer)
        if not sel.any():
            continue
        d2 = ((pa[sel, None, :] - b[None, :, :2]) ** 2).sum(-1)
        j = d2.argmin(1)
        d = np.sqrt(d2.min(1))
        same = lb[j] == layer
        print(f"layer {layer:2d}: n {sel.sum():5d}  nn dist median {np.median(d):6.3f} p25 {np.percentile(d, 25):6.3f} "
              f"<0.5px {np.mean(d < 0.5):.2f} <1px {np.mean(d < 1):.2f} <2px {np.mean(d < 2):.2f}  "
              f"same layer {np.mean(same):.2f}  size {np.median(a[sel, 2]):.1f}")


if __name__ == "__main__":
    main()
