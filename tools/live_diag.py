"""Diagnostics of the live loop on device BRISK detections (tests/test_gpu_live.py
run_brisk): per keyframe BA the problem size, LM iterations, residual
distribution at the solution, and the keyframe motion against the video's
ground truth.   python tools/live_diag.py [n_frames]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from sfm_amd.live import BriskVideoStream, LiveSfM, _project
from sfm_amd.mapping import _rodrigues


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    st = BriskVideoStream()
    s = LiveSfM(st)
    s.run(n)
    print("keyframes", [f.no for f in s.kfs], "stats", s.stats)
    for k, rec in enumerate(s.ba_log):
        sm = rec["summary"]
        K = rec["K"][0].reshape(3, 3)
        res = []
        for c in range(len(rec["rot_out"])):
            m = rec["cam_idx"] == c
            uv, _ = _project(K, rec["rot_out"][c], rec["t_out"][c], rec["X_out"][rec["pt_idx"][m]])
            res.append(np.linalg.norm(uv - rec["uv"][m], axis=1))
        r = np.concatenate(res)
        r0 = []
        for c in range(len(rec["rot"])):
            m = rec["cam_idx"] == c
            uv, _ = _project(K, rec["rot"][c], rec["t"][c], rec["X"][rec["pt_idx"][m]])
            r0.append(np.linalg.norm(uv - rec["uv"][m], axis=1))
        r0 = np.concatenate(r0)
        print(f"BA {k}: cams {len(rec['rot'])} pts {len(rec['X'])} obs {len(rec['uv'])} iters {sm.num_iterations} "
              f"term {sm.termination_type} cost {sm.initial_cost:.1f} -> {sm.final_cost:.1f}; residual px before "
              f"median {np.median(r0):.2f} p99 {np.percentile(r0, 99):.1f} max {r0.max():.1f}; after median "
              f"{np.median(r):.2f} p90 {np.percentile(r, 90):.2f} p99 {np.percentile(r, 99):.1f} >7px {np.mean(r > 7):.3f}")
    C = np.array([-_rodrigues(f.rot).T @ f.t for f in s.kfs])
    Cg = np.array([-_rodrigues(st.pose(f.no)[0]).T @ st.pose(f.no)[1] for f in s.kfs])
    print("centres", np.round(C, 3).tolist())
    print("truth  ", np.round(Cg, 3).tolist())
    s.close()


if __name__ == "__main__":
    main()
