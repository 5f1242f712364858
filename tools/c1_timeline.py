"""Device timeline of the resident C1 solve (sfm_ba_solve_resident): how much
of the call is kernel time, how much dispatch gaps between dependent
kernels, how much host time before the first / after the last kernel.
  cd /tmp && SFM_ROCTX=1 rocprofv3 --marker-trace --kernel-trace --output-format csv \
      -d $R/gpurun_out/c1tl -- python3 $R/tools/c1_timeline.py
  python3 tools/c1_timeline.py --summarise gpurun_out/c1tl"""
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run():
    import sfm_amd
    from sfm_amd import scene as S
    sc = S.config("C1")
    ba = sfm_amd.BundleAdjuster(0)
    ba.set_problem(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, sc.rot, sc.t, sc.X)
    for _ in range(40):
        ba.reset()
        sm, _ = ba.solve()
    print("iterations", sm.num_iterations)
    ba.close()


def summarise(d):
    import csv
    import numpy as np
    ks, ms = [], []
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("sfm::", "").split("(")[0]
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n[:40]))
    for f in glob.glob(d + "/**/*marker*.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "sfm_ba_solve_resident" in (r.get("Function", "") + r.get("Marker_Name", "") + r.get("Name", "")):
                ms.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    ks.sort()
    ms.sort()
    rows = []
    for a, b in ms[10:]:
        kk = [k for k in ks if a <= k[0] < b]
        if not kk:
            continue
        busy = sum(e - s for s, e, _ in kk)
        gaps = sum(max(0, kk[i + 1][0] - kk[i][1]) for i in range(len(kk) - 1))
        rows.append(((b - a) / 1e3, len(kk), busy / 1e3, gaps / 1e3, (kk[0][0] - a) / 1e3, (b - kk[-1][1]) / 1e3,
                     (kk[-1][1] - kk[0][0]) / 1e3))
    r = np.median(np.array(rows), axis=0)
    print(f"resident C1 solves: {len(rows)} (median)")
    print(f"  call {r[0]:.1f} us, kernels {r[1]:.0f}, kernel time {r[2]:.1f} us, gaps between kernels {r[3]:.1f} us")
    print(f"  call start -> first kernel {r[4]:.1f} us, last kernel end -> call end {r[5]:.1f} us, "
          f"first kernel start -> last kernel end {r[6]:.1f} us")
    a, b = ms[-1]
    kk = [k for k in ks if a <= k[0] < b]
    print("last solve:")
    prev = None
    for s, e, n in kk:
        g = (s - prev) / 1e3 if prev is not None else (s - a) / 1e3
        print(f"  +{(s - a) / 1e3:7.1f} us  gap {g:5.1f}  dur {(e - s) / 1e3:6.1f}  {n}")
        prev = e


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarise":
        summarise(sys.argv[2])
    else:
        run()
