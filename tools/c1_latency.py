"""C1 keyframe-sized one-shot solve latency (bench incremental_ba leg): wall
time per sfm_ba_solve, and with --trace the kernel / copy timeline of the
last solve from a rocprofv3 kernel + memory-copy trace directory.
    python tools/c1_latency.py                 # timing only
    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -- python3 tools/c1_latency.py
    python tools/c1_latency.py --summarise DIR"""
import glob
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run():
    import numpy as np
    import sfm_amd
    from sfm_amd import scene as S
    sc = S.config("C1")
    walls = []
    for k in range(30):
        r, t, X = sc.rot.copy(), sc.t.copy(), sc.X.copy()
        t0 = time.perf_counter()
        sm, _ = sfm_amd.solve(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, r, t, X)
        walls.append(time.perf_counter() - t0)
    w = np.array(walls[5:]) * 1e3
    print(f"C1 one-shot: median {np.median(w):.3f} ms, min {w.min():.3f} ms, iterations {sm.num_iterations}")
    # the same call through the C ABI alone (arguments prepared once, the
    # parameters reset by copyto outside the clock): what a C++ caller sees
    import ctypes
    from sfm_amd import ba as B
    L = B.lib()
    opts, smr = B.default_options(), B.BASummary()
    tr, tl = (B.BAIteration * 128)(), ctypes.c_int32(0)
    r, t, X = sc.rot.copy(), sc.t.copy(), sc.X.copy()
    uv, ci, pi, K = B._f64(sc.uv), B._i32(sc.cam_idx), B._i32(sc.pt_idx), B._f64(sc.K)
    args = (ctypes.byref(opts), B.STRUCT_AND_POSE, int(uv.shape[0]), B.ptr(uv), B.ptr(ci), B.ptr(pi), int(r.shape[0]), B.ptr(K),
            B.ptr(r), B.ptr(t), int(X.shape[0]), B.ptr(X), ctypes.byref(smr), tr, 128, ctypes.byref(tl))
    raw = []
    for k in range(30):
        np.copyto(r, sc.rot); np.copyto(t, sc.t); np.copyto(X, sc.X)
        t0 = time.perf_counter()
        rc = L.sfm_ba_solve(*args)
        raw.append(time.perf_counter() - t0)
        assert rc == 0
    w = np.array(raw[5:]) * 1e3
    print(f"C1 one-shot, C ABI call only: median {np.median(w):.3f} ms, min {w.min():.3f} ms")
    ba = sfm_amd.BundleAdjuster(0)
    ts, tv, tg = [], [], []
    for k in range(30):
        t0 = time.perf_counter()
        ba.set_problem(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, sc.rot, sc.t, sc.X)
        t1 = time.perf_counter()
        sm, _ = ba.solve()
        t2 = time.perf_counter()
        ba.parameters()
        t3 = time.perf_counter()
        ts.append(t1 - t0); tv.append(t2 - t1); tg.append(t3 - t2)
    f = lambda a: float(np.median(np.array(a[5:]) * 1e3))
    print(f"resident: set_problem {f(ts):.3f} ms, solve {f(tv):.3f} ms, get_parameters {f(tg):.3f} ms")
    ba.close()


def summarise(d):
    import csv
    kf = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)
    mf = glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True)
    ev = []
    for f in kf:
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("sfm::", "")
            n = n.split("(")[0] if not n.startswith("void rocprim") else "rocprim " + n.split("detail::")[2][:30]
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + n[:44]))
    for f in mf:
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C " + r.get("Direction", "copy")))
    ev.sort()
    # the last 25 solves (the first 5 are warm-up): per-solve averages
    nsolve = 25
    per = len(ev) // 30
    last = ev[len(ev) - per * nsolve:]
    t0 = last[0][0]
    busy = sum(e[1] - e[0] for e in last)
    print(f"per solve: {len(last) / nsolve:.0f} events, span {(last[-1][1] - t0) / 1e3 / nsolve:.1f} us, "
          f"busy {busy / 1e3 / nsolve:.1f} us")
    kinds = {}
    for s_, e_, n in last:
        kinds.setdefault(n, [0, 0])
        kinds[n][0] += 1
        kinds[n][1] += e_ - s_
    for n, (c, tt) in sorted(kinds.items(), key=lambda x: -x[1][1])[:30]:
        print(f"  {n:46s} x{c / nsolve:5.1f} {tt / 1e3 / nsolve:8.1f} us")
    prev = t0
    gaps = []
    for s_, e_, n in last:
        gaps.append((s_ - prev, n))
        prev = max(prev, e_)
    gaps.sort(reverse=True)
    print("gap total per solve (us):", round(sum(g for g, _ in gaps) / 1e3 / nsolve, 1))
    print("largest gaps before:", [(round(g / 1e3, 1), n) for g, n in gaps[:12]])
    # the last resident solve in order: from the event after its set_problem's
    # last host-to-device copy to the parameters' download
    k = len(ev) - 1
    while k > 0 and ev[k][2] != "C MEMORY_COPY_HOST_TO_DEVICE":
        k -= 1
    seq = ev[k + 1:]
    t0 = seq[0][0] if seq else 0
    print("last solve timeline (start us, duration us, gap before us):")
    prev = t0
    for s_, e_, n in seq:
        print(f"  {(s_ - t0) / 1e3:8.1f} {(e_ - s_) / 1e3:7.1f} {(s_ - prev) / 1e3:6.1f}  {n}")
        prev = max(prev, e_)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarise":
        summarise(sys.argv[2])
    else:
        run()
