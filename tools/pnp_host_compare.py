"""Compare the host build of the device EPnP (tools/pnp_host_check) with the
oracle's epnp on every subset of the oracle's RANSAC trace (CPU only)."""
import os, subprocess, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import pnp_oracle as P
from tests.pnp_cases import CASES, K, scene

EXE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pnp_host_check")
for case in CASES:
    n, seed, noise, outl, planar = case
    X, uv, rv, tv = scene(n, seed, noise=noise, outliers=outl, planar=planar)
    tr = []
    P.solve_pnp_ransac(X, uv, K, trace=tr)
    Xf, uf = X.astype(np.float32), uv.astype(np.float32)
    worst = 0.0
    for it, (sub, r, t, good) in enumerate(tr):
        inp = f"{float(K[0,0])!r} {float(K[1,1])!r} {float(K[0,2])!r} {float(K[1,2])!r} 5\n" + "".join(
            f"{float(Xf[q,0])!r} {float(Xf[q,1])!r} {float(Xf[q,2])!r} {float(uf[q,0])!r} {float(uf[q,1])!r}\n"
            for q in sub)
        out = subprocess.run([EXE], input=inp, capture_output=True, text=True).stdout.split()
        v = np.array([float(x) for x in out])
        Ro, to = P.epnp(K, Xf[sub], uf[sub])
        d = max(np.abs(v[:9].reshape(3, 3) - Ro).max(), np.abs(v[9:] - to).max())
        worst = max(worst, d)
    print(case, "iters", len(tr), "worst |host - oracle|", worst)
