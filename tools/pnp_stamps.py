"""Per-phase times of k_pnp_epnp from a stamped variant build (tools/mkvar.sh
with the patch below; abvar/var_stamps.so): wall-clock stamps (100 MHz) per
hypothesis and wave at the start, around the 12x12 SVD, at the end of the
common part, after the beta case's least squares and Gauss-Newton, and at the
end.  Build:  bash tools/mkvar.sh stamps "$(python tools/pnp_stamps.py --patch)" pnp_kernels.hip
Run (GPU): SFM_AMD_LIB=abvar/var_stamps.so python tools/pnp_stamps.py"""
import ctypes
import os
import sys

import numpy as np

PATCH = r'''
s = s.replace("constexpr int kSvdHead", "constexpr int kSvdHead", 1)
hdr = """
__device__ unsigned long long g_pnp_st[256 * 3 * 8];
#if defined(__HIP_DEVICE_COMPILE__)
#define PNP_STAMP(i) do { if ((threadIdx.x & 63) == 0) g_pnp_st[(blockIdx.x * 3 + (threadIdx.x >> 6)) * 8 + (i)] = wall_clock64(); } while (0)
#else
#define PNP_STAMP(i) do {} while (0)
#endif
"""
a = s.index("struct EpnpIn {")
s = s[:a] + hdr + s[a:]
s = s.replace("    cv_svd12_lanes(u, lds, ut);", "    PNP_STAMP(1);\n    cv_svd12_lanes(u, lds, ut);\n    PNP_STAMP(2);", 1)
s = s.replace("    cv_lstsq<6, 4>(A4, rho, b4, lds);", "    cv_lstsq<6, 4>(A4, rho, b4, lds);\n    PNP_STAMP(4);", 1)
s = s.replace("    cv_lstsq<6, 3>(A3, rho, b3, lds);", "    cv_lstsq<6, 3>(A3, rho, b3, lds);\n    PNP_STAMP(4);", 1)
s = s.replace("    cv_lstsq<6, 5>(A5, rho, b5, lds);", "    cv_lstsq<6, 5>(A5, rho, b5, lds);\n    PNP_STAMP(4);", 1)
s = s.replace("    gauss_newton(L, rho, be, lds);\n    return r_and_t", "    gauss_newton(L, rho, be, lds);\n    PNP_STAMP(5);\n    return r_and_t")
s = s.replace("  const int w = threadIdx.x >> 6;\n  EpnpIn in;", "  const int w = threadIdx.x >> 6;\n  PNP_STAMP(0);\n  EpnpIn in;", 1)
s = s.replace("  epnp5_common(in, k, lds[w], cm);\n  double R[9], t[3], r[3];", "  epnp5_common(in, k, lds[w], cm);\n  PNP_STAMP(3);\n  double R[9], t[3], r[3];", 1)
s = s.replace("  const double e = epnp5_case(w, in, k, cm, R, t, lds[w]);", "  const double e = epnp5_case(w, in, k, cm, R, t, lds[w]);\n  PNP_STAMP(6);", 1)
s += """
extern "C" int sfm_pnp_stamps(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(sfm::g_pnp_st), sizeof(unsigned long long) * n) == hipSuccess ? 0 : 1;
}
"""
'''

if __name__ == "__main__":
    if "--patch" in sys.argv:
        print(PATCH)
        sys.exit(0)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import sfm_amd
    from tests.pnp_cases import K, scene
    X, uv, _, _ = scene(500, 77, noise=0.5, outliers=0.3)
    for _ in range(5):
        sfm_amd.solvePnPRansac(X, uv, K)
    lib = sfm_amd.lib()
    st = np.zeros(256 * 3 * 8, np.uint64)
    assert lib.sfm_pnp_stamps(st.ctypes.data_as(ctypes.c_void_p), st.size) == 0
    st = st.reshape(256, 3, 8).astype(np.float64) * 0.01  # 100 MHz -> us
    used = st[:, 0, 0] > 0
    st = st[used]
    names = [(0, 1, "start -> M^T M"), (1, 2, "12x12 SVD"), (2, 3, "rest of common"), (3, 4, "least squares"),
             (4, 5, "Gauss-Newton"), (5, 6, "R, t + error")]
    print(f"k_pnp_epnp phases (us, {len(st)} hypotheses; median / max)")
    for a, b, n in names:
        for w in range(3):
            d = st[:, w, b] - st[:, w, a]
            if n in ("start -> M^T M", "12x12 SVD", "rest of common") and w > 0:
                continue
            print(f"  {n:18s} wave {w}: {np.median(d):7.2f} / {d.max():7.2f}")
    tot = st[:, :, 6].max(axis=1) - st[:, :, 0].min(axis=1)
    print(f"  hypothesis total        {np.median(tot):7.2f} / {tot.max():7.2f}")
