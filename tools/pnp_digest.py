"""Bit-level digest of the device solvePnPRansac on the test scenes (and the
bench leg's scene): the found flags, inlier lists and the exact bytes of
every pose.  Two library builds whose digests agree compute bitwise the same
poses (used by A/B runs: SFM_AMD_LIB=... python tools/pnp_digest.py, and
pinned by tests/test_gpu_pnp.py)."""
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def digest():
    import sfm_amd
    from tests.pnp_cases import CASES, K, scene
    h = hashlib.sha256()
    cases = list(CASES) + [(500, 77, 0.5, 0.3, False)]
    for n, seed, noise, outl, planar in cases:
        X, uv, _, _ = scene(n, seed, noise=noise, outliers=outl, planar=planar)
        ok, r, t, inl = sfm_amd.solvePnPRansac(X, uv, K)
        h.update(np.array([ok, len(inl)], np.int64).tobytes())
        h.update(np.asarray(inl, np.int64).tobytes())
        h.update(np.asarray(r, np.float64).tobytes() + np.asarray(t, np.float64).tobytes())
    return h.hexdigest()[:16], len(cases)


if __name__ == "__main__":
    d, n = digest()
    print("pnp_digest", d, "cases", n)
