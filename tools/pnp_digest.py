"""Bit-level digest of the device solvePnPRansac on the test scenes (and the
bench leg's scene): the found flags, inlier lists and the exact bytes of
every pose.  Two library builds whose digests agree compute bitwise the same
poses (used by A/B runs: SFM_AMD_LIB=... python tools/pnp_digest.py)."""
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sfm_amd  # noqa: E402
from tests.pnp_cases import CASES, K, scene  # noqa: E402

h = hashlib.sha256()
cases = list(CASES) + [(500, 77, 0.5, 0.3, False)]
for n, seed, noise, outl, planar in cases:
    X, uv, _, _ = scene(n, seed, noise=noise, outliers=outl, planar=planar)
    ok, r, t, inl = sfm_amd.solvePnPRansac(X, uv, K)
    h.update(np.array([ok, len(inl)], np.int64).tobytes())
    h.update(np.asarray(inl, np.int64).tobytes())
    h.update(np.asarray(r, np.float64).tobytes() + np.asarray(t, np.float64).tobytes())
print("pnp_digest", h.hexdigest()[:16], "cases", len(cases))
