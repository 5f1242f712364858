"""GPU: CMap::getRepresentativeDescriptors (CMap.cpp:345-381, SURVEY.md §8f
row 2) through the C ABI, bit-exact against the oracle: random maps, points
with more rows than a wavefront has lanes, engineered ties, single-row
points, 32-byte descriptors, and the error on a point without rows."""
import numpy as np
import pytest

import sfm_amd
from oracle import ffi as O
from tests.test_repr_oracle import _case

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,n,kmax,nbytes,dup", [(1, 2000, 20, 64, False), (2, 300, 9, 64, True),
                                                     (3, 40, 300, 64, False), (4, 500, 1, 64, False),
                                                     (5, 700, 40, 32, False)])
def test_representative_descriptors_bit_exact(seed, n, kmax, nbytes, dup):
    desc, off = _case(seed, n, kmax, nbytes, dup)
    best, out = sfm_amd.representative_descriptors(desc, off)
    ref = O.representative_descriptors(desc, off)
    assert np.array_equal(best, ref)
    assert np.array_equal(out, desc[off[:-1] + ref])


def test_cmap_mirror_and_errors():
    rng = np.random.default_rng(9)
    m = sfm_amd.CMap()
    for _ in range(30):
        m.addPoint(rng.integers(0, 256, (int(rng.integers(1, 12)), 64), dtype=np.uint8))
    m.addDescriptor(3, rng.integers(0, 256, 64, dtype=np.uint8))
    idx = [5, 3, 3, 29, 0]
    got = m.getRepresentativeDescriptors(idx)
    mats = [m._descriptor[i] for i in idx]
    off = np.concatenate([[0], np.cumsum([x.shape[0] for x in mats])]).astype(np.int32)
    ref = O.representative_descriptors(np.vstack(mats), off)
    assert np.array_equal(got, np.vstack(mats)[off[:-1] + ref])
    with pytest.raises(sfm_amd.SfmError):
        sfm_amd.representative_descriptors(np.zeros((2, 64), np.uint8), np.array([0, 2, 2], np.int32))
