"""CPU: the CMap::getRepresentativeDescriptors restatement (oracle/
match_oracle.cpp; /root/reference/CMap.cpp:345-381) against an independent
numpy one: full distance matrices, column sums, first minimum."""
import numpy as np

from oracle import ffi as O


def numpy_repr(desc, row_off):
    bits = np.unpackbits(desc, axis=1).astype(np.int64)
    out = []
    for i in range(len(row_off) - 1):
        b = bits[row_off[i]:row_off[i + 1]]
        d = (b[:, None, :] != b[None, :, :]).sum(axis=2)
        out.append(int(np.argmin(d.sum(axis=0))))   # argmin: first minimum
    return np.array(out, np.int32)


def _case(seed, n, kmax, nbytes=64, dup=False):
    rng = np.random.default_rng(seed)
    ks = rng.integers(1, kmax + 1, n)
    row_off = np.concatenate([[0], np.cumsum(ks)]).astype(np.int32)
    desc = rng.integers(0, 256, (row_off[-1], nbytes), dtype=np.uint8)
    if dup:  # engineered ties: each point's rows are two alternating patterns
        for i in range(n):
            a, b = desc[row_off[i]], desc[row_off[i]] ^ 0x0F
            for r in range(row_off[i], row_off[i + 1]):
                desc[r] = a if (r - row_off[i]) % 2 == 0 else b
    return desc, row_off


def test_repr_matches_numpy_random():
    desc, off = _case(1, 300, 20)
    assert np.array_equal(O.representative_descriptors(desc, off), numpy_repr(desc, off))


def test_repr_ties_first_minimum_and_single_rows():
    desc, off = _case(2, 100, 9, dup=True)
    got = O.representative_descriptors(desc, off)
    assert np.array_equal(got, numpy_repr(desc, off))
    desc1, off1 = _case(3, 50, 1)
    assert np.all(O.representative_descriptors(desc1, off1) == 0)


def test_repr_other_width():
    desc, off = _case(4, 80, 30, nbytes=32)
    assert np.array_equal(O.representative_descriptors(desc, off), numpy_repr(desc, off))
