"""CPU: the row-parallel Jacobi schedule of the PnP 12x12 SVD
(sfm_amd/csrc/pnp_kernels.hip, kSvdN / kSvdI / kSvdJ) is OpenCV's sweep
(JacobiSVDImpl_: pairs (i, j), i < j, i-major) regrouped without changing
any row's sequence of rotations: every pair exactly once, the rotations of a
pass on disjoint rows, and for each row its rotations in sequential order.
Those three properties make the device sweep bitwise the sequential one
(tests/test_gpu_pnp.py checks the result against the oracle on the GPU)."""
import os
import re

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sfm_amd", "csrc", "pnp_kernels.hip")


def _array(src, name):
    m = re.search(name + r"\[[^\]]*\](?:\[4\])?\s*=\s*\{(.*?)\};", src, re.S)
    assert m, name
    return [int(x) for x in re.findall(r"-?\d+", m.group(1))]


def test_schedule_is_opencv_order_regrouped():
    src = open(SRC).read()
    npass = int(re.search(r"kSvdPasses\s*=\s*(\d+)", src).group(1))
    n = _array(src, "kSvdN")
    I = _array(src, "kSvdI")
    J = _array(src, "kSvdJ")
    assert len(n) == npass and len(I) == 4 * npass and len(J) == 4 * npass
    rots = []
    for p in range(npass):
        assert 1 <= n[p] <= 4
        pas = [(I[4 * p + q], J[4 * p + q]) for q in range(n[p])]
        rows = [r for ij in pas for r in ij]
        assert len(rows) == len(set(rows)), (p, pas)  # disjoint rows within a pass
        rots += pas
    seq = [(i, j) for i in range(11) for j in range(i + 1, 12)]
    assert sorted(rots) == sorted(seq) and len(rots) == 66
    for r in range(12):  # each row sees its rotations in OpenCV's order
        assert [ij for ij in rots if r in ij] == [ij for ij in seq if r in ij], r
