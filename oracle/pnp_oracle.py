"""ORACLE (test infrastructure only -- never imported by the product): a
NumPy restatement of the per-frame pose solve of CSfM::tracking,
cv::solvePnPRansac(currMatch3D, currMatch2D, K, 0, rvec, tvec, false,
iter = 20, reprErr = _maxReprErr = 7, confidence = 0.99, inliers,
SOLVEPNP_ITERATIVE)  (/root/reference/CSfM.cpp:553-565, _maxReprErr at
CSfM.cpp:35).

The arithmetic lives in OpenCV 3.0 (README.md:28), which is absent here
(SURVEY.md §8c), so this restates the published 3.0.0 sources
(modules/calib3d/src/solvepnp.cpp, ptsetreg.cpp, epnp.cpp, calibration.cpp)
as the build reads them -- PARITY UNPINNED against OpenCV itself:

* inputs converted to float32 (solvePnPRansac converts CV_64F point sets);
* RANSAC (RANSACPointSetRegistrator::run) with cv::RNG(uint64(-1)): subsets
  of 5 distinct uniform draws (getSubset), the kernel = EPnP on the subset
  (SOLVEPNP_EPNP: undistortPoints to normalised float coordinates, then
  epnp::compute_pose), the error of a point = float distance between its
  image point and the projection of its object point through
  Rodrigues(rvec) (PnPRansacCallback::computeError), an inlier when that
  DISTANCE is <= reprErr^2 (findInliers squares the threshold: the 3.0
  behaviour), a model kept when its inlier count exceeds max(best, 4), and
  the iteration bound shrunk by RANSACUpdateNumIters(confidence, outlier
  ratio, 5, bound);
* output = the best RANSAC model (in 3.0 the final solvePnP over the inliers
  only decides the return value; its pose is not what is returned) and the
  inlier indices of its mask.  Fewer than 5 points: no model (3.0 switches
  to P3P at exactly 4 points; not restated).
Linear algebra follows OpenCV's own routines (cv::SVD = JacobiSVDImpl_,
cv::solve / cv::invert DECOMP_SVD = SVBkSb, epnp::qr_solve) in their
operation order, so the device kernel (pnp_kernels.hip, same routines) and
this restatement agree to rounding even where EPnP's 5-point problem is
ill-conditioned (the near-null space of M^T M).  Rodrigues matrix->vector is
restated without the SVD re-orthogonalisation OpenCV applies first (a
rounding-level difference), in the product too.
"""
from __future__ import annotations

import math

import numpy as np

U64 = (1 << 64) - 1


class CvRNG:
    """cv::RNG: multiply-with-carry, state = (uint32)state * 4164903690 + (state >> 32)."""

    def __init__(self, state: int = U64):
        self.state = state if state else 0xFFFFFFFF

    def next(self) -> int:
        self.state = ((self.state & 0xFFFFFFFF) * 4164903690 + (self.state >> 32)) & U64
        return self.state & 0xFFFFFFFF

    def uniform(self, a: int, b: int) -> int:
        return a if a == b else int(self.next() % (b - a) + a)


def get_subset(rng: CvRNG, count: int, model_points: int = 5, max_attempts: int = 10000):
    """RANSACPointSetRegistrator::getSubset with checkPartialSubsets = false and
    the default checkSubset (always true): model_points distinct draws."""
    idx = []
    for _ in range(model_points):
        while True:
            v = rng.uniform(0, count)
            if v not in idx:
                break
        idx.append(v)
    return idx


def ransac_update_num_iters(p: float, ep: float, model_points: int, max_iters: int) -> int:
    p = min(max(p, 0.0), 1.0)
    ep = min(max(ep, 0.0), 1.0)
    num = max(1.0 - p, np.finfo(float).tiny)
    denom = 1.0 - math.pow(1.0 - ep, model_points)
    if denom < np.finfo(float).tiny:
        return 0
    num = math.log(num)
    denom = math.log(denom)
    if denom >= 0 or -num >= max_iters * (-denom):
        return max_iters
    return int(np.rint(num / denom))  # cvRound: round half to even


def rodrigues_v2m(r):
    """cvRodrigues2 vector -> matrix: c I + (1 - c) u u^T + s [u]x, u = r / |r|
    (as r * (1/|r|)), summed elementwise in that order (cv::Matx33d)."""
    r0, r1, r2 = (float(x) for x in r)
    th = math.sqrt(r0 * r0 + r1 * r1 + r2 * r2)
    if th < np.finfo(float).eps:
        return np.eye(3)
    c, s = math.cos(th), math.sin(th)
    c1 = 1.0 - c
    it = 1.0 / th
    x, y, z = r0 * it, r1 * it, r2 * it
    return np.array([[c + c1 * (x * x), c1 * (x * y) + s * -z, c1 * (x * z) + s * y],
                     [c1 * (x * y) + s * z, c + c1 * (y * y), c1 * (y * z) + s * -x],
                     [c1 * (x * z) + s * -y, c1 * (y * z) + s * x, c + c1 * (z * z)]])


def rodrigues_m2v(R):
    """cvRodrigues2 matrix -> vector (without the SVD re-orthogonalisation)."""
    R = [[float(x) for x in row] for row in np.asarray(R, np.float64)]
    rx, ry, rz = R[2][1] - R[1][2], R[0][2] - R[2][0], R[1][0] - R[0][1]
    s = math.sqrt((rx * rx + ry * ry + rz * rz) * 0.25)
    c = (R[0][0] + R[1][1] + R[2][2] - 1.0) * 0.5
    c = 1.0 if c > 1.0 else (-1.0 if c < -1.0 else c)
    th = math.acos(c)
    if s < 1e-5:
        if c > 0:
            return np.zeros(3)
        t = (R[0][0] + 1) * 0.5
        rx = math.sqrt(max(t, 0.0))
        t = (R[1][1] + 1) * 0.5
        ry = math.sqrt(max(t, 0.0)) * (-1.0 if R[0][1] < 0 else 1.0)
        t = (R[2][2] + 1) * 0.5
        rz = math.sqrt(max(t, 0.0)) * (-1.0 if R[0][2] < 0 else 1.0)
        if abs(rx) < abs(ry) and abs(rx) < abs(rz) and (R[1][2] > 0) != (ry * rz > 0):
            rz = -rz
        k = th / math.sqrt(rx * rx + ry * ry + rz * rz)
        return np.array([rx * k, ry * k, rz * k])
    k = th / (2.0 * s)
    return np.array([rx * k, ry * k, rz * k])


# ---- cv::SVD as OpenCV 3.0 computes it (lapack.cpp JacobiSVDImpl_,
# SVBkSbImpl_): one-sided Jacobi on the rows of At = A^T, eps = 10
# DBL_EPSILON, max(m, 30) sweeps, singular values sorted descending, zero
# singular values completed by cv::RNG(0x12345678) vectors; the
# back-substitution drops w_i <= 2 DBL_EPSILON sum(w).  Scalar Python loops in
# OpenCV's operation order (no fused multiply-adds, as an SSE2 build).
DBL_EPS = np.finfo(float).eps
DBL_MIN = np.finfo(float).tiny


def tree16(v):
    """The 16-lane butterfly sum of pnp_kernels.hip (shfl_xor 8, 4, 2, 1 within
    16 lanes; entries past len(v) are zeros): ((v_k + v_k^8) + ...)."""
    a = list(map(float, v)) + [0.0] * (16 - len(v))
    for off in (8, 4, 2, 1):
        a = [a[k] + a[k ^ off] for k in range(16)]
    return a[0]


def cv_svd(A, tree=False):
    """A (m x n), m >= n -> (w [n] descending, U [m x n] columns, Vt [n x n]).
    tree=True: every sum over the m entries of a row is the 16-lane butterfly
    (tree16) -- the order in which the kernel's lane-parallel 12x12 SVD of
    EPnP's M^T M adds (m <= 16); otherwise OpenCV's sequential order."""
    A = np.asarray(A, np.float64)
    m, n = A.shape
    assert m >= n and (not tree or m <= 16)

    def ssum(vals):
        if tree:
            return tree16(vals)
        acc = 0.0
        for x in vals:
            acc += x
        return acc

    At = [list(map(float, A[:, i])) for i in range(n)]
    Vt = [[1.0 if i == j else 0.0 for j in range(n)] for i in range(n)]
    W = [0.0] * n
    for i in range(n):
        W[i] = ssum([At[i][k] * At[i][k] for k in range(m)])
    eps = DBL_EPS * 10
    for _ in range(max(m, 30)):
        changed = False
        for i in range(n - 1):
            for j in range(i + 1, n):
                Ai, Aj = At[i], At[j]
                a, b = W[i], W[j]
                p = ssum([Ai[k] * Aj[k] for k in range(m)])
                if abs(p) <= eps * math.sqrt(a * b):
                    continue
                p *= 2
                beta = a - b
                gamma = math.sqrt(p * p + beta * beta)  # one hypot formula on every side (pnp_kernels.hip)
                if beta < 0:
                    delta = (gamma - beta) * 0.5
                    s = math.sqrt(delta / gamma)
                    c = p / (gamma * s * 2)
                else:
                    c = math.sqrt((gamma + beta) / (gamma * 2))
                    s = p / (gamma * c * 2)
                for k in range(m):
                    t0 = c * Ai[k] + s * Aj[k]
                    t1 = -s * Ai[k] + c * Aj[k]
                    Ai[k] = t0
                    Aj[k] = t1
                W[i] = ssum([x * x for x in Ai])
                W[j] = ssum([x * x for x in Aj])
                changed = True
                Vi, Vj = Vt[i], Vt[j]
                for k in range(n):
                    t0 = c * Vi[k] + s * Vj[k]
                    t1 = -s * Vi[k] + c * Vj[k]
                    Vi[k] = t0
                    Vj[k] = t1
        if not changed:
            break
    for i in range(n):
        W[i] = math.sqrt(ssum([At[i][k] * At[i][k] for k in range(m)]))
    for i in range(n - 1):
        j = i
        for k in range(i + 1, n):
            if W[j] < W[k]:
                j = k
        if i != j:
            W[i], W[j] = W[j], W[i]
            At[i], At[j] = At[j], At[i]
            Vt[i], Vt[j] = Vt[j], Vt[i]
    rng = CvRNG(0x12345678)
    for i in range(n):
        sd = W[i]
        ii = 0
        while ii < 100 and sd <= DBL_MIN:
            val0 = 1.0 / m
            for k in range(m):
                At[i][k] = val0 if (rng.next() & 256) != 0 else -val0
            for _ in range(2):
                for j in range(i):
                    sd = ssum([At[i][k] * At[j][k] for k in range(m)])
                    for k in range(m):
                        At[i][k] = At[i][k] - sd * At[j][k]
                    asum = ssum([abs(At[i][k]) for k in range(m)])
                    asum = 1.0 / asum if asum > eps * 100 else 0.0
                    for k in range(m):
                        At[i][k] *= asum
            sd = math.sqrt(ssum([At[i][k] * At[i][k] for k in range(m)]))
            ii += 1
        s = 1.0 / sd if sd > DBL_MIN else 0.0
        for k in range(m):
            At[i][k] *= s
    return np.array(W), np.array(At).T.copy(), np.array(Vt)


def cv_svbksb(w, U, Vt, b=None):
    """x = V diag(1/w) U^T b over w_i > 2 DBL_EPSILON sum(w) (b = None: the
    pseudo-inverse), accumulated in descending-w order."""
    m, n = U.shape
    thr = 0.0
    for i in range(n):
        thr += w[i]
    thr *= DBL_EPS * 2
    if b is None:
        X = [[0.0] * m for _ in range(n)]
        for i in range(n):
            wi = w[i]
            if abs(wi) <= thr:
                continue
            wi = 1.0 / wi
            for j in range(n):
                vw = Vt[i][j] * wi
                for k in range(m):
                    X[j][k] = X[j][k] + vw * U[k][i]
        return np.array(X)
    x = [0.0] * n
    for i in range(n):
        wi = w[i]
        if abs(wi) <= thr:
            continue
        wi = 1.0 / wi
        s = 0.0
        for j in range(m):
            s += U[j][i] * b[j]
        s *= wi
        for j in range(n):
            x[j] = x[j] + s * Vt[i][j]
    return np.array(x)


def qr_solve(A, b):
    """epnp::qr_solve: Householder QR of A (6 x 4) as Lepetit's code does it."""
    A = [list(map(float, r)) for r in A]
    b = list(map(float, b))
    nr, nc = len(A), len(A[0])
    A1, A2 = [0.0] * nc, [0.0] * nc
    for k in range(nc):
        eta = abs(A[k][k])
        for i in range(k + 1, nr):
            elt = abs(A[i][k])
            if eta < elt:
                eta = elt
        if eta == 0:
            return None  # "A is singular": x left unchanged by the caller
        inv_eta = 1.0 / eta
        sum1 = 0.0
        for i in range(k, nr):
            A[i][k] *= inv_eta
            sum1 += A[i][k] * A[i][k]
        sigma = math.sqrt(sum1)
        if A[k][k] < 0:
            sigma = -sigma
        A[k][k] += sigma
        A1[k] = sigma * A[k][k]
        A2[k] = -eta * sigma
        for j in range(k + 1, nc):
            sm = 0.0
            for i in range(k, nr):
                sm += A[i][k] * A[i][j]
            tau = sm / A1[k]
            for i in range(k, nr):
                A[i][j] -= tau * A[i][k]
    for j in range(nc):
        tau = 0.0
        for i in range(j, nr):
            tau += A[i][j] * b[i]
        tau /= A1[j]
        for i in range(j, nr):
            b[i] -= tau * A[i][j]
    x = [0.0] * nc
    x[nc - 1] = b[nc - 1] / A2[nc - 1]
    for i in range(nc - 2, -1, -1):
        sm = 0.0
        for j in range(i + 1, nc):
            sm += A[i][j] * x[j]
        x[i] = (b[i] - sm) / A2[i]
    return np.array(x)


def epnp(K, opts, ipts):
    """epnp::compute_pose on object points opts [n][3] and image points ipts
    [n][2] (float32 data, double arithmetic, OpenCV's operation order) ->
    R (3x3), t (3)."""
    fu, fv, uc, vc = float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2])
    n = len(opts)
    pws = [list(map(float, p)) for p in np.asarray(opts, np.float64)]
    ip = np.asarray(ipts, np.float64)
    # solvePnP(EPNP): undistortPoints -> normalised float coordinates; epnp
    # maps them back to pixels with fu, fv, uc, vc
    us = []
    for i in range(n):
        xn = float(np.float32((ip[i, 0] - uc) * (1.0 / fu)))
        yn = float(np.float32((ip[i, 1] - vc) * (1.0 / fv)))
        us.append([xn * fu + uc, yn * fv + vc])
    # choose_control_points
    cws = [[0.0, 0.0, 0.0] for _ in range(4)]
    for i in range(n):
        for j in range(3):
            cws[0][j] += pws[i][j]
    for j in range(3):
        cws[0][j] /= n
    PW0 = np.array([[pws[i][j] - cws[0][j] for j in range(3)] for i in range(n)])
    PtP = [[0.0] * 3 for _ in range(3)]  # cvMulTransposed(PW0, PtP, 1): PW0^T PW0
    for a in range(3):
        for b in range(3):
            s = 0.0
            for i in range(n):
                s += PW0[i, a] * PW0[i, b]
            PtP[a][b] = s
    dc, Uc, _ = cv_svd(PtP)
    for i in range(1, 4):
        k = math.sqrt(dc[i - 1] / n)
        for j in range(3):
            cws[i][j] = cws[0][j] + k * Uc[j, i - 1]
    # compute_barycentric_coordinates (cvInvert(CV_SVD))
    cc = [[cws[j][i] - cws[0][i] for j in range(1, 4)] for i in range(3)]
    wc, Ucc, Vtc = cv_svd(cc)
    ci = cv_svbksb(wc, Ucc, Vtc)
    alphas = []
    for i in range(n):
        a = [0.0] * 4
        for j in range(3):
            a[1 + j] = (ci[j][0] * (pws[i][0] - cws[0][0]) + ci[j][1] * (pws[i][1] - cws[0][1]) +
                        ci[j][2] * (pws[i][2] - cws[0][2]))
        a[0] = 1.0 - a[1] - a[2] - a[3]
        alphas.append(a)
    M = [[0.0] * 12 for _ in range(2 * n)]
    for i in range(n):
        for j in range(4):
            M[2 * i][3 * j] = alphas[i][j] * fu
            M[2 * i][3 * j + 2] = alphas[i][j] * (uc - us[i][0])
            M[2 * i + 1][3 * j + 1] = alphas[i][j] * fv
            M[2 * i + 1][3 * j + 2] = alphas[i][j] * (vc - us[i][1])
    MtM = [[0.0] * 12 for _ in range(12)]
    for a in range(12):
        for b in range(12):
            s = 0.0
            for r in range(2 * n):
                s += M[r][a] * M[r][b]
            MtM[a][b] = s
    _, Um, _ = cv_svd(MtM, tree=True)
    ut = Um.T  # rows: left singular vectors, descending singular values
    v = [ut[11], ut[10], ut[9], ut[8]]
    pairs = [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]

    def dot3(x, y):
        return x[0] * y[0] + x[1] * y[1] + x[2] * y[2]

    dv = [[[v[i][3 * a + m] - v[i][3 * b + m] for m in range(3)] for a, b in pairs] for i in range(4)]
    L = []
    for i in range(6):
        d0, d1, d2, d3 = dv[0][i], dv[1][i], dv[2][i], dv[3][i]
        L.append([dot3(d0, d0), 2.0 * dot3(d0, d1), dot3(d1, d1), 2.0 * dot3(d0, d2), 2.0 * dot3(d1, d2),
                  dot3(d2, d2), 2.0 * dot3(d0, d3), 2.0 * dot3(d1, d3), 2.0 * dot3(d2, d3), dot3(d3, d3)])
    rho = []
    for a, b in pairs:
        rho.append((cws[a][0] - cws[b][0]) ** 2 + (cws[a][1] - cws[b][1]) ** 2 + (cws[a][2] - cws[b][2]) ** 2)

    def solve_ls(cols):
        A = [[L[i][c] for c in cols] for i in range(6)]
        w, U, Vt = cv_svd(A)
        return cv_svbksb(w, U, Vt, rho)

    def gauss_newton(betas):
        betas = list(betas)
        for _ in range(5):
            A, bb = [], []
            b0, b1, b2, b3 = betas
            for i in range(6):
                r = L[i]
                A.append([2 * r[0] * b0 + r[1] * b1 + r[3] * b2 + r[6] * b3,
                          r[1] * b0 + 2 * r[2] * b1 + r[4] * b2 + r[7] * b3,
                          r[3] * b0 + r[4] * b1 + 2 * r[5] * b2 + r[8] * b3,
                          r[6] * b0 + r[7] * b1 + r[8] * b2 + 2 * r[9] * b3])
                bb.append(rho[i] - (r[0] * b0 * b0 + r[1] * b0 * b1 + r[2] * b1 * b1 + r[3] * b0 * b2 +
                                    r[4] * b1 * b2 + r[5] * b2 * b2 + r[6] * b0 * b3 + r[7] * b1 * b3 +
                                    r[8] * b2 * b3 + r[9] * b3 * b3))
            x = qr_solve(A, bb)
            if x is None:
                return betas
            for i in range(4):
                betas[i] += x[i]
        return betas

    def r_and_t(betas):
        ccs = [[0.0] * 3 for _ in range(4)]
        for i in range(4):
            vv = ut[11 - i]
            for j in range(4):
                for k in range(3):
                    ccs[j][k] += betas[i] * vv[3 * j + k]
        pcs = []
        for i in range(n):
            a = alphas[i]
            pcs.append([a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j] for j in range(3)])
        if pcs[0][2] < 0.0:
            pcs = [[-x for x in p] for p in pcs]
        pc0, pw0 = [0.0] * 3, [0.0] * 3
        for i in range(n):
            for j in range(3):
                pc0[j] += pcs[i][j]
                pw0[j] += pws[i][j]
        for j in range(3):
            pc0[j] /= n
            pw0[j] /= n
        abt = [[0.0] * 3 for _ in range(3)]
        for i in range(n):
            for j in range(3):
                for k in range(3):
                    abt[j][k] += (pcs[i][j] - pc0[j]) * (pws[i][k] - pw0[k])
        _, Ua, Vta = cv_svd(abt)
        R = [[Ua[i][0] * Vta[0][j] + Ua[i][1] * Vta[1][j] + Ua[i][2] * Vta[2][j] for j in range(3)] for i in range(3)]
        det = (R[0][0] * R[1][1] * R[2][2] + R[0][1] * R[1][2] * R[2][0] + R[0][2] * R[1][0] * R[2][1] -
               R[0][2] * R[1][1] * R[2][0] - R[0][1] * R[1][0] * R[2][2] - R[0][0] * R[1][2] * R[2][1])
        if det < 0:
            R[2] = [-x for x in R[2]]
        t = [pc0[i] - dot3(R[i], pw0) for i in range(3)]
        sum2 = 0.0
        for i in range(n):
            pw = pws[i]
            Xc = dot3(R[0], pw) + t[0]
            Yc = dot3(R[1], pw) + t[1]
            inv_Zc = 1.0 / (dot3(R[2], pw) + t[2])
            ue = uc + fu * Xc * inv_Zc
            ve = vc + fv * Yc * inv_Zc
            sum2 += math.sqrt((us[i][0] - ue) * (us[i][0] - ue) + (us[i][1] - ve) * (us[i][1] - ve))
        return sum2 / n, np.array(R), np.array(t)

    res = []
    b4 = solve_ls([0, 1, 3, 6])
    if b4[0] < 0:
        s0 = math.sqrt(-b4[0])
        betas = [s0, -b4[1] / s0, -b4[2] / s0, -b4[3] / s0]
    else:
        s0 = math.sqrt(b4[0])
        betas = [s0, b4[1] / s0, b4[2] / s0, b4[3] / s0]
    res.append(r_and_t(gauss_newton(betas)))
    b3 = solve_ls([0, 1, 2])
    if b3[0] < 0:
        betas = [math.sqrt(-b3[0]), math.sqrt(-b3[2]) if b3[2] < 0 else 0.0, 0.0, 0.0]
    else:
        betas = [math.sqrt(b3[0]), math.sqrt(b3[2]) if b3[2] > 0 else 0.0, 0.0, 0.0]
    if b3[1] < 0:
        betas[0] = -betas[0]
    res.append(r_and_t(gauss_newton(betas)))
    b5 = solve_ls([0, 1, 2, 3, 4])
    if b5[0] < 0:
        betas = [math.sqrt(-b5[0]), math.sqrt(-b5[2]) if b5[2] < 0 else 0.0, 0.0, 0.0]
    else:
        betas = [math.sqrt(b5[0]), math.sqrt(b5[2]) if b5[2] > 0 else 0.0, 0.0, 0.0]
    if b5[1] < 0:
        betas[0] = -betas[0]
    betas[2] = b5[3] / betas[0]
    res.append(r_and_t(gauss_newton(betas)))
    best = 0
    if res[1][0] < res[0][0]:
        best = 1
    if res[2][0] < res[best][0]:
        best = 2
    return res[best][1], res[best][2]


def point_errors(K, opts, ipts, rvec, tvec):
    """PnPRansacCallback::computeError: float distance image point <->
    projectPoints(object point, Rodrigues(rvec), tvec, K) (stored as float)."""
    R = rodrigues_v2m(rvec)
    P = np.asarray(opts, np.float64)
    x, y, z = P[:, 0], P[:, 1], P[:, 2]
    X = R[0, 0] * x + R[0, 1] * y + R[0, 2] * z + tvec[0]
    Y = R[1, 0] * x + R[1, 1] * y + R[1, 2] * z + tvec[1]
    Z = R[2, 0] * x + R[2, 1] * y + R[2, 2] * z + tvec[2]
    iz = np.where(Z != 0, 1.0 / np.where(Z != 0, Z, 1.0), 1.0)
    u = (X * iz * K[0, 0] + K[0, 2]).astype(np.float32)
    v = (Y * iz * K[1, 1] + K[1, 2]).astype(np.float32)
    du = np.asarray(ipts, np.float32)[:, 0] - u
    dv = np.asarray(ipts, np.float32)[:, 1] - v
    return np.sqrt((du.astype(np.float64) ** 2 + dv.astype(np.float64) ** 2)).astype(np.float32)


def solve_pnp_ransac(opts, ipts, K, iterations: int = 20, reproj_err: float = 7.0, confidence: float = 0.99,
                     trace: list | None = None):
    """-> (ok, rvec[3], tvec[3], inlier indices int32).  `trace`, when a list,
    receives per iteration (subset, rvec, tvec, inlier count)."""
    K = np.asarray(K, np.float64).reshape(3, 3)
    opts = np.asarray(opts, np.float64).reshape(-1, 3).astype(np.float32)
    ipts = np.asarray(ipts, np.float64).reshape(-1, 2).astype(np.float32)
    n = len(opts)
    model_points = 5
    if n < model_points:
        return False, np.zeros(3), np.zeros(3), np.zeros(0, np.int32)
    thresh = np.float32(reproj_err * reproj_err)
    rng = CvRNG()
    niters = max(iterations, 1)
    best = None
    best_mask = None
    max_good = 0
    it = 0
    while it < niters:
        sub = list(range(n)) if n == model_points else get_subset(rng, n, model_points)
        R, t = epnp(K, opts[sub], ipts[sub])
        rvec = rodrigues_m2v(R)
        mask = point_errors(K, opts, ipts, rvec, t) <= thresh
        good = int(mask.sum())
        if trace is not None:
            trace.append((sub, rvec, t, good))
        if n == model_points:
            return True, rvec, t, np.arange(n, dtype=np.int32)
        if good > max(max_good, model_points - 1):
            best, best_mask, max_good = (rvec, t), mask, good
            niters = ransac_update_num_iters(confidence, (n - good) / n, model_points, niters)
        it += 1
    if best is None:
        return False, np.zeros(3), np.zeros(3), np.zeros(0, np.int32)
    return True, best[0], best[1], np.nonzero(best_mask)[0].astype(np.int32)


def triangulate_points(cam0, cam1, uv0, uv1, P):
    """cv::triangulatePoints (cvTriangulatePoints) per point on P = K [R|t]
    (P [C][3][4]): the 4x4 DLT system of both views, the right singular
    vector of its smallest singular value (cv_svd), homogeneous division
    (the CSfM.cpp:156 / :918 call; GeometryUtils is absent: parity
    unpinned).  -> X [n][3]."""
    P = np.asarray(P, np.float64).reshape(-1, 3, 4)
    n = len(cam0)
    X = np.zeros((n, 3))
    for i in range(n):
        Pa, Pb = P[cam0[i]], P[cam1[i]]
        xa, ya = float(uv0[i][0]), float(uv0[i][1])
        xb, yb = float(uv1[i][0]), float(uv1[i][1])
        A = [[xa * Pa[2, k] - Pa[0, k] for k in range(4)], [ya * Pa[2, k] - Pa[1, k] for k in range(4)],
             [xb * Pb[2, k] - Pb[0, k] for k in range(4)], [yb * Pb[2, k] - Pb[1, k] for k in range(4)]]
        _, _, Vt = cv_svd(A)
        h = Vt[3][3]
        X[i] = [Vt[3][0] / h, Vt[3][1] / h, Vt[3][2] / h]
    return X
