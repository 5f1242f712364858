// Per-frame pose: cv::solvePnPRansac as CSfM::tracking calls it
// (/root/reference/CSfM.cpp:553-565: iterationsCount 20, reprojectionError
// _maxReprErr = 7 (CSfM.cpp:35), confidence 0.99, SOLVEPNP_ITERATIVE), on
// gfx950.  The semantics are OpenCV 3.0's (README.md:28), restated in
// oracle/pnp_oracle.py (parity unpinned: OpenCV is absent):
//   * RANSAC over 5-point subsets drawn by cv::RNG(uint64(-1)), kernel =
//     EPnP on the subset, inlier when the float reprojection DISTANCE is
//     <= reprErr^2 (3.0's findInliers squares the threshold), model kept
//     when its inlier count beats max(best, 4), iteration bound shrunk by
//     RANSACUpdateNumIters;
//   * the returned pose is the best RANSAC model (3.0 discards the pose of
//     its final refinement), the inliers are its mask.
//
// Device mapping.  RANSAC's hypotheses are independent once the subsets are
// drawn, so: one thread draws every subset of the iteration bound (the RNG
// sequence is inherently sequential, ~100 draws); one WAVE per hypothesis
// solves its EPnP (the 12x12 M^T M eigen-decomposition by one-sided Jacobi
// with lane i holding row i, everything else wave-uniform in registers);
// one workgroup per hypothesis scores all n points (fixed-order count);
// one wave replays the sequential acceptance rule over the counts (the
// bound only shrinks, so evaluating the full bound and replaying gives the
// sequential result exactly) and compacts the winner's inliers in order.
#include <hip/hip_runtime.h>
#include <utility>
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>
#include "sfm_trace.h"
#include "../../include/sfm_amd.h"
#include "cv_linalg.h"

void sfm_internal_set_error(const std::string& msg);

namespace sfm {
namespace {

constexpr int kModel = 5;      // RANSAC subset size (EPnP kernel)
constexpr int kMaxIters = 1024;

struct PnPCam {
  double fu, fv, uc, vc;
};

__host__ __device__ void rodrigues_v2m(const double r[3], double R[9]) {
  const double th = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
  if (th < DBL_EPSILON) {
    for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
    return;
  }
  const double c = cos(th), s = sin(th), c1 = 1.0 - c, it = 1.0 / th;
  const double x = r[0] * it, y = r[1] * it, z = r[2] * it;
  // c I + c1 r r^T + s [r]x, summed as cv::Matx33d does (elementwise, in order)
  R[0] = c + c1 * (x * x);     R[1] = c1 * (x * y) + s * -z; R[2] = c1 * (x * z) + s * y;
  R[3] = c1 * (x * y) + s * z; R[4] = c + c1 * (y * y);       R[5] = c1 * (y * z) + s * -x;
  R[6] = c1 * (x * z) + s * -y; R[7] = c1 * (y * z) + s * x;  R[8] = c + c1 * (z * z);
}

__host__ __device__ void rodrigues_m2v(const double R[9], double r[3]) {
  double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
  const double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
  double c = (R[0] + R[4] + R[8] - 1.0) * 0.5;
  c = c > 1.0 ? 1.0 : (c < -1.0 ? -1.0 : c);
  const double th = acos(c);
  if (s < 1e-5) {
    if (c > 0) {
      r[0] = r[1] = r[2] = 0.0;
      return;
    }
    double t = (R[0] + 1) * 0.5;
    rx = sqrt(fmax(t, 0.0));
    t = (R[4] + 1) * 0.5;
    ry = sqrt(fmax(t, 0.0)) * (R[1] < 0 ? -1.0 : 1.0);
    t = (R[8] + 1) * 0.5;
    rz = sqrt(fmax(t, 0.0)) * (R[2] < 0 ? -1.0 : 1.0);
    if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
    const double k = th / sqrt(rx * rx + ry * ry + rz * rz);
    r[0] = rx * k; r[1] = ry * k; r[2] = rz * k;
    return;
  }
  const double k = th / (2.0 * s);
  r[0] = rx * k; r[1] = ry * k; r[2] = rz * k;
}

// ---- cv::SVD of EPnP's 12x12 M^T M with the 12 columns over lanes --------
// Lane k (mod 16) holds entry k of every row of At (lanes 12..15 of each
// 16-lane segment hold zeros); the row sums are the 16-lane butterfly
// (shfl_xor 8, 4, 2, 1 -- every lane ends with the same value, floating
// addition being commutative), which oracle/pnp_oracle.py cv_svd(tree=True)
// reproduces.  Otherwise JacobiSVDImpl_ step for step (no V).
// The partner values come by DPP row rotation (row_ror 8, 4, 2, 1 within
// each 16-lane row) instead of ds_bpermute.  Rotating by 8 is xor 8; after
// the levels above distance d, a lane's partial sum depends only on L mod 2d,
// and (L + d) mod 2d == (L ^ d) mod 2d, so rotating by d delivers exactly
// the xor partner's partial: the sum is bitwise the xor butterfly's (the
// oracle's tree order), at a few cycles per level instead of an LDS round
// trip.
template <int kCtrl>
__device__ __forceinline__ double dpp_f64(double v) {
  // (every lane of a row rotation is written: no "old" operand to set up)
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), kCtrl, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), kCtrl, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double tree16(double v) {
  constexpr int kRowRor = 0x120;  // DPP row_ror:n = 0x120 + n
  v += dpp_f64<kRowRor + 8>(v);
  v += dpp_f64<kRowRor + 4>(v);
  v += dpp_f64<kRowRor + 2>(v);
  v += dpp_f64<kRowRor + 1>(v);
  return v;
}

// The Jacobi sweeps in OpenCV's order (0,1), (0,2), ..., (10,11), sweep
// after sweep, scheduled by row dependencies (a rotation (i, j) waits only
// for the latest earlier rotation on row i and on row j, in its own sweep or
// the one before) into passes of up to 4 rotations on disjoint rows
// (svd_schedule.h, tools/svd_schedule.py): the wave's four 16-lane rows each
// hold the whole 12-row state and take one rotation of a pass, then exchange
// the rotated rows.  Every rotation is the same arithmetic on the same
// values as in the sequential order, so the result is bitwise OpenCV's.  (A
// branch-free sequential sweep, for the scheduler to overlap, measured
// slower: 0.375-0.388 vs 0.313 ms per PnP call.)  One sweep alone is 23
// passes; the tail of sweep s with the head of sweep s + 1 (run once sweep s
// has rotated something, i.e. once sweep s + 1 is certain) is 18 for 66
// rotations.  The slots of a pass with fewer than 4 rotations repeat (n = 1:
// slot 0 everywhere, n = 2: 0 1 0 1, n = 3: 0 1 2 0), so a row pair / the
// whole wave already agrees on them.
// (svd_schedule.h comes with cv_linalg.h)
template <int S>
struct SvdSched;
template <>
struct SvdSched<0> {  // head of a sweep
  static constexpr int P = kSvdProPasses;
  static constexpr const int* N = kSvdProN;
  static constexpr const int (*I)[4] = kSvdProI;
  static constexpr const int (*J)[4] = kSvdProJ;
  static constexpr const int (*T)[4] = kSvdProT;
};
template <>
struct SvdSched<1> {  // tail of sweep s + head of sweep s + 1
  static constexpr int P = kSvdPerPasses;
  static constexpr const int* N = kSvdPerN;
  static constexpr const int (*I)[4] = kSvdPerI;
  static constexpr const int (*J)[4] = kSvdPerJ;
  static constexpr const int (*T)[4] = kSvdPerT;
};
template <>
struct SvdSched<2> {  // tail of a sweep
  static constexpr int P = kSvdEpiPasses;
  static constexpr const int* N = kSvdEpiN;
  static constexpr const int (*I)[4] = kSvdEpiI;
  static constexpr const int (*J)[4] = kSvdEpiJ;
  static constexpr const int (*T)[4] = kSvdEpiT;
};
// row g's value of four: three independent selects on the row's masks
// (a nested g == 0 ? : g == 1 ? ... became divergent branches)
struct RowSel {
  bool s1, s2, s3;
};
__device__ __forceinline__ double sel4(const RowSel& m, double a0, double a1, double a2, double a3) {
  double r = m.s1 ? a1 : a0;
  r = m.s2 ? a2 : r;
  return m.s3 ? a3 : r;
}

// The rotated rows change hands across the wave's 16-lane rows with gfx950's
// row swaps (lane k of one row with lane k of another, no LDS round trip):
// pair16(x) = (x of the even, x of the odd row of my row pair), pair32(x) =
// (x of my row in the lower, in the upper half of the wave).
__device__ __forceinline__ double2 pair16(double x) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  const auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return make_double2(__hiloint2double(rh[0], rl[0]), __hiloint2double(rh[1], rl[1]));
}
__device__ __forceinline__ double2 pair32(double x) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return make_double2(__hiloint2double(rh[0], rl[0]), __hiloint2double(rh[1], rl[1]));
}
// x of rows 0..3 at my lane (mod 16), for a pass of n rotations
template <int n>
__device__ __forceinline__ void gather_rows(double x, double (&v)[4]) {
  if constexpr (n == 1) {
    v[0] = v[1] = v[2] = v[3] = x;
  } else if constexpr (n == 2) {
    const double2 e = pair16(x);
    v[0] = v[2] = e.x;
    v[1] = v[3] = e.y;
  } else {
    const double2 e = pair16(x);
    const double2 a = pair32(e.x), b = pair32(e.y);
    v[0] = a.x; v[2] = a.y; v[1] = b.x; v[3] = b.y;
  }
}

// u[i] = At[i][lane & 15] on entry (M^T M is symmetric); on return the
// four left singular vectors of the smallest singular values are in
// ut[q] = OpenCV's ut row 11 - q, every lane holding all 12 entries.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// lds: this wave's kSvdLds doubles (ut at the end of the 12x12; the rows of
// the beta cases' 6x5 / 6x4 SVDs, cv_linalg.h cv_svd_sweeps_lanes)
constexpr int kSvdLds = 6 * 10 + 6;  // (>= 5 (6 + 5): also L and rho for the Gauss-Newton rows)
// One pass of schedule S; ch[t] |= a rotation of tag t turned.
// JacobiSVDImpl_ keeps W_i = |row i|^2, set from the row itself after every
// rotation of row i (and at the start), so W_i is always tree16(u_i * u_i)
// of the current row, bitwise: the pass recomputes a = W_i and b = W_j from
// the rows (two trees beside p's) instead of carrying W through the
// exchange -- two trees fewer after the rotation, W never exchanged.
template <int S, int ps>
__device__ __forceinline__ void svd_pass(const RowSel& g, double (&u)[12], double eps, bool (&ch)[2]) {
  using Sc = SvdSched<S>;
  constexpr int n = Sc::N[ps];
  constexpr int I0 = Sc::I[ps][0], I1 = Sc::I[ps][1], I2 = Sc::I[ps][2], I3 = Sc::I[ps][3];
  constexpr int J0 = Sc::J[ps][0], J1 = Sc::J[ps][1], J2 = Sc::J[ps][2], J3 = Sc::J[ps][3];
  constexpr uint64_t kTag1 = (Sc::T[ps][0] ? 0xFFFFull : 0) | (Sc::T[ps][1] ? 0xFFFFull << 16 : 0) |
                             (Sc::T[ps][2] ? 0xFFFFull << 32 : 0) | (Sc::T[ps][3] ? 0xFFFFull << 48 : 0);
  // row g's rotation (I[g], J[g])
  const double ui = sel4(g, u[I0], u[I1], u[I2], u[I3]);
  const double uj = sel4(g, u[J0], u[J1], u[J2], u[J3]);
  const double a = tree16(ui * ui), b = tree16(uj * uj);
  double p = tree16(ui * uj);
  const bool act = !(fabs(p) <= eps * sqrt(a * b));
  const uint64_t turned = __builtin_amdgcn_ballot_w64(act);
  if (turned == 0) return;  // every rotation of the pass skipped
  if (turned & kTag1) ch[1] = true;
  if (turned & ~kTag1) ch[0] = true;
  p *= 2;
  const double beta = a - b, gamma = sqrt(p * p + beta * beta);
  // JacobiSVDImpl_'s two cases with their operands selected, not branched
  // (rows of the wave take either): beta < 0: sn = sqrt(((gamma - beta) *
  // 0.5) / gamma), c = p / (gamma * sn * 2); else c = sqrt((gamma + beta) /
  // (gamma * 2)), sn = p / (gamma * c * 2) -- the same operations on the
  // same values either way.
  const bool neg = beta < 0;
  const double num = neg ? (gamma - beta) * 0.5 : gamma + beta;
  const double den = neg ? gamma : gamma * 2;
  const double s1 = sqrt(num / den);
  const double o = p / (gamma * s1 * 2);
  const double c = neg ? o : s1, sn = neg ? s1 : o;
  double t0 = c * ui + sn * uj, t1 = -sn * ui + c * uj;
  t0 = act ? t0 : ui;
  t1 = act ? t1 : uj;
  double vt0[4], vt1[4];
  gather_rows<n>(t0, vt0);
  gather_rows<n>(t1, vt1);
  u[I0] = vt0[0]; u[J0] = vt1[0];
  if constexpr (n > 1) { u[I1] = vt0[1]; u[J1] = vt1[1]; }
  if constexpr (n > 2) { u[I2] = vt0[2]; u[J2] = vt1[2]; }
  if constexpr (n > 3) { u[I3] = vt0[3]; u[J3] = vt1[3]; }
}
template <int S, int... ps>
__device__ __forceinline__ void svd_run(const RowSel& g, double (&u)[12], double eps, bool (&ch)[2],
                                        std::integer_sequence<int, ps...>) {
  (svd_pass<S, ps>(g, u, eps, ch), ...);
}
template <int S>
__device__ __forceinline__ void svd_run(const RowSel& g, double (&u)[12], double eps, bool (&ch)[2]) {
  svd_run<S>(g, u, eps, ch, std::make_integer_sequence<int, SvdSched<S>::P>{});
}
__device__ void cv_svd12_lanes(double (&u)[12], double* lds, double (&ut)[4][12]) {
  const int k = threadIdx.x & 15, g = (threadIdx.x & 63) >> 4;
  const RowSel gs{g == 1, g == 2, g == 3};
  const double eps = kDblEps * 10;
  // sweep s runs iff s < 30 and sweeps 0..s-1 each rotated something
  bool ch[2] = {false, false}, head = true;
  for (int s = 0;;) {
    if (head) svd_run<0>(gs, u, eps, ch);  // head of sweep s (tag 1)
    head = false;
    if (ch[1] && s + 1 < 30) {  // sweep s has turned: its tail with sweep s + 1's head
      ch[0] = ch[1] = false;
      svd_run<1>(gs, u, eps, ch);
      ++s;
    } else {
      const bool turned = ch[1];
      ch[0] = false;
      svd_run<2>(gs, u, eps, ch);  // tail of sweep s (tag 0)
      if (!(turned || ch[0]) || ++s >= 30) break;
      ch[1] = false;
      head = true;
    }
  }
  int ord[12];
  double W[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) { W[i] = sqrt(tree16(u[i] * u[i])); ord[i] = i; }
  {
    // Fast path: every W distinct and > DBL_MIN -- the selection sort below is
    // then the descending order and completes nothing, and only rows 8..11
    // (the four smallest) are kept: lane k < 12 ranks W_k, the rows of ranks
    // 11..8 are picked by ballot, normalised and published.  (Ties or zero
    // singular values -- e.g. planar points -- take the full path.)
    double wk = W[0];
#pragma unroll
    for (int i = 1; i < 12; ++i) wk = k == i ? W[i] : wk;
    int rank = 0;
    bool tie = false;
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      rank += W[i] > wk ? 1 : 0;
      tie = tie || (i != k && W[i] == wk);
    }
    if (__builtin_amdgcn_ballot_w64(k < 12 && (tie || !(wk > kDblMin))) == 0) {
      double rq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int src = __builtin_ctzll(__builtin_amdgcn_ballot_w64(k < 12 && rank == 11 - q) & 0xFFFull);
        double x = u[0], sd = W[0];
#pragma unroll
        for (int c = 1; c < 12; ++c) {
          x = src == c ? u[c] : x;
          sd = src == c ? W[c] : sd;
        }
        rq[q] = x * (1.0 / sd);
      }
      if (k < 12 && (threadIdx.x & 63) < 16)
#pragma unroll
        for (int q = 0; q < 4; ++q) lds[q * 12 + k] = rq[q];
      wave_sync();
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int m = 0; m < 12; ++m) ut[q][m] = lds[q * 12 + m];
      return;
    }
  }
#pragma unroll
  for (int i = 0; i < 11; ++i) {
    int j = i;
#pragma unroll
    for (int q = i + 1; q < 12; ++q)
      if (W[j] < W[q]) j = q;
#pragma unroll
    for (int q = i + 1; q < 12; ++q)
      if (j == q) {
        const double tw = W[i]; W[i] = W[q]; W[q] = tw;
        const int to = ord[i]; ord[i] = ord[q]; ord[q] = to;
      }
  }
  // rows in sorted order (row r = u[ord[r]]), zero singular values completed
  // from cv::RNG(0x12345678), then normalised; only rows 8..11 are kept
  double row[12];
#pragma unroll
  for (int r = 0; r < 12; ++r) {
    double x = 0.0;
#pragma unroll
    for (int c = 0; c < 12; ++c) x = ord[r] == c ? u[c] : x;
    row[r] = x;
  }
  uint64_t rng = 0x12345678ull;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    double sd = W[i];
    for (int ii = 0; ii < 100 && sd <= kDblMin; ++ii) {
      const double val0 = 1.0 / 12;
      for (int e = 0; e < 12; ++e) {
        const double v = (cv_rng_next(rng) & 256) != 0 ? val0 : -val0;
        if (e == k) row[i] = v;
      }
      for (int it2 = 0; it2 < 2; ++it2)
#pragma unroll
        for (int j = 0; j < i; ++j) {
          sd = tree16(row[i] * row[j]);
          row[i] = row[i] - sd * row[j];
          double asum = tree16(fabs(row[i]));
          asum = asum > eps * 100 ? 1.0 / asum : 0.0;
          row[i] *= asum;
        }
      sd = sqrt(tree16(row[i] * row[i]));
    }
    const double sc = sd > kDblMin ? 1.0 / sd : 0.0;
    row[i] *= sc;
  }
  if (k < 12 && (threadIdx.x & 63) < 16)
#pragma unroll
    for (int q = 0; q < 4; ++q) lds[q * 12 + k] = row[11 - q];
  wave_sync();
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int m = 0; m < 12; ++m) ut[q][m] = lds[q * 12 + m];
}

// Host build of the same 12x12 SVD (tools/pnp_host_check): the butterfly
// order computed serially.
__host__ inline double host_tree16(const double (&v)[12]) {
  double a[16];
  for (int q = 0; q < 16; ++q) a[q] = q < 12 ? v[q] : 0.0;
  for (int off = 8; off > 0; off >>= 1) {
    double b[16];
    for (int q = 0; q < 16; ++q) b[q] = a[q] + a[q ^ off];
    for (int q = 0; q < 16; ++q) a[q] = b[q];
  }
  return a[0];
}
__host__ inline void host_svd12_tree(double (&U)[12][12], double (&ut)[4][12]) {
  double W[12], tmp[12];
  for (int i = 0; i < 12; ++i) {
    for (int q = 0; q < 12; ++q) tmp[q] = U[i][q] * U[i][q];
    W[i] = host_tree16(tmp);
  }
  const double eps = kDblEps * 10;
  for (int iter = 0; iter < 30; ++iter) {
    bool changed = false;
    for (int i = 0; i < 11; ++i)
      for (int j = i + 1; j < 12; ++j) {
        const double a = W[i], b = W[j];
        for (int q = 0; q < 12; ++q) tmp[q] = U[i][q] * U[j][q];
        double p = host_tree16(tmp);
        if (fabs(p) <= eps * sqrt(a * b)) continue;
        p *= 2;
        const double beta = a - b, gamma = sqrt(p * p + beta * beta);
        double c, sn;
        if (beta < 0) {
          const double delta = (gamma - beta) * 0.5;
          sn = sqrt(delta / gamma);
          c = p / (gamma * sn * 2);
        } else {
          c = sqrt((gamma + beta) / (gamma * 2));
          sn = p / (gamma * c * 2);
        }
        for (int q = 0; q < 12; ++q) {
          const double t0 = c * U[i][q] + sn * U[j][q], t1 = -sn * U[i][q] + c * U[j][q];
          U[i][q] = t0;
          U[j][q] = t1;
        }
        for (int q = 0; q < 12; ++q) tmp[q] = U[i][q] * U[i][q];
        W[i] = host_tree16(tmp);
        for (int q = 0; q < 12; ++q) tmp[q] = U[j][q] * U[j][q];
        W[j] = host_tree16(tmp);
        changed = true;
      }
    if (!changed) break;
  }
  int ord[12];
  for (int i = 0; i < 12; ++i) {
    for (int q = 0; q < 12; ++q) tmp[q] = U[i][q] * U[i][q];
    W[i] = sqrt(host_tree16(tmp));
    ord[i] = i;
  }
  for (int i = 0; i < 11; ++i) {
    int j = i;
    for (int q = i + 1; q < 12; ++q)
      if (W[j] < W[q]) j = q;
    if (j != i) {
      const double tw = W[i]; W[i] = W[j]; W[j] = tw;
      const int to = ord[i]; ord[i] = ord[j]; ord[j] = to;
    }
  }
  double row[12][12];
  for (int r = 0; r < 12; ++r)
    for (int q = 0; q < 12; ++q) row[r][q] = U[ord[r]][q];
  uint64_t rng = 0x12345678ull;
  for (int i = 0; i < 12; ++i) {
    double sd = W[i];
    for (int ii = 0; ii < 100 && sd <= kDblMin; ++ii) {
      for (int e = 0; e < 12; ++e) row[i][e] = (cv_rng_next(rng) & 256) != 0 ? 1.0 / 12 : -1.0 / 12;
      for (int it2 = 0; it2 < 2; ++it2)
        for (int j = 0; j < i; ++j) {
          for (int q = 0; q < 12; ++q) tmp[q] = row[i][q] * row[j][q];
          sd = host_tree16(tmp);
          for (int q = 0; q < 12; ++q) row[i][q] = row[i][q] - sd * row[j][q];
          for (int q = 0; q < 12; ++q) tmp[q] = fabs(row[i][q]);
          double asum = host_tree16(tmp);
          asum = asum > eps * 100 ? 1.0 / asum : 0.0;
          for (int q = 0; q < 12; ++q) row[i][q] *= asum;
        }
      for (int q = 0; q < 12; ++q) tmp[q] = row[i][q] * row[i][q];
      sd = sqrt(host_tree16(tmp));
    }
    const double sc = sd > kDblMin ? 1.0 / sd : 0.0;
    for (int q = 0; q < 12; ++q) row[i][q] *= sc;
  }
  for (int q = 0; q < 4; ++q)
    for (int m = 0; m < 12; ++m) ut[q][m] = row[11 - q][m];
}

// ---- EPnP (epnp::compute_pose) on 5 correspondences, one wave ----------
struct EpnpIn {
  double pw[kModel][3];
  double us[kModel][2];
};

__host__ __device__ __forceinline__ double dot3(const double* x, const double* y) { return x[0] * y[0] + x[1] * y[1] + x[2] * y[2]; }

__host__ __device__ double r_and_t(const EpnpIn& in, const double (&alpha)[kModel][4], const double (&ut)[4][12],
                          const double betas[4], const PnPCam& k, double R[9], double t[3]) {
  double ccs[4][3] = {};
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int m = 0; m < 3; ++m) ccs[j][m] += betas[i] * ut[i][3 * j + m];
  double pcs[kModel][3];
#pragma unroll
  for (int p = 0; p < kModel; ++p)
#pragma unroll
    for (int m = 0; m < 3; ++m)
      pcs[p][m] = alpha[p][0] * ccs[0][m] + alpha[p][1] * ccs[1][m] + alpha[p][2] * ccs[2][m] + alpha[p][3] * ccs[3][m];
  if (pcs[0][2] < 0.0) {
#pragma unroll
    for (int p = 0; p < kModel; ++p)
#pragma unroll
      for (int m = 0; m < 3; ++m) pcs[p][m] = -pcs[p][m];
  }
  double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
#pragma unroll
  for (int p = 0; p < kModel; ++p)
#pragma unroll
    for (int m = 0; m < 3; ++m) { pc0[m] += pcs[p][m]; pw0[m] += in.pw[p][m]; }
#pragma unroll
  for (int m = 0; m < 3; ++m) { pc0[m] /= kModel; pw0[m] /= kModel; }
  double abt[3][3] = {};
#pragma unroll
  for (int p = 0; p < kModel; ++p)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int m = 0; m < 3; ++m) abt[j][m] += (pcs[p][j] - pc0[j]) * (in.pw[p][m] - pw0[m]);
  double U3[3][3], w3[3], Vt3[3][3];
  cv_svd<3, 3>(abt, U3, w3, Vt3);
  // R = U V^T: R(i, j) = sum_k U(i, k) V(j, k), U(i, k) = U3[k][i], V(j, k) = Vt3[k][j]
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) R[3 * i + j] = U3[0][i] * Vt3[0][j] + U3[1][i] * Vt3[1][j] + U3[2][i] * Vt3[2][j];
  const double det = R[0] * R[4] * R[8] + R[1] * R[5] * R[6] + R[2] * R[3] * R[7] - R[2] * R[4] * R[6] -
                     R[1] * R[3] * R[8] - R[0] * R[5] * R[7];
  if (det < 0) { R[6] = -R[6]; R[7] = -R[7]; R[8] = -R[8]; }
#pragma unroll
  for (int i = 0; i < 3; ++i) t[i] = pc0[i] - dot3(R + 3 * i, pw0);
  double sum = 0.0;
#pragma unroll
  for (int p = 0; p < kModel; ++p) {
    const double* x = in.pw[p];
    const double Xc = dot3(R, x) + t[0];
    const double Yc = dot3(R + 3, x) + t[1];
    const double iz = 1.0 / (dot3(R + 6, x) + t[2]);
    const double ue = k.uc + k.fu * Xc * iz, ve = k.vc + k.fv * Yc * iz;
    const double du = in.us[p][0] - ue, dv = in.us[p][1] - ve;
    sum += sqrt(du * du + dv * dv);
  }
  return sum / kModel;
}

// One row of epnp::compute_A_and_b_gauss_newton: A row i (4) and b_i.
__host__ __device__ __forceinline__ void gn_row(const double* l, double rho_i, const double b[4], double A[4],
                                                double& r) {
  A[0] = 2 * l[0] * b[0] + l[1] * b[1] + l[3] * b[2] + l[6] * b[3];
  A[1] = l[1] * b[0] + 2 * l[2] * b[1] + l[4] * b[2] + l[7] * b[3];
  A[2] = l[3] * b[0] + l[4] * b[1] + 2 * l[5] * b[2] + l[8] * b[3];
  A[3] = l[6] * b[0] + l[7] * b[1] + l[8] * b[2] + 2 * l[9] * b[3];
  r = rho_i - (l[0] * b[0] * b[0] + l[1] * b[0] * b[1] + l[2] * b[1] * b[1] + l[3] * b[0] * b[2] +
               l[4] * b[1] * b[2] + l[5] * b[2] * b[2] + l[6] * b[0] * b[3] + l[7] * b[1] * b[3] +
               l[8] * b[2] * b[3] + l[9] * b[3] * b[3]);
}

// epnp::gauss_newton: 5 iterations of compute_A_and_b + qr_solve.  lds
// (device): the six rows of A and b are built one per lane (the same
// arithmetic per row) and gathered through this wave's LDS slice (30
// doubles), the wave-uniform QR solve then reads them -- a sixth of the
// row-building instructions of the issue-bound wave.
__host__ __device__ void gauss_newton(const double (&L)[6][10], const double (&rho)[6], double b[4],
                                      double* lds = nullptr) {
#if defined(__HIP_DEVICE_COMPILE__)
  {  // (every device caller passes its wave's slice)
    const int ln = threadIdx.x & 63, i = ln < 6 ? ln : 0;
    // lane i's row of L through the slice (a select chain over the rows
    // becomes a dynamically indexed L, i.e. scratch)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (earlier readers of the slice done)
    if (ln == 0) {
#pragma unroll
      for (int row = 0; row < 6; ++row) {
#pragma unroll
        for (int q = 0; q < 10; ++q) lds[10 * row + q] = L[row][q];
        lds[60 + row] = rho[row];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double l[10];
#pragma unroll
    for (int q = 0; q < 10; ++q) l[q] = lds[10 * i + q];
    const double rho_i = lds[60 + i];
    for (int it = 0; it < 5; ++it) {
      double Ai[4], ri;
      gn_row(l, rho_i, b, Ai, ri);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (the previous iteration's reads done)
      if (ln < 6) {
#pragma unroll
        for (int q = 0; q < 4; ++q) lds[5 * ln + q] = Ai[q];
        lds[5 * ln + 4] = ri;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      double A[6][4], r[6], x[4];
#pragma unroll
      for (int row = 0; row < 6; ++row) {
#pragma unroll
        for (int q = 0; q < 4; ++q) A[row][q] = lds[5 * row + q];
        r[row] = lds[5 * row + 4];
      }
      if (!qr_solve(A, r, x)) break;
#pragma unroll
      for (int q = 0; q < 4; ++q) b[q] += x[q];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (read before the slice is reused)
  }
#else
  (void)lds;
  for (int it = 0; it < 5; ++it) {
    double A[6][4], r[6], x[4];
#pragma unroll
    for (int i = 0; i < 6; ++i) gn_row(L[i], rho[i], b, A[i], r[i]);
    if (!qr_solve(A, r, x)) return;
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] += x[i];
  }
#endif
}

// EPnP of one 5-point subset, in three parts: the control points, the
// barycentric coordinates, the null space of M (the 12x12 SVD) and the
// distance constraints (epnp5_common), then the three beta solutions (N = 0,
// 1, 2 in OpenCV's order; epnp5_case), then the one with the smallest
// reprojection error.  Every lane of a wave computes the same (wave-uniform
// control flow); k_pnp_epnp runs the three cases in three waves.
struct EpnpCommon {
  double alpha[kModel][4];
  double ut[4][12];  // ut[q] = OpenCV's ut row 11 - q
  double L[6][10], rho[6];
};
__host__ __device__ void epnp5_common(const EpnpIn& in, const PnPCam& k, double* lds, EpnpCommon& cm) {
  // choose_control_points: centroid + PCA (cv::SVD of PW0^T PW0)
  double cws[4][3];
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    double s = 0.0;
#pragma unroll
    for (int p = 0; p < kModel; ++p) s += in.pw[p][m];
    cws[0][m] = s / kModel;
  }
  double pw0[kModel][3];
#pragma unroll
  for (int p = 0; p < kModel; ++p)
#pragma unroll
    for (int m = 0; m < 3; ++m) pw0[p][m] = in.pw[p][m] - cws[0][m];
  double ptp[3][3];
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      double s = 0.0;
#pragma unroll
      for (int p = 0; p < kModel; ++p) s += pw0[p][a] * pw0[p][b];
      ptp[a][b] = s;
    }
  {
    double Uc[3][3], dc[3], Vtc[3][3];
    cv_svd<3, 3>(ptp, Uc, dc, Vtc);
#pragma unroll
    for (int i = 1; i < 4; ++i) {
      const double kk = sqrt(dc[i - 1] / kModel);
#pragma unroll
      for (int m = 0; m < 3; ++m) cws[i][m] = cws[0][m] + kk * Uc[i - 1][m];
    }
  }
  // compute_barycentric_coordinates: cvInvert(CC, CV_SVD) = SVBkSb pinv
  double ci[3][3];
  {
    double cc[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 1; j < 4; ++j) cc[i][j - 1] = cws[j][i] - cws[0][i];
    double Uc[3][3], wc[3], Vtc[3][3];
    cv_svd<3, 3>(cc, Uc, wc, Vtc);
    double thr = (wc[0] + wc[1] + wc[2]) * (kDblEps * 2);
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int q = 0; q < 3; ++q) ci[j][q] = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      double wi = wc[i];
      if (fabs(wi) <= thr) continue;
      wi = 1.0 / wi;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const double vw = Vtc[i][j] * wi;
#pragma unroll
        for (int q = 0; q < 3; ++q) ci[j][q] = ci[j][q] + vw * Uc[i][q];
      }
    }
  }
  double (&alpha)[kModel][4] = cm.alpha;
#pragma unroll
  for (int p = 0; p < kModel; ++p) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
      alpha[p][1 + j] = ci[j][0] * (in.pw[p][0] - cws[0][0]) + ci[j][1] * (in.pw[p][1] - cws[0][1]) +
                        ci[j][2] * (in.pw[p][2] - cws[0][2]);
    alpha[p][0] = 1.0 - alpha[p][1] - alpha[p][2] - alpha[p][3];
  }
  // M^T M (cvMulTransposed: the rows of M summed in order), then cv::SVD of
  // it.  The 5-point problem leaves a 2-D (near-)null space whose basis any
  // change of rounding rotates, so the device and the oracle fix one order:
  // sequential over the rows of M, the 16-lane butterfly over the 12 entries
  // of a row of At (cv_svd12_lanes; oracle cv_svd(tree=True)).
  double (&ut)[4][12] = cm.ut;
  {
    double M1[kModel][12], M2[kModel][12];
#pragma unroll
    for (int p = 0; p < kModel; ++p)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        M1[p][3 * jj] = alpha[p][jj] * k.fu; M1[p][3 * jj + 1] = 0.0;
        M1[p][3 * jj + 2] = alpha[p][jj] * (k.uc - in.us[p][0]);
        M2[p][3 * jj] = 0.0; M2[p][3 * jj + 1] = alpha[p][jj] * k.fv;
        M2[p][3 * jj + 2] = alpha[p][jj] * (k.vc - in.us[p][1]);
      }
#if defined(__HIP_DEVICE_COMPILE__)
    // lane col (mod 16) holds column col of M^T M = entry col of every row of At
    const int col = threadIdx.x & 15;
    double mc1[kModel], mc2[kModel];  // this lane's column of M (row p of M1 / M2)
#pragma unroll
    for (int p = 0; p < kModel; ++p) {
      mc1[p] = 0.0;
      mc2[p] = 0.0;
#pragma unroll
      for (int c = 0; c < 12; ++c) {
        mc1[p] = c == col ? M1[p][c] : mc1[p];
        mc2[p] = c == col ? M2[p][c] : mc2[p];
      }
    }
    double u[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      double acc = 0.0;
#pragma unroll
      for (int p = 0; p < kModel; ++p) {
        acc = acc + M1[p][i] * mc1[p];
        acc = acc + M2[p][i] * mc2[p];
      }
      u[i] = col < 12 ? acc : 0.0;
    }
    cv_svd12_lanes(u, lds, ut);
#else
    double MtM[12][12];
#pragma unroll
    for (int x = 0; x < 12; ++x)
#pragma unroll
      for (int y = 0; y < 12; ++y) {
        double acc = 0.0;
#pragma unroll
        for (int p = 0; p < kModel; ++p) {
          acc = acc + M1[p][x] * M1[p][y];
          acc = acc + M2[p][x] * M2[p][y];
        }
        MtM[x][y] = acc;
      }
    host_svd12_tree(MtM, ut);
#endif
  }
  double (&L)[6][10] = cm.L;
  double (&rho)[6] = cm.rho;
  {
    const int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      double dv[4][3];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int m = 0; m < 3; ++m) dv[q][m] = ut[q][3 * pa[i] + m] - ut[q][3 * pb[i] + m];
      L[i][0] = dot3(dv[0], dv[0]); L[i][1] = 2.0 * dot3(dv[0], dv[1]); L[i][2] = dot3(dv[1], dv[1]);
      L[i][3] = 2.0 * dot3(dv[0], dv[2]); L[i][4] = 2.0 * dot3(dv[1], dv[2]); L[i][5] = dot3(dv[2], dv[2]);
      L[i][6] = 2.0 * dot3(dv[0], dv[3]); L[i][7] = 2.0 * dot3(dv[1], dv[3]); L[i][8] = 2.0 * dot3(dv[2], dv[3]);
      L[i][9] = dot3(dv[3], dv[3]);
      const double d0 = cws[pa[i]][0] - cws[pb[i]][0], d1 = cws[pa[i]][1] - cws[pb[i]][1],
                   d2 = cws[pa[i]][2] - cws[pb[i]][2];
      rho[i] = d0 * d0 + d1 * d1 + d2 * d2;
    }
  }
}

__host__ __device__ double epnp5_case(int N, const EpnpIn& in, const PnPCam& k, const EpnpCommon& cm, double R[9],
                                      double t[3], double* lds = nullptr) {
  const double (&alpha)[kModel][4] = cm.alpha;
  const double (&ut)[4][12] = cm.ut;
  const double (&L)[6][10] = cm.L;
  const double (&rho)[6] = cm.rho;
  if (N == 0) {
    double A4[6][4], b4[4];
#pragma unroll
    for (int i = 0; i < 6; ++i) { A4[i][0] = L[i][0]; A4[i][1] = L[i][1]; A4[i][2] = L[i][3]; A4[i][3] = L[i][6]; }
    cv_lstsq<6, 4>(A4, rho, b4, lds);
    double be[4];
    if (b4[0] < 0) {
      be[0] = sqrt(-b4[0]); be[1] = -b4[1] / be[0]; be[2] = -b4[2] / be[0]; be[3] = -b4[3] / be[0];
    } else {
      be[0] = sqrt(b4[0]); be[1] = b4[1] / be[0]; be[2] = b4[2] / be[0]; be[3] = b4[3] / be[0];
    }
    gauss_newton(L, rho, be, lds);
    return r_and_t(in, alpha, ut, be, k, R, t);
  } else if (N == 1) {
    double A3[6][3], b3[3];
#pragma unroll
    for (int i = 0; i < 6; ++i) { A3[i][0] = L[i][0]; A3[i][1] = L[i][1]; A3[i][2] = L[i][2]; }
    cv_lstsq<6, 3>(A3, rho, b3, lds);
    double be[4];
    if (b3[0] < 0) { be[0] = sqrt(-b3[0]); be[1] = b3[2] < 0 ? sqrt(-b3[2]) : 0.0; }
    else { be[0] = sqrt(b3[0]); be[1] = b3[2] > 0 ? sqrt(b3[2]) : 0.0; }
    if (b3[1] < 0) be[0] = -be[0];
    be[2] = 0.0; be[3] = 0.0;
    gauss_newton(L, rho, be, lds);
    return r_and_t(in, alpha, ut, be, k, R, t);
  } else {
    double A5[6][5], b5[5];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 5; ++j) A5[i][j] = L[i][j];
    cv_lstsq<6, 5>(A5, rho, b5, lds);
    double be[4];
    if (b5[0] < 0) { be[0] = sqrt(-b5[0]); be[1] = b5[2] < 0 ? sqrt(-b5[2]) : 0.0; }
    else { be[0] = sqrt(b5[0]); be[1] = b5[2] > 0 ? sqrt(b5[2]) : 0.0; }
    if (b5[1] < 0) be[0] = -be[0];
    be[2] = b5[3] / be[0];
    be[3] = 0.0;
    gauss_newton(L, rho, be, lds);
    return r_and_t(in, alpha, ut, be, k, R, t);
  }
}

__host__ __device__ void epnp5(const EpnpIn& in, const PnPCam& k, double* lds, double R[9], double t[3]) {
  EpnpCommon cm;
  epnp5_common(in, k, lds, cm);
  double Rs[3][9], ts[3][3], err[3];
#pragma unroll
  for (int n = 0; n < 3; ++n) err[n] = epnp5_case(n, in, k, cm, Rs[n], ts[n]);
  int N = 0;
  if (err[1] < err[0]) N = 1;
  if (err[2] < err[N]) N = 2;
#pragma unroll
  for (int i = 0; i < 9; ++i) R[i] = N == 0 ? Rs[0][i] : N == 1 ? Rs[1][i] : Rs[2][i];
#pragma unroll
  for (int i = 0; i < 3; ++i) t[i] = N == 0 ? ts[0][i] : N == 1 ? ts[1][i] : ts[2][i];
}

// cv::RNG(uint64(-1)) subsets of the whole iteration bound (one thread).
// nd: the point count on the device (sfm_track_pnp; n otherwise), below
// `gate` no model is sought (zero subsets keep the later kernels in bounds).
__global__ void k_pnp_subsets(int n_arg, const int* __restrict__ nd, int gate, int iters, int* __restrict__ sub) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int n = nd ? *nd : n_arg;
  if (n < gate) {
    for (int i = 0; i < iters * kModel; ++i) sub[i] = 0;
    return;
  }
  uint64_t state = ~0ull;
  auto next = [&]() -> unsigned { return cv_rng_next(state); };
  for (int it = 0; it < iters; ++it) {
    int idx[kModel];
    if (n == kModel) {
      for (int i = 0; i < kModel; ++i) idx[i] = i;
    } else {
      for (int i = 0; i < kModel; ++i) {
        int v;
        while (true) {
          v = int(next() % unsigned(n));
          int j = 0;
          for (; j < i; ++j)
            if (idx[j] == v) break;
          if (j == i) break;
        }
        idx[i] = v;
      }
    }
    for (int i = 0; i < kModel; ++i) sub[it * kModel + i] = idx[i];
  }
}

// One workgroup of three waves per hypothesis: EPnP on its subset -> model
// (rvec 3 | tvec 3).  Every wave computes the common part (the SVD of M is
// the long pole and a wave-wide exchange); wave w then solves beta case w,
// and wave 0 picks the case with the smallest reprojection error as epnp5
// does (err[1] < err[0], then err[2] < err[N]).
__global__ __launch_bounds__(192) void k_pnp_epnp(const double* __restrict__ obj, const double* __restrict__ img,
                                                  const int* __restrict__ sub, PnPCam k, double* __restrict__ model) {
  __shared__ __attribute__((aligned(16))) double lds[3][kSvdLds];
  __shared__ double res[3][13];
  const int it = blockIdx.x;
  const int w = threadIdx.x >> 6;
  EpnpIn in;
#pragma unroll
  for (int p = 0; p < kModel; ++p) {
    const int q = sub[it * kModel + p];
#pragma unroll
    for (int m = 0; m < 3; ++m) in.pw[p][m] = double(float(obj[3 * q + m]));
    // undistortPoints (normalised, stored as float), mapped back by epnp
    const float xn = float((double(float(img[2 * q])) - k.uc) * (1.0 / k.fu));
    const float yn = float((double(float(img[2 * q + 1])) - k.vc) * (1.0 / k.fv));
    in.us[p][0] = double(xn) * k.fu + k.uc;
    in.us[p][1] = double(yn) * k.fv + k.vc;
  }
  EpnpCommon cm;
  epnp5_common(in, k, lds[w], cm);
  double R[9], t[3], r[3];
  const double e = epnp5_case(w, in, k, cm, R, t, lds[w]);
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int i = 0; i < 9; ++i) res[w][i] = R[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) res[w][9 + i] = t[i];
    res[w][12] = e;
  }
  __syncthreads();
  if (w != 0) return;
  int N = 0;
  if (res[1][12] < res[0][12]) N = 1;
  if (res[2][12] < res[N][12]) N = 2;
#pragma unroll
  for (int i = 0; i < 9; ++i) R[i] = res[N][i];
#pragma unroll
  for (int i = 0; i < 3; ++i) t[i] = res[N][9 + i];
  rodrigues_m2v(R, r);
  if (threadIdx.x == 0) {
    double* o = model + 6 * it;
    o[0] = r[0]; o[1] = r[1]; o[2] = r[2]; o[3] = t[0]; o[4] = t[1]; o[5] = t[2];
  }
}

// PnPRansacCallback::computeError + findInliers for object point q.
__device__ __forceinline__ bool pnp_inlier(const double* __restrict__ obj, const double* __restrict__ img, int q,
                                           const double R[9], const double t[3], const PnPCam& k, float thr) {
  const double x = double(float(obj[3 * q])), y = double(float(obj[3 * q + 1])), z = double(float(obj[3 * q + 2]));
  const double X = R[0] * x + R[1] * y + R[2] * z + t[0];
  const double Y = R[3] * x + R[4] * y + R[5] * z + t[1];
  const double Z = R[6] * x + R[7] * y + R[8] * z + t[2];
  const double iz = Z != 0.0 ? 1.0 / Z : 1.0;
  const float pu = float(X * iz * k.fu + k.uc), pv = float(Y * iz * k.fv + k.vc);
  const float du = float(img[2 * q]) - pu, dv = float(img[2 * q + 1]) - pv;
  const float e = float(sqrt(double(du) * du + double(dv) * dv));
  return e <= thr;
}

__global__ __launch_bounds__(256) void k_pnp_count(int n_arg, const int* __restrict__ nd, const double* __restrict__ obj,
                                                   const double* __restrict__ img, const double* __restrict__ model,
                                                   PnPCam k, float thr, int* __restrict__ cnt) {
  __shared__ int sh[4];
  const int n = nd ? *nd : n_arg;
  const int it = blockIdx.x;
  double R[9], t[3];
  rodrigues_v2m(model + 6 * it, R);
  t[0] = model[6 * it + 3]; t[1] = model[6 * it + 4]; t[2] = model[6 * it + 5];
  int c = 0;
  for (int q = threadIdx.x; q < n; q += 256) c += pnp_inlier(obj, img, q, R, t, k, thr) ? 1 : 0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[it] = sh[0] + sh[1] + sh[2] + sh[3];
}

// Replay of RANSACPointSetRegistrator::run's acceptance over the counts, then
// the winner's inliers in index order.  One wave.  res: [0] found, [1] best
// iteration, [2] inlier count.
__global__ __launch_bounds__(64) void k_pnp_select(int n_arg, const int* __restrict__ nd, int gate, int iters,
                                                   double confidence, const double* __restrict__ obj,
                                                   const double* __restrict__ img, const double* __restrict__ model,
                                                   const int* __restrict__ cnt, PnPCam k, float thr,
                                                   int* __restrict__ res, int* __restrict__ inl) {
  const int lane = threadIdx.x;
  const int n = nd ? *nd : n_arg;
  if (n < gate) {
    if (lane == 0) { res[0] = 0; res[1] = -1; res[2] = 0; }
    return;
  }
  int best = -1, max_good = 0;
  int niters = iters > 1 ? iters : 1;
  for (int it = 0; it < niters && it < iters; ++it) {
    const int good = cnt[it];
    if (n == kModel) { best = it; max_good = n; break; }
    if (good > (max_good > kModel - 1 ? max_good : kModel - 1)) {
      best = it;
      max_good = good;
      // RANSACUpdateNumIters(confidence, outlier ratio, 5, niters)
      double p = fmin(fmax(confidence, 0.0), 1.0), ep = fmin(fmax(double(n - good) / n, 0.0), 1.0);
      double num = fmax(1.0 - p, DBL_MIN);
      double denom = 1.0 - pow(1.0 - ep, double(kModel));
      if (denom < DBL_MIN) {
        niters = 0;
      } else {
        num = log(num);
        denom = log(denom);
        niters = (denom >= 0 || -num >= niters * (-denom)) ? niters : int(rint(num / denom));
      }
    }
  }
  if (lane == 0) { res[0] = best >= 0 ? 1 : 0; res[1] = best; res[2] = best >= 0 ? max_good : 0; }
  if (best < 0) return;
  // the winner's model next to the counts (res + 4: 16-B aligned), so one
  // download returns counts, model and inliers
  if (lane < 6) reinterpret_cast<double*>(res + 4)[lane] = model[6 * best + lane];
  if (n == kModel) {  // run() with count == modelPoints: the mask is all ones
    if (lane < kModel) inl[lane] = lane;
    return;
  }
  double R[9], t[3];
  rodrigues_v2m(model + 6 * best, R);
  t[0] = model[6 * best + 3]; t[1] = model[6 * best + 4]; t[2] = model[6 * best + 5];
  int base = 0;
  for (int q0 = 0; q0 < n; q0 += 64) {
    const int q = q0 + lane;
    const bool in = q < n && pnp_inlier(obj, img, q, R, t, k, thr);
    const unsigned long long m = __ballot(in);
    if (in) inl[base + __popcll(m & ((1ull << lane) - 1ull))] = q;
    base += __popcll(m);
  }
}

struct PnPCtx {
  hipStream_t stream = nullptr;
  size_t cap = 0;
  double* obj = nullptr;
  double* img = nullptr;
  // one device block returned by ONE download: counts (4 ints), the
  // winner's model (6 doubles), the inlier list (cap ints)
  int* out = nullptr;
  int* inl = nullptr;
  uint8_t* pin = nullptr;  // pinned staging: the points up, the block down
  size_t pin_cap = 0;
  int* sub = nullptr;
  int sub_n = -1, sub_iters = -1;  // the (n, iterations) whose subsets `sub` holds
  double* model = nullptr;
  int* cnt = nullptr;
  ~PnPCtx() {
    if (stream) hipStreamSynchronize(stream);
    hipFree(obj); hipFree(img); hipFree(out); hipFree(sub); hipFree(model); hipFree(cnt);
    if (pin) hipHostFree(pin);
    if (stream) hipStreamDestroy(stream);
  }
};

int pfail(int code, const char* msg) {
  sfm_internal_set_error(msg);
  return code;
}

}  // namespace
}  // namespace sfm

namespace sfm {
// cv::solvePnPRansac on points already on the device, their count at d_n
// (device; below `gate` no model: found = 0), launched on stream s without
// a synchronisation (sfm_track_pnp).  Scratch from the caller: d_sub
// [kModel kMaxIters], d_model [6 kMaxIters], d_cnt [kMaxIters]; result block
// d_res: found, best iteration, inlier count, (pad) | the model (6 doubles,
// 16-B aligned) | then d_inl [n_cap] the inliers' indices.
int pnp_ransac_dev(hipStream_t s, const int* d_n, int gate, const double* d_obj, const double* d_img, const double* K9,
                   int iterations, double reproj_err, double confidence, int* d_sub, double* d_model, int* d_cnt,
                   int* d_res, int* d_inl) {
  if (iterations < 0 || iterations > kMaxIters) return pfail(SFM_EINVAL, "bad iterations");
  if (!(confidence > 0.0 && confidence < 1.0)) return pfail(SFM_EINVAL, "confidence must lie in (0, 1)");
  const PnPCam k{K9[0], K9[4], K9[2], K9[5]};
  const int iters = iterations > 0 ? iterations : 1;
  const float thr = float(reproj_err * reproj_err);
  gate = gate > kModel ? gate : kModel;
  k_pnp_subsets<<<1, 64, 0, s>>>(0, d_n, gate, iters, d_sub);
  k_pnp_epnp<<<iters, 192, 0, s>>>(d_obj, d_img, d_sub, k, d_model);
  k_pnp_count<<<iters, 256, 0, s>>>(0, d_n, d_obj, d_img, d_model, k, thr, d_cnt);
  k_pnp_select<<<1, 64, 0, s>>>(0, d_n, gate, iters, confidence, d_obj, d_img, d_model, d_cnt, k, thr, d_res, d_inl);
  return hipGetLastError() == hipSuccess ? 0 : pfail(SFM_EIO, "PnP launch failed");
}
int pnp_max_iters() { return kMaxIters; }
int pnp_model_size() { return kModel; }
}  // namespace sfm

using namespace sfm;

extern "C" int sfm_pnp_ransac(int32_t device, int32_t n, const double* obj, const double* img, const double* K9,
                              int32_t iterations, double reproj_err, double confidence, double* rvec, double* tvec,
                              int32_t* inliers, int32_t* n_inliers, int32_t* found) {
  SFM_TRACE("sfm_pnp_ransac");
  if (!found || !n_inliers || !rvec || !tvec || !K9) return pfail(SFM_EINVAL, "NULL argument");
  *found = 0;
  *n_inliers = 0;
  if (n < 0 || iterations < 0 || iterations > kMaxIters) return pfail(SFM_EINVAL, "bad n or iterations");
  if (!(confidence > 0.0 && confidence < 1.0)) return pfail(SFM_EINVAL, "confidence must lie in (0, 1)");
  if (n > 0 && (!obj || !img)) return pfail(SFM_EINVAL, "NULL point arrays");
  if (n < kModel) return 0;  // RANSAC needs a full subset: no model (as cv::solvePnPRansac's false)
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return pfail(SFM_ENODEV, "no device");
  if (hipSetDevice(device) != hipSuccess) return pfail(SFM_ENODEV, "hipSetDevice failed");
  struct Cache {
    std::map<int, PnPCtx*> m;
    ~Cache() {
      for (auto& kv : m) delete kv.second;
    }
  };
  static thread_local Cache cache;
  PnPCtx*& c = cache.m[device];
  if (!c) {
    c = new PnPCtx();
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
      delete c;
      c = nullptr;
      return pfail(SFM_EIO, "hipStreamCreate failed");
    }
    if (hipMalloc(&c->sub, sizeof(int) * kModel * kMaxIters) != hipSuccess ||
        hipMalloc(&c->model, sizeof(double) * 6 * kMaxIters) != hipSuccess ||
        hipMalloc(&c->cnt, sizeof(int) * kMaxIters) != hipSuccess)
      return pfail(SFM_ENOMEM, "hipMalloc failed");
  }
  // result block: counts (4 ints = 16 B) | winner's model (6 doubles) | inliers
  constexpr size_t kOutHead = 16 + 6 * sizeof(double);
  if (size_t(n) > c->cap) {
    hipFree(c->obj); hipFree(c->img); hipFree(c->out);
    c->obj = nullptr; c->img = nullptr; c->out = nullptr; c->inl = nullptr; c->cap = 0;
    if (c->pin) hipHostFree(c->pin);
    c->pin = nullptr;
    const size_t cap = std::max<size_t>(size_t(n), 1024);
    if (hipMalloc(&c->obj, sizeof(double) * 3 * cap) != hipSuccess ||
        hipMalloc(&c->img, sizeof(double) * 2 * cap) != hipSuccess ||
        hipMalloc(&c->out, kOutHead + sizeof(int) * cap) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&c->pin), sizeof(double) * 5 * cap + kOutHead + sizeof(int) * cap) !=
            hipSuccess)
      return pfail(SFM_ENOMEM, "hipMalloc failed");
    c->inl = reinterpret_cast<int*>(reinterpret_cast<uint8_t*>(c->out) + kOutHead);
    c->cap = cap;
  }
  const PnPCam k{K9[0], K9[4], K9[2], K9[5]};
  const int iters = iterations > 0 ? iterations : 1;
  const float thr = float(reproj_err * reproj_err);
  hipStream_t s = c->stream;
  // the points through the pinned stage (the previous call has drained the
  // stream: it synchronised before returning)
  double* pin_obj = reinterpret_cast<double*>(c->pin);
  double* pin_img = pin_obj + 3 * size_t(n);
  uint8_t* pin_out = c->pin + sizeof(double) * 5 * c->cap;
  std::memcpy(pin_obj, obj, sizeof(double) * 3 * size_t(n));
  std::memcpy(pin_img, img, sizeof(double) * 2 * size_t(n));
  if (hipMemcpyAsync(c->obj, pin_obj, sizeof(double) * 3 * size_t(n), hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(c->img, pin_img, sizeof(double) * 2 * size_t(n), hipMemcpyHostToDevice, s) != hipSuccess)
    return pfail(SFM_EIO, "upload failed");
  // the subsets depend on (n, iterations) alone (cv::RNG(-1) restarted per
  // call): drawn once per pair, then reused
  if (c->sub_n != n || c->sub_iters != iters) {
    k_pnp_subsets<<<1, 64, 0, s>>>(n, nullptr, kModel, iters, c->sub);
    c->sub_n = n;
    c->sub_iters = iters;
  }
  k_pnp_epnp<<<iters, 192, 0, s>>>(c->obj, c->img, c->sub, k, c->model);
  k_pnp_count<<<iters, 256, 0, s>>>(n, nullptr, c->obj, c->img, c->model, k, thr, c->cnt);
  k_pnp_select<<<1, 64, 0, s>>>(n, nullptr, kModel, iters, confidence, c->obj, c->img, c->model, c->cnt, k, thr,
                                c->out, c->inl);
  // ONE download: counts, model and (up to n) inliers
  const size_t down = kOutHead + (inliers ? sizeof(int) * size_t(n) : 0);
  if (hipMemcpyAsync(pin_out, c->out, down, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return pfail(SFM_EIO, "PnP kernels failed");
  int res[4];
  double mdl[6];
  std::memcpy(res, pin_out, sizeof(res));
  if (!res[0]) return 0;
  std::memcpy(mdl, pin_out + 16, sizeof(mdl));
  if (inliers && res[2] > 0) std::memcpy(inliers, pin_out + kOutHead, sizeof(int) * size_t(res[2]));
  for (int i = 0; i < 3; ++i) { rvec[i] = mdl[i]; tvec[i] = mdl[3 + i]; }
  *n_inliers = res[2];
  *found = 1;
  return 0;
}
