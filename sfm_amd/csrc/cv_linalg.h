// OpenCV 3.0's small dense linear algebra (lapack.cpp JacobiSVDImpl_ /
// SVBkSbImpl_, epnp.cpp qr_solve) as __host__ __device__ routines, for the
// geometry kernels that restate OpenCV calls of the reference pipeline
// (pnp_kernels.hip: solvePnPRansac; tri_kernels.hip: triangulatePoints).
// Compile the including file with -ffp-contract=off: products and sums then
// round as OpenCV's SSE2 build and the oracle (oracle/pnp_oracle.py) do.
#pragma once
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <utility>
#include "svd_schedule.h"

namespace sfm {
namespace {

constexpr double kDblEps = DBL_EPSILON, kDblMin = DBL_MIN;

__host__ __device__ __forceinline__ unsigned cv_rng_next(uint64_t& state) {
  state = uint64_t(unsigned(state)) * 4164903690ull + (state >> 32);
  return unsigned(state);
}

// cv::SVD of A (M x N, M >= N) as JacobiSVDImpl_ computes it: one-sided
// Jacobi on the rows of At = A^T (eps 10 DBL_EPSILON, max(M, 30) sweeps),
// singular values sorted descending, rows of At normalised to the left
// singular vectors (zero singular values completed from cv::RNG(0x12345678)
// vectors).  On return U[i] = i-th left singular vector (At row i), w
// descending, Vt rows = right singular vectors.
// In place on At (= A^T, N rows of length M); kV = false skips the right
// singular vectors (Vt is then not touched): EPnP needs only U of M^T M,
// and without the second 12x12 array the kernel stays in registers.
// The sweeps (until one rotates nothing, at most max(M, 30)), in OpenCV's
// order, one rotation after another.
template <int M, int N, bool kV>
__host__ __device__ void cv_svd_sweeps(double (&U)[N][M], double (&W)[N], double (&Vt)[N][N]) {
  const double eps = kDblEps * 10;
  for (int iter = 0; iter < (M > 30 ? M : 30); ++iter) {
    bool changed = false;
#pragma unroll
    for (int i = 0; i < N - 1; ++i)
#pragma unroll
      for (int j = i + 1; j < N; ++j) {
        double a = W[i], b = W[j], p = 0.0;
#pragma unroll
        for (int k = 0; k < M; ++k) p += U[i][k] * U[j][k];
        if (fabs(p) <= eps * sqrt(a * b)) continue;
        p *= 2;
        // hypot as sqrt(p^2 + beta^2): one formula on every side (std::hypot /
        // CPython / ocml disagree in the last ulp, which rotates the 2-D
        // near-null space of the 5-point M^T M arbitrarily)
        const double beta = a - b, gamma = sqrt(p * p + beta * beta);
        double c, s;
        if (beta < 0) {
          const double delta = (gamma - beta) * 0.5;
          s = sqrt(delta / gamma);
          c = p / (gamma * s * 2);
        } else {
          c = sqrt((gamma + beta) / (gamma * 2));
          s = p / (gamma * c * 2);
        }
        a = b = 0.0;
#pragma unroll
        for (int k = 0; k < M; ++k) {
          const double t0 = c * U[i][k] + s * U[j][k], t1 = -s * U[i][k] + c * U[j][k];
          U[i][k] = t0; U[j][k] = t1;
          a += t0 * t0; b += t1 * t1;
        }
        W[i] = a; W[j] = b;
        changed = true;
        if (kV)
#pragma unroll
          for (int k = 0; k < N; ++k) {
            const double t0 = c * Vt[i][k] + s * Vt[j][k], t1 = -s * Vt[i][k] + c * Vt[j][k];
            Vt[i][k] = t0; Vt[j][k] = t1;
          }
      }
    if (!changed) break;
  }
}

#if defined(__HIP_DEVICE_COMPILE__)
// The same sweeps with one row per lane (lane r < N holds row r of At, of
// Vt and W_r), for the 4- and 5-row SVDs of the EPnP beta cases: two
// rotations on disjoint rows per pass, the tail of sweep s overlapped with
// the head of sweep s + 1 once sweep s has rotated something
// (svd_schedule.h, tools/svd_schedule.py; the 12x12 of pnp_kernels.hip
// cv_svd12_lanes does the same with four 16-lane rotations).  Both lanes of
// a rotation fetch the partner's row and compute the same p, c, s (the
// products commute, the sums keep OpenCV's order); lane i keeps c*U_i +
// s*U_j, lane j -s*U_i + c*U_j, exactly the sequential rotation's values.
template <int N, int S>
struct LaneSched;
#define SFM_LANE_SCHED(NR, SS, NAME)                         \
  template <>                                                \
  struct LaneSched<NR, SS> {                                 \
    static constexpr int P = kSvd##NAME##Passes;             \
    static constexpr const int* Nr = kSvd##NAME##N;          \
    static constexpr const int (*I)[2] = kSvd##NAME##I;      \
    static constexpr const int (*J)[2] = kSvd##NAME##J;      \
    static constexpr const int (*T)[2] = kSvd##NAME##T;      \
  };
SFM_LANE_SCHED(4, 0, L4Pro)
SFM_LANE_SCHED(4, 1, L4Per)
SFM_LANE_SCHED(4, 2, L4Epi)
SFM_LANE_SCHED(5, 0, L5Pro)
SFM_LANE_SCHED(5, 1, L5Per)
SFM_LANE_SCHED(5, 2, L5Epi)
#undef SFM_LANE_SCHED

__device__ __forceinline__ void cvl_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int M, int N, int S, int ps>
__device__ __forceinline__ void lane_pass(int r, double (&u)[M], double (&v)[N], double& wr, bool (&ch)[2]) {
  using Sc = LaneSched<N, S>;
  constexpr int n = Sc::Nr[ps];
  constexpr int i0 = Sc::I[ps][0], j0 = Sc::J[ps][0], i1 = Sc::I[ps][1], j1 = Sc::J[ps][1];
  constexpr uint64_t kTag1 = (Sc::T[ps][0] ? (1ull << i0) | (1ull << j0) : 0) |
                             (n > 1 && Sc::T[ps][1] ? (1ull << i1) | (1ull << j1) : 0);
  int partner = r;
  bool lo = false;
  if (r == i0) { partner = j0; lo = true; }
  if (r == j0) partner = i0;
  if (n > 1 && r == i1) { partner = j1; lo = true; }
  if (n > 1 && r == j1) partner = i1;
  double pu[M], pv[N];
#pragma unroll
  for (int k = 0; k < M; ++k) pu[k] = __shfl(u[k], partner);
#pragma unroll
  for (int k = 0; k < N; ++k) pv[k] = __shfl(v[k], partner);
  // the partner's W is the sum of squares of its row in order (as set after
  // its last rotation, or initially): recomputed here, not fetched
  double p = 0.0, pw = 0.0;
#pragma unroll
  for (int k = 0; k < M; ++k) {
    p += u[k] * pu[k];
    pw += pu[k] * pu[k];
  }
  const double a = lo ? wr : pw, b = lo ? pw : wr;
  const bool act = partner != r && !(fabs(p) <= kDblEps * 10 * sqrt(a * b));
  const uint64_t turned = __builtin_amdgcn_ballot_w64(act);
  if (turned == 0) return;
  if (turned & kTag1) ch[1] = true;
  if (turned & ~kTag1) ch[0] = true;
  p *= 2;
  const double beta = a - b, gamma = sqrt(p * p + beta * beta);
  // the two cases of the rotation with their operands selected (see
  // cv_svd_sweeps): the same operations on the same values either way
  const bool neg = beta < 0;
  const double num = neg ? (gamma - beta) * 0.5 : gamma + beta;
  const double den = neg ? gamma : gamma * 2;
  const double s1 = sqrt(num / den);
  const double o = p / (gamma * s1 * 2);
  const double c = neg ? o : s1, s = neg ? s1 : o;
  // lane i: c U_i + s U_j; lane j: -s U_i + c U_j = c U_j + (-s) U_i (the
  // sum commutes): both c * own + cb * partner, no per-entry select
  const double cb = lo ? s : -s;
  double nu[M], nv[N], nw = 0.0;
#pragma unroll
  for (int k = 0; k < M; ++k) {
    const double t = c * u[k] + cb * pu[k];
    nu[k] = t;
    nw += t * t;
  }
#pragma unroll
  for (int k = 0; k < N; ++k) nv[k] = c * v[k] + cb * pv[k];
  if (act) {
#pragma unroll
    for (int k = 0; k < M; ++k) u[k] = nu[k];
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = nv[k];
    wr = nw;
  }
}
template <int M, int N, int S, int... ps>
__device__ __forceinline__ void lane_run(int r, double (&u)[M], double (&v)[N], double& wr, bool (&ch)[2],
                                         std::integer_sequence<int, ps...>) {
  (lane_pass<M, N, S, ps>(r, u, v, wr, ch), ...);
}
template <int M, int N, int S>
__device__ __forceinline__ void lane_run(int r, double (&u)[M], double (&v)[N], double& wr, bool (&ch)[2]) {
  lane_run<M, N, S>(r, u, v, wr, ch, std::make_integer_sequence<int, LaneSched<N, S>::P>{});
}

// lds: N (M + N) doubles of this wave's LDS
template <int M, int N>
__device__ void cv_svd_sweeps_lanes(double (&U)[N][M], double (&W)[N], double (&Vt)[N][N], double* lds) {
  const int r = threadIdx.x & 63;
  double u[M], v[N], wr = W[0];
#pragma unroll
  for (int k = 0; k < M; ++k) u[k] = U[0][k];
#pragma unroll
  for (int i = 1; i < N; ++i) {
    wr = r == i ? W[i] : wr;
#pragma unroll
    for (int k = 0; k < M; ++k) u[k] = r == i ? U[i][k] : u[k];
  }
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] = r == k ? 1.0 : 0.0;  // (Vt = I on entry)
  constexpr int kSweeps = M > 30 ? M : 30;
  bool ch[2] = {false, false}, head = true;
  for (int s = 0;;) {
    if (head) lane_run<M, N, 0>(r, u, v, wr, ch);  // head of sweep s (tag 1)
    head = false;
    if (ch[1] && s + 1 < kSweeps) {  // sweep s has turned: its tail with sweep s + 1's head
      ch[0] = ch[1] = false;
      lane_run<M, N, 1>(r, u, v, wr, ch);
      ++s;
    } else {
      const bool turned = ch[1];
      ch[0] = false;
      lane_run<M, N, 2>(r, u, v, wr, ch);  // tail of sweep s (tag 0)
      if (!(turned || ch[0]) || ++s >= kSweeps) break;
      ch[1] = false;
      head = true;
    }
  }
  cvl_wave_sync();  // (earlier readers of this LDS slice done)
  if (r < N) {
#pragma unroll
    for (int k = 0; k < M; ++k) lds[r * (M + N) + k] = u[k];
#pragma unroll
    for (int k = 0; k < N; ++k) lds[r * (M + N) + M + k] = v[k];
  }
  cvl_wave_sync();
#pragma unroll
  for (int i = 0; i < N; ++i) {
#pragma unroll
    for (int k = 0; k < M; ++k) U[i][k] = lds[i * (M + N) + k];
#pragma unroll
    for (int k = 0; k < N; ++k) Vt[i][k] = lds[i * (M + N) + M + k];
  }
  cvl_wave_sync();  // (read before the slice is reused)
}
#endif

// lds (device, kV, N = 4 or 5): the sweeps one row per lane through this
// wave's LDS slice of N (M + N) doubles; nullptr: one rotation after another.
template <int M, int N, bool kV>
__host__ __device__ void cv_svd_at(double (&U)[N][M], double (&w)[N], double (&Vt)[N][N], double* lds = nullptr) {
  double W[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double sd = 0.0;
#pragma unroll
    for (int k = 0; k < M; ++k) sd += U[i][k] * U[i][k];
    W[i] = sd;
    if (kV)
#pragma unroll
      for (int k = 0; k < N; ++k) Vt[i][k] = i == k ? 1.0 : 0.0;
  }
  const double eps = kDblEps * 10;
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (kV && (N == 4 || N == 5)) {
    if (lds) cv_svd_sweeps_lanes<M, N>(U, W, Vt, lds);
    else cv_svd_sweeps<M, N, kV>(U, W, Vt);
  } else {
    cv_svd_sweeps<M, N, kV>(U, W, Vt);
  }
#else
  (void)lds;
  cv_svd_sweeps<M, N, kV>(U, W, Vt);
#endif
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double sd = 0.0;
#pragma unroll
    for (int k = 0; k < M; ++k) sd += U[i][k] * U[i][k];
    W[i] = sqrt(sd);
  }
#pragma unroll
  for (int i = 0; i < N - 1; ++i) {
    int j = i;
#pragma unroll
    for (int k = i + 1; k < N; ++k)
      if (W[j] < W[k]) j = k;
    // swap rows i and j (j is data-dependent: a select over the candidates)
#pragma unroll
    for (int k = i + 1; k < N; ++k)
      if (j == k) {
        const double tw = W[i]; W[i] = W[k]; W[k] = tw;
#pragma unroll
        for (int e = 0; e < M; ++e) { const double x = U[i][e]; U[i][e] = U[k][e]; U[k][e] = x; }
        if (kV)
#pragma unroll
          for (int e = 0; e < N; ++e) { const double x = Vt[i][e]; Vt[i][e] = Vt[k][e]; Vt[k][e] = x; }
      }
  }
  uint64_t rng = 0x12345678ull;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double sd = W[i];
    for (int ii = 0; ii < 100 && sd <= kDblMin; ++ii) {
      const double val0 = 1.0 / M;
#pragma unroll
      for (int k = 0; k < M; ++k) U[i][k] = (cv_rng_next(rng) & 256) != 0 ? val0 : -val0;
      for (int it2 = 0; it2 < 2; ++it2)
#pragma unroll
        for (int j = 0; j < i; ++j) {
          sd = 0.0;
#pragma unroll
          for (int k = 0; k < M; ++k) sd += U[i][k] * U[j][k];
          double asum = 0.0;
#pragma unroll
          for (int k = 0; k < M; ++k) {
            const double t = U[i][k] - sd * U[j][k];
            U[i][k] = t;
            asum += fabs(t);
          }
          asum = asum > eps * 100 ? 1.0 / asum : 0.0;
#pragma unroll
          for (int k = 0; k < M; ++k) U[i][k] *= asum;
        }
      sd = 0.0;
#pragma unroll
      for (int k = 0; k < M; ++k) sd += U[i][k] * U[i][k];
      sd = sqrt(sd);
    }
    const double sc = sd > kDblMin ? 1.0 / sd : 0.0;
#pragma unroll
    for (int k = 0; k < M; ++k) U[i][k] *= sc;
    w[i] = W[i];
  }
}

// cv::SVD of A itself (A is copied transposed into U first).
template <int M, int N>
__host__ __device__ void cv_svd(const double (&A)[M][N], double (&U)[N][M], double (&w)[N], double (&Vt)[N][N],
                                double* lds = nullptr) {
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int k = 0; k < M; ++k) U[i][k] = A[k][i];
  cv_svd_at<M, N, true>(U, w, Vt, lds);
}

// cv::solve(A, b, x, DECOMP_SVD) = SVBkSb: x = sum over w_i > 2 DBL_EPSILON
// sum(w) of (u_i . b / w_i) v_i, in descending-w order.
template <int M, int N>
__host__ __device__ void cv_lstsq(const double (&A)[M][N], const double (&b)[M], double (&x)[N],
                                  double* lds = nullptr) {
  double U[N][M], w[N], Vt[N][N];
  cv_svd<M, N>(A, U, w, Vt, lds);
  double thr = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) thr += w[i];
  thr *= kDblEps * 2;
#pragma unroll
  for (int j = 0; j < N; ++j) x[j] = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double wi = w[i];
    if (fabs(wi) <= thr) continue;
    wi = 1.0 / wi;
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < M; ++j) s += U[i][j] * b[j];
    s *= wi;
#pragma unroll
    for (int j = 0; j < N; ++j) x[j] = x[j] + s * Vt[i][j];
  }
}

// epnp::qr_solve (Householder, Lepetit's code) for the 6 x 4 Gauss-Newton
// system; false when A is singular (the caller's betas stay unchanged).
__host__ __device__ bool qr_solve(double (&A)[6][4], double (&b)[6], double (&x)[4]) {
  double A1[4], A2[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    double eta = fabs(A[k][k]);
#pragma unroll
    for (int i = k + 1; i < 6; ++i) {
      const double elt = fabs(A[i][k]);
      if (eta < elt) eta = elt;
    }
    if (eta == 0) return false;
    const double inv_eta = 1. / eta;
    double sum1 = 0.0;
#pragma unroll
    for (int i = k; i < 6; ++i) { A[i][k] *= inv_eta; sum1 += A[i][k] * A[i][k]; }
    double sigma = sqrt(sum1);
    if (A[k][k] < 0) sigma = -sigma;
    A[k][k] += sigma;
    A1[k] = sigma * A[k][k];
    A2[k] = -eta * sigma;
#pragma unroll
    for (int j = k + 1; j < 4; ++j) {
      double sum = 0.0;
#pragma unroll
      for (int i = k; i < 6; ++i) sum += A[i][k] * A[i][j];
      const double tau = sum / A1[k];
#pragma unroll
      for (int i = k; i < 6; ++i) A[i][j] -= tau * A[i][k];
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double tau = 0.0;
#pragma unroll
    for (int i = j; i < 6; ++i) tau += A[i][j] * b[i];
    tau /= A1[j];
#pragma unroll
    for (int i = j; i < 6; ++i) b[i] -= tau * A[i][j];
  }
  x[3] = b[3] / A2[3];
#pragma unroll
  for (int i = 2; i >= 0; --i) {
    double sum = 0.0;
#pragma unroll
    for (int j = i + 1; j < 4; ++j) sum += A[i][j] * x[j];
    x[i] = (b[i] - sum) / A2[i];
  }
  return true;
}

}  // namespace
}  // namespace sfm
