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
template <int M, int N, bool kV>
__host__ __device__ void cv_svd_at(double (&U)[N][M], double (&w)[N], double (&Vt)[N][N]) {
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
__host__ __device__ void cv_svd(const double (&A)[M][N], double (&U)[N][M], double (&w)[N], double (&Vt)[N][N]) {
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int k = 0; k < M; ++k) U[i][k] = A[k][i];
  cv_svd_at<M, N, true>(U, w, Vt);
}

// cv::solve(A, b, x, DECOMP_SVD) = SVBkSb: x = sum over w_i > 2 DBL_EPSILON
// sum(w) of (u_i . b / w_i) v_i, in descending-w order.
template <int M, int N>
__host__ __device__ void cv_lstsq(const double (&A)[M][N], const double (&b)[M], double (&x)[N]) {
  double U[N][M], w[N], Vt[N][N];
  cv_svd<M, N>(A, U, w, Vt);
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
