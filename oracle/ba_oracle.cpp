// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called
// from the product (sfm_amd/).  Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load liboracle.so, and only as the checker
// or the timed CPU baseline.
//
// What this is: a C++ restatement of the reference's bundle
// adjustment hot path, CTracker::bundleAdjustmentStructAndPose
// (/root/reference/CTracker.cpp:670-702), including the third-party solver it
// calls.  The reference cannot be built in this pipeline (OpenCV, Eigen,
// Ceres and BRISK are absent: SURVEY.md §8c), so the arithmetic of
// Ceres Solver (~1.12, README.md:30 says "3.12.0", which is not a release)
// is restated from its published algorithm:
//
//   * BAStructAndPoseFunctor::operator() (CTracker.cpp:585-604) evaluated with
//     forward-mode dual numbers that mirror ceres::Jet<double,9>
//     (AutoDiffCostFunction<F,2,3,3,3>, CTracker.h:108-110);
//   * ceres::AngleAxisRotatePoint with its theta^2 > DBL_EPSILON branch
//     (called at CTracker.cpp:588);
//   * Problem: one residual block per observation over (R[c], t[c], X[i]),
//     no loss, no constant blocks (CTracker.cpp:676-696); parameter identity
//     is the point index (the reference's double* address);
//   * Solver options (CTracker.cpp:571-577): DENSE_SCHUR, every other option
//     a Ceres default: LM trust region, Jacobi scaling, 50 iterations,
//     function/gradient/parameter tolerance 1e-6/1e-10/1e-8, radius 1e4
//     (max 1e16, min 1e-32), LM diagonal in [1e-6, 1e32], min relative
//     decrease 1e-3, 5 consecutive invalid steps, monotonic steps;
//   * SchurEliminator<2,3,3> (point blocks eliminated, f-blocks R_c and t_c
//     of size 3), dense LLT of the reduced camera matrix, back substitution.
//   * Modes (CTracker.h:67, CTracker.cpp:679-694): 0 STRUCT_ONLY
//     (BAStructFunctor, :638-668), 1 POSE_ONLY (BAPoseFunctor, :607-636),
//     2 STRUCT_AND_POSE; any other value adds no residual blocks.
//
// Threads (oracle_set_threads, default 1 = Ceres' default num_threads, the
// reference's setting): the per-observation / per-point / per-row work runs
// in OpenMP loops, but every sum keeps the serial order (partitions own
// whole output rows; reductions are serial passes over per-item results),
// so any thread count gives bitwise the 1-thread result.  Only the timed
// all-cores CPU figure of bench.py uses more than one.
//
// PARITY UNPINNED: the reference has no tests, fixtures or golden data for
// this path and cannot be executed here, so this
// restatement is checked only against independent restatements
// (torch fp64 autograd for r/J, a numpy LM for the step sequence; see
// tests/golden/make_golden.py), never against reference outputs.
// ============================================================================
#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

namespace oracle {

static int g_threads = 1;
// Summation orders (tests only, oracle_set_order; a bit mask, 0 = Ceres'):
// bit 1: the reduced camera matrix's diagonal blocks in the device solver's
// association (U_c = sum F^T F first, then + D^2, then minus the outer
// products) instead of Ceres' running sum per block, point by point;
// bit 2: the model cost change summed over the observations in reverse.
// The same arithmetic in other valid orders, used to show which LM
// decisions of a near-singular problem rounding decides.
static int g_order = 0;

// ---------------------------------------------------------------------------
// Jet<double, N>: restates the arithmetic of ceres/jet.h (value part `a`,
// infinitesimal part `v`).  Only the operations the functor uses.
// ---------------------------------------------------------------------------
template <int N>
struct Jet {
  double a;
  double v[N];
  Jet() : a(0) { for (int i = 0; i < N; ++i) v[i] = 0; }
  explicit Jet(double x) : a(x) { for (int i = 0; i < N; ++i) v[i] = 0; }
  Jet(double x, int k) : a(x) { for (int i = 0; i < N; ++i) v[i] = 0; v[k] = 1.0; }
};
template <int N> inline Jet<N> operator+(const Jet<N>& f, const Jet<N>& g) {
  Jet<N> r; r.a = f.a + g.a; for (int i = 0; i < N; ++i) r.v[i] = f.v[i] + g.v[i]; return r; }
template <int N> inline Jet<N> operator-(const Jet<N>& f, const Jet<N>& g) {
  Jet<N> r; r.a = f.a - g.a; for (int i = 0; i < N; ++i) r.v[i] = f.v[i] - g.v[i]; return r; }
template <int N> inline Jet<N> operator-(const Jet<N>& f) {
  Jet<N> r; r.a = -f.a; for (int i = 0; i < N; ++i) r.v[i] = -f.v[i]; return r; }
template <int N> inline Jet<N> operator*(const Jet<N>& f, const Jet<N>& g) {
  Jet<N> r; r.a = f.a * g.a; for (int i = 0; i < N; ++i) r.v[i] = f.a * g.v[i] + f.v[i] * g.a; return r; }
template <int N> inline Jet<N> operator/(const Jet<N>& f, const Jet<N>& g) {
  // ceres: g_a_inverse = 1/g.a; f_a_by_g_a = f.a * g_a_inverse;
  //        Jet(f.a * g_a_inverse, (f.v - f_a_by_g_a * g.v) * g_a_inverse)
  const double gi = 1.0 / g.a, fg = f.a * gi;
  Jet<N> r; r.a = f.a * gi; for (int i = 0; i < N; ++i) r.v[i] = (f.v[i] - fg * g.v[i]) * gi; return r; }
template <int N> inline Jet<N> operator*(double s, const Jet<N>& g) {
  Jet<N> r; r.a = s * g.a; for (int i = 0; i < N; ++i) r.v[i] = s * g.v[i]; return r; }
template <int N> inline Jet<N> operator/(double s, const Jet<N>& g) {
  // ceres: minus_s_g_a_inverse2 = -s / (g.a * g.a); Jet(s / g.a, g.v * minus_s_g_a_inverse2)
  const double m = -s / (g.a * g.a);
  Jet<N> r; r.a = s / g.a; for (int i = 0; i < N; ++i) r.v[i] = g.v[i] * m; return r; }
template <int N> inline Jet<N> sqrt(const Jet<N>& f) {
  const double t = std::sqrt(f.a), tai = 1.0 / (2.0 * t);
  Jet<N> r; r.a = t; for (int i = 0; i < N; ++i) r.v[i] = f.v[i] * tai; return r; }
template <int N> inline Jet<N> cos(const Jet<N>& f) {
  const double s = -std::sin(f.a);
  Jet<N> r; r.a = std::cos(f.a); for (int i = 0; i < N; ++i) r.v[i] = s * f.v[i]; return r; }
template <int N> inline Jet<N> sin(const Jet<N>& f) {
  const double c = std::cos(f.a);
  Jet<N> r; r.a = std::sin(f.a); for (int i = 0; i < N; ++i) r.v[i] = c * f.v[i]; return r; }
template <int N> inline bool operator>(const Jet<N>& f, const Jet<N>& g) { return f.a > g.a; }

inline double sqrt(double x) { return std::sqrt(x); }
inline double cos(double x) { return std::cos(x); }
inline double sin(double x) { return std::sin(x); }

template <typename T> inline T make_const(double x) { return T(x); }

// ceres::AngleAxisRotatePoint (rotation.h), restated.
template <typename T>
inline void AngleAxisRotatePoint(const T aa[3], const T pt[3], T out[3]) {
  const T theta2 = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
  if (theta2 > make_const<T>(std::numeric_limits<double>::epsilon())) {
    const T theta = sqrt(theta2);
    const T costheta = cos(theta);
    const T sintheta = sin(theta);
    const T theta_inverse = 1.0 / theta;
    const T w[3] = {aa[0] * theta_inverse, aa[1] * theta_inverse, aa[2] * theta_inverse};
    const T w_cross_pt[3] = {w[1] * pt[2] - w[2] * pt[1], w[2] * pt[0] - w[0] * pt[2],
                             w[0] * pt[1] - w[1] * pt[0]};
    const T tmp = (w[0] * pt[0] + w[1] * pt[1] + w[2] * pt[2]) * (make_const<T>(1.0) - costheta);
    out[0] = pt[0] * costheta + w_cross_pt[0] * sintheta + w[0] * tmp;
    out[1] = pt[1] * costheta + w_cross_pt[1] * sintheta + w[1] * tmp;
    out[2] = pt[2] * costheta + w_cross_pt[2] * sintheta + w[2] * tmp;
  } else {
    const T w_cross_pt[3] = {aa[1] * pt[2] - aa[2] * pt[1], aa[2] * pt[0] - aa[0] * pt[2],
                             aa[0] * pt[1] - aa[1] * pt[0]};
    out[0] = pt[0] + w_cross_pt[0];
    out[1] = pt[1] + w_cross_pt[1];
    out[2] = pt[2] + w_cross_pt[2];
  }
}

// BAStructAndPoseFunctor::operator() (CTracker.cpp:585-604).  k = Matx33d::val
// row-major: k0 fx, k1 skew, k2 cx, k4 fy, k5 cy.
template <typename T>
inline void Functor(const T R[3], const T t[3], const T X[3], const double* k, double u, double v, T res[2]) {
  T p[3];
  AngleAxisRotatePoint(R, X, p);
  p[0] = p[0] + t[0]; p[1] = p[1] + t[1]; p[2] = p[2] + t[2];
  const T xp = p[0] / p[2];
  const T yp = p[1] / p[2];
  const T px = make_const<T>(k[0]) * xp + make_const<T>(k[1]) * yp + make_const<T>(k[2]);
  const T py = make_const<T>(k[4]) * yp + make_const<T>(k[5]);
  res[0] = px - make_const<T>(u);
  res[1] = py - make_const<T>(v);
}

// One observation: residual (2) and Jacobian (2 x 9, columns dR | dt | dX).
inline void EvalJet(const double* R, const double* t, const double* X, const double* k, double u, double v,
                    double res[2], double J[18]) {
  typedef Jet<9> J9;
  J9 Rj[3], tj[3], Xj[3], r[2];
  for (int i = 0; i < 3; ++i) { Rj[i] = J9(R[i], i); tj[i] = J9(t[i], 3 + i); Xj[i] = J9(X[i], 6 + i); }
  Functor(Rj, tj, Xj, k, u, v, r);
  res[0] = r[0].a; res[1] = r[1].a;
  for (int i = 0; i < 9; ++i) { J[i] = r[0].v[i]; J[9 + i] = r[1].v[i]; }
}
inline void EvalPlain(const double* R, const double* t, const double* X, const double* k, double u, double v,
                      double res[2]) {
  Functor<double>(R, t, X, k, u, v, res);
}

// ---------------------------------------------------------------------------
// Problem / solver state
// ---------------------------------------------------------------------------
struct Options {
  int32_t max_num_iterations;
  int32_t max_num_consecutive_invalid_steps;
  int32_t jacobi_scaling;
  int32_t pad_;
  double function_tolerance, gradient_tolerance, parameter_tolerance;
  double initial_trust_region_radius, max_trust_region_radius, min_trust_region_radius;
  double min_lm_diagonal, max_lm_diagonal, min_relative_decrease;
};

struct Summary {
  int32_t termination_type;  // 0 CONVERGENCE, 1 NO_CONVERGENCE, 2 FAILURE
  int32_t num_iterations;    // LM iterations performed (iteration 0 not counted)
  int32_t num_successful_steps, num_unsuccessful_steps, num_invalid_steps;
  int32_t num_residual_evaluations, num_jacobian_evaluations, num_linear_solves;
  double initial_cost, final_cost;
  double wall_time_s, jacobian_time_s, linear_solver_time_s, residual_time_s;
};

struct Iteration {
  int32_t iteration, step_is_valid, step_is_successful, pad_;
  double cost, cost_change, gradient_max_norm, step_norm, relative_decrease, trust_region_radius;
};

// Dense symmetric positive definite factorisation A = L L^T on the lower
// triangle of a row-major n x n matrix (Eigen's LLT<Upper> computes the same
// factor, transposed).  Blocked right-looking, nb = 64.  Returns false on a
// non-positive or non-finite pivot (Eigen: `x <= 0` -> failure; a NaN pivot
// leads to a non-finite step, which Ceres also treats as a linear solver
// failure).
static bool Cholesky(double* A, int n) {
  const int nb = 64;
  for (int k0 = 0; k0 < n; k0 += nb) {
    const int k1 = std::min(n, k0 + nb);
    // factor diagonal block (left-looking within the block)
    for (int j = k0; j < k1; ++j) {
      double* Aj = A + size_t(j) * n;
      double d = Aj[j];
      for (int l = k0; l < j; ++l) d -= Aj[l] * Aj[l];
      if (!(d > 0.0) || !std::isfinite(d)) return false;
      d = std::sqrt(d);
      Aj[j] = d;
      const double inv = 1.0 / d;
      for (int i = j + 1; i < k1; ++i) {
        double* Ai = A + size_t(i) * n;
        double s = Ai[j];
        for (int l = k0; l < j; ++l) s -= Ai[l] * Aj[l];
        Ai[j] = s * inv;
      }
    }
    // panel: rows below, columns k0..k1 : solve X L_kk^T = A_ik
#pragma omp parallel for num_threads(g_threads) schedule(static) if (g_threads > 1 && n - k1 > 256)
    for (int i = k1; i < n; ++i) {
      double* Ai = A + size_t(i) * n;
      for (int j = k0; j < k1; ++j) {
        const double* Aj = A + size_t(j) * n;
        double s = Ai[j];
        for (int l = k0; l < j; ++l) s -= Ai[l] * Aj[l];
        Ai[j] = s / Aj[j];
      }
    }
    // trailing update A_ij -= L_ik L_jk^T (i >= j >= k1), blocked for cache
    const int w = k1 - k0;
#pragma omp parallel for num_threads(g_threads) schedule(dynamic, 1) if (g_threads > 1 && n - k1 > 256)
    for (int ib = k1; ib < n; ib += nb) {
      const int ie = std::min(n, ib + nb);
      for (int jb = k1; jb <= ib; jb += nb) {
        const int je = std::min(n, jb + nb);
        for (int i = ib; i < ie; ++i) {
          double* Ai = A + size_t(i) * n;
          const double* Lik = Ai + k0;
          const int jend = std::min(je, i + 1);
          for (int j = jb; j < jend; ++j) {
            const double* Ljk = A + size_t(j) * n + k0;
            double s = 0.0;
            for (int l = 0; l < w; ++l) s += Lik[l] * Ljk[l];
            Ai[j] -= s;
          }
        }
      }
    }
  }
  return true;
}

// Solve L L^T x = b in place (row-major lower factor).
static void CholSolve(const double* L, int n, double* b) {
  for (int i = 0; i < n; ++i) {
    const double* Li = L + size_t(i) * n;
    double s = b[i];
    for (int l = 0; l < i; ++l) s -= Li[l] * b[l];
    b[i] = s / Li[i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
    for (int l = i + 1; l < n; ++l) s -= L[size_t(l) * n + i] * b[l];
    b[i] = s / L[size_t(i) * n + i];
  }
}

// 3x3 symmetric PD inverse through LLT (Eigen's selfadjointView<Upper>().llt()
// .solve(Identity)).  Returns false if not PD.
static bool Llt3(const double A[9], double L[9]) {
  std::memset(L, 0, 9 * sizeof(double));
  for (int j = 0; j < 3; ++j) {
    double d = A[3 * j + j];
    for (int l = 0; l < j; ++l) d -= L[3 * j + l] * L[3 * j + l];
    if (!(d > 0.0)) return false;
    L[3 * j + j] = std::sqrt(d);
    for (int i = j + 1; i < 3; ++i) {
      double s = A[3 * i + j];
      for (int l = 0; l < j; ++l) s -= L[3 * i + l] * L[3 * j + l];
      L[3 * i + j] = s / L[3 * j + j];
    }
  }
  return true;
}
static void Llt3Solve(const double L[9], double b[3]) {
  for (int i = 0; i < 3; ++i) { double s = b[i]; for (int l = 0; l < i; ++l) s -= L[3 * i + l] * b[l]; b[i] = s / L[3 * i + i]; }
  for (int i = 2; i >= 0; --i) { double s = b[i]; for (int l = i + 1; l < 3; ++l) s -= L[3 * l + i] * b[l]; b[i] = s / L[3 * i + i]; }
}

// The whole LM problem.  Parameter vector layout (one block per Ceres
// parameter block): points [P][3] first (the eliminated e-blocks), then
// cameras [C][6] = (R_c, t_c).
struct Problem {
  int mode;  // 0 struct only, 1 pose only, 2 struct and pose
  int64_t n_obs;
  int n_cams, n_pts;
  const double* uv;
  const int32_t* cam;
  const int32_t* pt;
  const double* K9;
  // variable layout
  bool pts_var, cams_var;
  int np;   // number of variable point params (3P or 0)
  int nc;   // number of variable camera params (6C or 0)
  int n;    // np + nc
  // point-major observation order (stable) — the Schur chunks
  std::vector<int64_t> order;
  std::vector<int64_t> pt_off;
  // camera usage (cameras with no residual are not parameter blocks in Ceres)
  std::vector<int> cam_used, pt_used;
};

struct State {
  std::vector<double> x;      // [n]
};

static inline void GetParams(const Problem& pb, const double* x, const double* rot0, const double* t0,
                             const double* X0, int c, int p, const double*& R, const double*& t, const double*& X) {
  if (pb.cams_var) { R = x + pb.np + 6 * size_t(c); t = R + 3; } else { R = rot0 + 3 * size_t(c); t = t0 + 3 * size_t(c); }
  if (pb.pts_var) X = x + 3 * size_t(p); else X = X0 + 3 * size_t(p);
}

struct Evaluation {
  double cost;
  std::vector<double> r;     // [2N] in point-major order
  std::vector<double> J;     // [N][18] in point-major order (dR dt dX)
  std::vector<double> grad;  // [n]
};

}  // namespace oracle

using namespace oracle;

extern "C" {

// Residuals and Jacobians of every observation in caller order:
// res [N][2], jac [N][2][9] (row-major; columns dR0..2 dt0..2 dX0..2) or NULL.
int oracle_ba_residuals_jacobians(int64_t n_obs, const double* obs_uv, const int32_t* cam_idx,
                                  const int32_t* pt_idx, const double* K9, const double* rot,
                                  const double* t, const double* X, double* res, double* jac) {
  for (int64_t i = 0; i < n_obs; ++i) {
    const int c = cam_idx[i], p = pt_idx[i];
    if (jac)
      EvalJet(rot + 3 * size_t(c), t + 3 * size_t(c), X + 3 * size_t(p), K9 + 9 * size_t(c), obs_uv[2 * i],
              obs_uv[2 * i + 1], res + 2 * i, jac + 18 * i);
    else
      EvalPlain(rot + 3 * size_t(c), t + 3 * size_t(c), X + 3 * size_t(p), K9 + 9 * size_t(c), obs_uv[2 * i],
                obs_uv[2 * i + 1], res + 2 * i);
  }
  return 0;
}

void oracle_default_options(Options* o) {
  o->max_num_iterations = 50;
  o->max_num_consecutive_invalid_steps = 5;
  o->jacobi_scaling = 1;
  o->pad_ = 0;
  o->function_tolerance = 1e-6;
  o->gradient_tolerance = 1e-10;
  o->parameter_tolerance = 1e-8;
  o->initial_trust_region_radius = 1e4;
  o->max_trust_region_radius = 1e16;
  o->min_trust_region_radius = 1e-32;
  o->min_lm_diagonal = 1e-6;
  o->max_lm_diagonal = 1e32;
  o->min_relative_decrease = 1e-3;
}

// The restated solve.  rot/t [C][3], X [P][3] are updated in place (as the
// reference's double* parameter blocks are).  trace may be NULL.
int oracle_ba_solve(const Options* opts, int mode, int64_t n_obs, const double* obs_uv,
                    const int32_t* cam_idx, const int32_t* pt_idx, int32_t n_cams, const double* K9,
                    double* rot, double* t, int32_t n_pts, double* X, Summary* summary, Iteration* trace,
                    int32_t trace_cap, int32_t* trace_len) {
  const auto t_start = std::chrono::steady_clock::now();
  auto now_s = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count(); };
  Summary sm;
  std::memset(&sm, 0, sizeof(sm));
  if (trace_len) *trace_len = 0;
  int tl = 0;
  auto push = [&](const Iteration& it) { if (trace && tl < trace_cap) trace[tl] = it; ++tl; if (trace_len) *trace_len = std::min(tl, trace_cap); };

  for (int64_t i = 0; i < n_obs; ++i)
    if (cam_idx[i] < 0 || cam_idx[i] >= n_cams || pt_idx[i] < 0 || pt_idx[i] >= n_pts) return -22;
  // Ceres 1.12 Solver::Options::IsValid (CommonOptionsAreValid +
  // TrustRegionOptionsAreValid): ceres::Solve refuses to run otherwise
  {
    const Options& o = *opts;
    const bool ok = o.max_num_iterations >= 0 && o.function_tolerance >= 0 && o.gradient_tolerance >= 0 &&
                    o.parameter_tolerance >= 0 && o.initial_trust_region_radius > 0 &&
                    o.min_trust_region_radius > 0 && o.max_trust_region_radius > 0 &&
                    o.min_trust_region_radius <= o.max_trust_region_radius &&
                    o.min_trust_region_radius <= o.initial_trust_region_radius &&
                    o.initial_trust_region_radius <= o.max_trust_region_radius && o.min_relative_decrease >= 0 &&
                    o.min_lm_diagonal >= 0 && o.max_lm_diagonal >= 0 && o.min_lm_diagonal <= o.max_lm_diagonal &&
                    o.max_num_consecutive_invalid_steps >= 0;
    if (!ok) return -22;
  }

  Problem pb;
  pb.mode = mode; pb.n_obs = (mode >= 0 && mode <= 2) ? n_obs : 0;
  pb.n_cams = n_cams; pb.n_pts = n_pts; pb.uv = obs_uv; pb.cam = cam_idx; pb.pt = pt_idx; pb.K9 = K9;
  pb.pts_var = (mode == 0 || mode == 2);
  pb.cams_var = (mode == 1 || mode == 2);
  pb.np = pb.pts_var ? 3 * n_pts : 0;
  pb.nc = pb.cams_var ? 6 * n_cams : 0;
  pb.n = pb.np + pb.nc;
  const int64_t N = pb.n_obs;
  if (N == 0) {
    // Ceres on a problem without residual blocks: nothing to do.
    sm.termination_type = 0;
    if (summary) *summary = sm;
    return 0;
  }
  // point-major order (Ceres' LexicographicallyOrderResidualBlocks groups the
  // residual blocks of each e-block, keeping their original order)
  pb.pt_off.assign(size_t(n_pts) + 1, 0);
  for (int64_t i = 0; i < N; ++i) pb.pt_off[pt_idx[i] + 1]++;
  for (int p = 0; p < n_pts; ++p) pb.pt_off[p + 1] += pb.pt_off[p];
  pb.order.resize(N);
  {
    std::vector<int64_t> fill(pb.pt_off.begin(), pb.pt_off.end() - 1);
    for (int64_t i = 0; i < N; ++i) pb.order[fill[pt_idx[i]]++] = i;
  }
  pb.cam_used.assign(n_cams, 0);
  pb.pt_used.assign(n_pts, 0);
  for (int64_t i = 0; i < N; ++i) { pb.cam_used[cam_idx[i]] = 1; pb.pt_used[pt_idx[i]] = 1; }

  const int n = pb.n;
  std::vector<double> x(n), x_new(n);
  if (pb.pts_var) std::memcpy(x.data(), X, sizeof(double) * 3 * size_t(n_pts));
  if (pb.cams_var)
    for (int c = 0; c < n_cams; ++c) {
      std::memcpy(&x[pb.np + 6 * size_t(c)], rot + 3 * size_t(c), 3 * sizeof(double));
      std::memcpy(&x[pb.np + 6 * size_t(c) + 3], t + 3 * size_t(c), 3 * sizeof(double));
    }
  // Parameter blocks that appear in no residual are not part of the Ceres
  // problem (they were never added); mask them out of norms and steps.
  std::vector<char> active(n, 0);
  if (pb.pts_var) for (int p = 0; p < n_pts; ++p) if (pb.pt_used[p]) for (int k = 0; k < 3; ++k) active[3 * p + k] = 1;
  if (pb.cams_var) for (int c = 0; c < n_cams; ++c) if (pb.cam_used[c]) for (int k = 0; k < 6; ++k) active[pb.np + 6 * c + k] = 1;
  // Immutable copies for constant blocks.
  std::vector<double> rot0(rot, rot + 3 * size_t(n_cams)), t0(t, t + 3 * size_t(n_cams)), X0(X, X + 3 * size_t(n_pts));

  auto norm_active = [&](const std::vector<double>& v) {
    double s = 0; for (int i = 0; i < n; ++i) if (active[i]) s += v[i] * v[i]; return std::sqrt(s); };

  // ---- evaluation -------------------------------------------------------
  std::vector<double> r(2 * N), J(18 * N), grad(n), rtmp(2 * N);
  auto evaluate = [&](const std::vector<double>& xx, bool with_jac, double* cost_out,
                      std::vector<double>* rr) -> bool {
    // per-observation arithmetic (parallel when g_threads > 1), then the
    // cost / gradient sums in the serial observation order
    double* rb = rr ? rr->data() : rtmp.data();
#pragma omp parallel for num_threads(g_threads) schedule(static) if (g_threads > 1)
    for (int64_t q = 0; q < N; ++q) {
      const int64_t i = pb.order[q];
      const int c = cam_idx[i], p = pt_idx[i];
      const double *Rp, *tp, *Xp;
      GetParams(pb, xx.data(), rot0.data(), t0.data(), X0.data(), c, p, Rp, tp, Xp);
      if (with_jac)  // rows stored as [row][dR dt dX]
        EvalJet(Rp, tp, Xp, K9 + 9 * size_t(c), obs_uv[2 * i], obs_uv[2 * i + 1], rb + 2 * q, &J[18 * q]);
      else
        EvalPlain(Rp, tp, Xp, K9 + 9 * size_t(c), obs_uv[2 * i], obs_uv[2 * i + 1], rb + 2 * q);
    }
    double cost = 0.0;
    if (with_jac) std::fill(grad.begin(), grad.end(), 0.0);
    for (int64_t q = 0; q < N; ++q) {
      const double res[2] = {rb[2 * q], rb[2 * q + 1]};
      if (with_jac) {
        const int64_t i = pb.order[q];
        const int c = cam_idx[i], p = pt_idx[i];
        const double* Jrow = &J[18 * q];
        if (pb.cams_var)
          for (int k = 0; k < 6; ++k) grad[pb.np + 6 * c + k] += Jrow[k] * res[0] + Jrow[9 + k] * res[1];
        if (pb.pts_var)
          for (int k = 0; k < 3; ++k) grad[3 * p + k] += Jrow[6 + k] * res[0] + Jrow[15 + k] * res[1];
      }
      cost += 0.5 * (res[0] * res[0] + res[1] * res[1]);
    }
    *cost_out = cost;
    return std::isfinite(cost);
  };

  // column access helpers: column index in x for (obs q, local col k in 0..8)
  auto col_of = [&](int64_t q, int k) -> int {
    const int64_t i = pb.order[q];
    if (k < 6) return pb.cams_var ? pb.np + 6 * cam_idx[i] + k : -1;
    return pb.pts_var ? 3 * pt_idx[i] + (k - 6) : -1;
  };

  std::vector<double> scale(n, 1.0), diag(n, 0.0);
  double cost = 0.0;
  double t0s = now_s();
  if (!evaluate(x, true, &cost, &r)) {
    sm.termination_type = 2;
    if (summary) *summary = sm;
    return -5;
  }
  sm.jacobian_time_s += now_s() - t0s;
  sm.num_jacobian_evaluations++;
  sm.num_residual_evaluations++;
  sm.initial_cost = cost;
  auto grad_max = [&]() { double m = 0; for (int i = 0; i < n; ++i) if (active[i]) m = std::max(m, std::fabs(grad[i])); return m; };
  auto col_sq_norms = [&](std::vector<double>& out, bool scaled) {
    std::fill(out.begin(), out.end(), 0.0);
    for (int64_t q = 0; q < N; ++q)
      for (int k = 0; k < 9; ++k) {
        const int col = col_of(q, k);
        if (col < 0) continue;
        const double a = J[18 * q + k], b = J[18 * q + 9 + k];
        double s = a * a + b * b;
        out[col] += s;
      }
    if (scaled) for (int i = 0; i < n; ++i) out[i] *= scale[i] * scale[i];
  };
  if (opts->jacobi_scaling) {
    std::vector<double> cn(n);
    col_sq_norms(cn, false);
    for (int i = 0; i < n; ++i) scale[i] = 1.0 / (1.0 + std::sqrt(cn[i]));
  }
  // J is kept unscaled; scaled entries are J * scale[col] on use.
  auto Js = [&](int64_t q, int row, int k) -> double {
    const int col = col_of(q, k);
    return col < 0 ? 0.0 : J[18 * q + 9 * row + k] * scale[col];
  };

  Iteration it0;
  std::memset(&it0, 0, sizeof(it0));
  it0.iteration = 0; it0.cost = cost; it0.gradient_max_norm = grad_max();
  it0.trust_region_radius = opts->initial_trust_region_radius;
  it0.step_is_valid = 1; it0.step_is_successful = 1;  // ceres records iteration 0 as successful
  push(it0);
  if (it0.gradient_max_norm <= opts->gradient_tolerance) {
    sm.termination_type = 0;
    sm.final_cost = cost;
    goto write_back;
  }

  {
    double radius = opts->initial_trust_region_radius;
    double decrease_factor = 2.0;
    bool reuse_diagonal = false;
    int num_consecutive_invalid = 0;
    double x_norm = norm_active(x);
    int iteration = 0;
    double last_grad_max = it0.gradient_max_norm;
    const int C = n_cams;
    // Schur sizes: f-blocks = cameras (6 params each as two 3-blocks)
    const int nf = pb.cams_var ? 6 * C : 0;
    std::vector<double> S, rhs, step(n), delta(n), lm_D(n), model_res(2 * N);

    while (true) {
      if (iteration >= opts->max_num_iterations) { sm.termination_type = 1; break; }
      ++iteration;
      Iteration itr;
      std::memset(&itr, 0, sizeof(itr));
      itr.iteration = iteration;

      // ---- LevenbergMarquardtStrategy::ComputeStep -------------------------
      if (!reuse_diagonal) {
        col_sq_norms(diag, true);
        for (int i = 0; i < n; ++i) diag[i] = std::min(std::max(diag[i], opts->min_lm_diagonal), opts->max_lm_diagonal);
      }
      for (int i = 0; i < n; ++i) lm_D[i] = std::sqrt(diag[i] / radius);
      reuse_diagonal = true;

      // ---- DENSE_SCHUR: solve (Js^T Js + D^2) y = Js^T r ---------------------
      const double tls = now_s();
      bool solve_ok = true;
      std::fill(step.begin(), step.end(), 0.0);
      if (pb.pts_var && pb.cams_var) {
        S.assign(size_t(nf) * nf, 0.0);
        rhs.assign(nf, 0.0);
        if (g_order & 1) {
          // U_c = sum_q F^T F (point order), then + D^2
          for (int p = 0; p < n_pts; ++p)
            for (int64_t q = pb.pt_off[p]; q < pb.pt_off[p + 1]; ++q) {
              const int c = cam_idx[pb.order[q]];
              double F[12];
              for (int row = 0; row < 2; ++row)
                for (int k = 0; k < 6; ++k) F[6 * row + k] = Js(q, row, k);
              for (int a = 0; a < 6; ++a)
                for (int bb = 0; bb < 6; ++bb)
                  S[size_t(6 * c + a) * nf + 6 * c + bb] += F[a] * F[bb] + F[6 + a] * F[6 + bb];
            }
        }
        for (int i = 0; i < nf; ++i) S[size_t(i) * nf + i] += lm_D[pb.np + i] * lm_D[pb.np + i];
        // Phase 1, per point (independent): ete = D_e^2 + sum E^T E,
        // g = sum E^T b, buffer_f = sum E^T F per distinct camera (slot order
        // = first appearance), inverse_ete.  Slots live at the point's
        // observation offsets.
        std::vector<double> ebuf(18 * size_t(N)), pinv(9 * size_t(n_pts)), pig(3 * size_t(n_pts));
        std::vector<int> fc(N), nslot(n_pts, 0);
        int any_bad = 0;
#pragma omp parallel for num_threads(g_threads) schedule(static) reduction(| : any_bad) if (g_threads > 1)
        for (int p = 0; p < n_pts; ++p) {
          const int64_t q0 = pb.pt_off[p], q1 = pb.pt_off[p + 1];
          if (q0 == q1) continue;
          double ete[9] = {0};
          for (int k = 0; k < 3; ++k) ete[4 * k] = lm_D[3 * p + k] * lm_D[3 * p + k];
          double g[3] = {0, 0, 0};
          int* fcams = &fc[q0];
          double* Ebuf = &ebuf[18 * size_t(q0)];
          int m = 0;
          for (int64_t q = q0; q < q1; ++q) {
            const int c = cam_idx[pb.order[q]];
            int slot = -1;
            for (int s2 = 0; s2 < m; ++s2) if (fcams[s2] == c) { slot = s2; break; }
            if (slot < 0) { slot = m++; fcams[slot] = c; std::fill(Ebuf + 18 * slot, Ebuf + 18 * slot + 18, 0.0); }
            double E[6], F[12];
            for (int row = 0; row < 2; ++row) {
              for (int k = 0; k < 3; ++k) E[3 * row + k] = Js(q, row, 6 + k);
              for (int k = 0; k < 6; ++k) F[6 * row + k] = Js(q, row, k);
            }
            const double b0 = r[2 * q], b1 = r[2 * q + 1];
            for (int a = 0; a < 3; ++a) {
              for (int bb = 0; bb < 3; ++bb) ete[3 * a + bb] += E[a] * E[bb] + E[3 + a] * E[3 + bb];
              g[a] += E[a] * b0 + E[3 + a] * b1;
              for (int k = 0; k < 6; ++k) Ebuf[18 * slot + 6 * a + k] += E[a] * F[k] + E[3 + a] * F[6 + k];
            }
          }
          nslot[p] = m;
          double L[9];
          if (!Llt3(ete, L)) { any_bad = 1; continue; }
          // inverse_ete = llt.solve(I)
          double* inv = &pinv[9 * size_t(p)];
          for (int col = 0; col < 3; ++col) {
            double e[3] = {0, 0, 0}; e[col] = 1.0;
            Llt3Solve(L, e);
            for (int a = 0; a < 3; ++a) inv[3 * a + col] = e[a];
          }
          for (int a = 0; a < 3; ++a)
            pig[3 * size_t(p) + a] = inv[3 * a] * g[0] + inv[3 * a + 1] * g[1] + inv[3 * a + 2] * g[2];
        }
        if (any_bad) solve_ok = false;
        // Phase 2, per camera row range (each S / rhs row has one owner; the
        // points are visited in order, so every entry sees the serial
        // sequence: F^T F, then UpdateRhs, then ChunkOuterProduct, point by
        // point).
        if (solve_ok) {
          const int T = std::max(1, std::min(g_threads, C));
#pragma omp parallel for num_threads(T) schedule(static, 1) if (T > 1)
          for (int th = 0; th < T; ++th) {
            const int clo = int(int64_t(C) * th / T), chi = int(int64_t(C) * (th + 1) / T);
            for (int p = 0; p < n_pts; ++p) {
              const int64_t q0 = pb.pt_off[p], q1 = pb.pt_off[p + 1];
              if (q0 == q1) continue;
              // F^T F into S (both 3-blocks of the camera and their coupling)
              for (int64_t q = q0; q < q1 && !(g_order & 1); ++q) {
                const int c = cam_idx[pb.order[q]];
                if (c < clo || c >= chi) continue;
                double F[12];
                for (int row = 0; row < 2; ++row)
                  for (int k = 0; k < 6; ++k) F[6 * row + k] = Js(q, row, k);
                const int base = 6 * c;
                for (int a = 0; a < 6; ++a)
                  for (int bb = 0; bb < 6; ++bb)
                    S[size_t(base + a) * nf + base + bb] += F[a] * F[bb] + F[6 + a] * F[6 + bb];
              }
              const double* inv = &pinv[9 * size_t(p)];
              const double* ig = &pig[3 * size_t(p)];
              // UpdateRhs: rhs_f += F^T (b - E * inverse_ete_g)
              for (int64_t q = q0; q < q1; ++q) {
                const int c = cam_idx[pb.order[q]];
                if (c < clo || c >= chi) continue;
                double sj[2];
                for (int row = 0; row < 2; ++row) {
                  sj[row] = r[2 * q + row];
                  for (int k = 0; k < 3; ++k) sj[row] -= Js(q, row, 6 + k) * ig[k];
                }
                for (int k = 0; k < 6; ++k) rhs[6 * c + k] += Js(q, 0, k) * sj[0] + Js(q, 1, k) * sj[1];
              }
              // ChunkOuterProduct: S(j,k) -= buffer_j^T inverse_ete buffer_k
              const int m = nslot[p];
              const int* fcams = &fc[q0];
              const double* Ebuf = &ebuf[18 * size_t(q0)];
              for (int j = 0; j < m; ++j) {
                const int cj = fcams[j];
                if (cj < clo || cj >= chi) continue;
                double bt_inv[18];  // (6x3) = buffer_j^T * inv
                for (int a = 0; a < 6; ++a)
                  for (int bb = 0; bb < 3; ++bb)
                    bt_inv[3 * a + bb] = Ebuf[18 * j + 0 * 6 + a] * inv[0 * 3 + bb] +
                                         Ebuf[18 * j + 1 * 6 + a] * inv[1 * 3 + bb] +
                                         Ebuf[18 * j + 2 * 6 + a] * inv[2 * 3 + bb];
                for (int k = 0; k < m; ++k) {
                  const int ck = fcams[k];
                  for (int a = 0; a < 6; ++a)
                    for (int bb = 0; bb < 6; ++bb) {
                      double s = bt_inv[3 * a] * Ebuf[18 * k + 0 * 6 + bb] + bt_inv[3 * a + 1] * Ebuf[18 * k + 1 * 6 + bb] +
                                 bt_inv[3 * a + 2] * Ebuf[18 * k + 2 * 6 + bb];
                      S[size_t(6 * cj + a) * nf + 6 * ck + bb] -= s;
                    }
                }
              }
            }
          }
        }
        if (solve_ok) {
          solve_ok = Cholesky(S.data(), nf);
          if (solve_ok) {
            std::vector<double> y(rhs);
            CholSolve(S.data(), nf, y.data());
            for (int i = 0; i < nf; ++i) step[pb.np + i] = y[i];
            // BackSubstitute: y_e = (E^T E + D_e^2)^-1 E^T (b - F y_f)
            int bs_bad = 0;
#pragma omp parallel for num_threads(g_threads) schedule(static) reduction(| : bs_bad) if (g_threads > 1)
            for (int p = 0; p < n_pts; ++p) {
              const int64_t q0 = pb.pt_off[p], q1 = pb.pt_off[p + 1];
              if (q0 == q1) continue;
              double ete[9] = {0};
              for (int k = 0; k < 3; ++k) ete[4 * k] = lm_D[3 * p + k] * lm_D[3 * p + k];
              double ye[3] = {0, 0, 0};
              for (int64_t q = q0; q < q1; ++q) {
                const int c = cam_idx[pb.order[q]];
                double sj[2];
                for (int row = 0; row < 2; ++row) {
                  sj[row] = r[2 * q + row];
                  for (int k = 0; k < 6; ++k) sj[row] -= Js(q, row, k) * y[6 * c + k];
                }
                for (int a = 0; a < 3; ++a) {
                  const double Ea0 = Js(q, 0, 6 + a), Ea1 = Js(q, 1, 6 + a);
                  ye[a] += Ea0 * sj[0] + Ea1 * sj[1];
                  for (int bb = 0; bb < 3; ++bb) ete[3 * a + bb] += Ea0 * Js(q, 0, 6 + bb) + Ea1 * Js(q, 1, 6 + bb);
                }
              }
              double L[9];
              if (!Llt3(ete, L)) { bs_bad = 1; continue; }
              Llt3Solve(L, ye);
              for (int k = 0; k < 3; ++k) step[3 * p + k] = ye[k];
            }
            if (bs_bad) solve_ok = false;
          }
        }
      } else {
        // Only one kind of parameter block: the normal matrix is block
        // diagonal (points: 3x3 per point; cameras: 6x6 per camera, R and t
        // coupled).  Ceres' DENSE_SCHUR on such a problem eliminates an
        // independent set of blocks and factors the rest densely; the
        // solution is the same block-diagonal solve.
        const int bs = pb.pts_var ? 3 : 6;
        const int nblk = pb.pts_var ? n_pts : n_cams;
        std::vector<double> H(size_t(nblk) * bs * bs, 0.0), b(n, 0.0);
        for (int64_t q = 0; q < N; ++q) {
          const int64_t i = pb.order[q];
          const int blk = pb.pts_var ? pt_idx[i] : cam_idx[i];
          const int k0 = pb.pts_var ? 6 : 0;
          for (int a = 0; a < bs; ++a) {
            const double ja0 = Js(q, 0, k0 + a), ja1 = Js(q, 1, k0 + a);
            b[bs * blk + a] += ja0 * r[2 * q] + ja1 * r[2 * q + 1];
            for (int bb = 0; bb < bs; ++bb)
              H[(size_t(blk) * bs + a) * bs + bb] += ja0 * Js(q, 0, k0 + bb) + ja1 * Js(q, 1, k0 + bb);
          }
        }
        for (int blk = 0; blk < nblk && solve_ok; ++blk) {
          double* Hb = &H[size_t(blk) * bs * bs];
          for (int a = 0; a < bs; ++a) Hb[a * bs + a] += lm_D[bs * blk + a] * lm_D[bs * blk + a];
          const bool used = pb.pts_var ? pb.pt_used[blk] : pb.cam_used[blk];
          if (!used) continue;
          if (!Cholesky(Hb, bs)) { solve_ok = false; break; }
          CholSolve(Hb, bs, &b[bs * blk]);
          for (int a = 0; a < bs; ++a) step[bs * blk + a] = b[bs * blk + a];
        }
      }
      sm.num_linear_solves++;
      sm.linear_solver_time_s += now_s() - tls;
      if (solve_ok) for (int i = 0; i < n; ++i) if (!std::isfinite(step[i])) { solve_ok = false; break; }
      if (solve_ok) for (int i = 0; i < n; ++i) step[i] = -step[i];

      // ---- model cost change ------------------------------------------------
      double model_cost_change = 0.0;
      itr.step_is_valid = 0;
      itr.step_is_successful = 0;
      if (solve_ok) {
        double mc = 0.0;
#pragma omp parallel for num_threads(g_threads) schedule(static) if (g_threads > 1)
        for (int64_t q = 0; q < N; ++q)
          for (int row = 0; row < 2; ++row) {
            double s = 0.0;
            for (int k = 0; k < 9; ++k) { const int col = col_of(q, k); if (col >= 0) s += Js(q, row, k) * step[col]; }
            model_res[2 * q + row] = s;
          }
        for (int64_t qq = 0; qq < N; ++qq) {
          const int64_t q = (g_order & 2) ? N - 1 - qq : qq;  // order bit 2: the other way round
          const double mr[2] = {model_res[2 * q], model_res[2 * q + 1]};
          mc += mr[0] * (r[2 * q] + mr[0] / 2.0) + mr[1] * (r[2 * q + 1] + mr[1] / 2.0);
        }
        model_cost_change = -mc;
        itr.step_is_valid = (model_cost_change >= 0.0) ? 1 : 0;
      }

      if (!itr.step_is_valid) {
        ++num_consecutive_invalid;
        sm.num_invalid_steps++;
        if (num_consecutive_invalid >= opts->max_num_consecutive_invalid_steps) {
          sm.termination_type = 2;
          itr.cost = cost; itr.gradient_max_norm = last_grad_max; itr.trust_region_radius = radius;
          push(itr);
          break;
        }
        itr.cost = cost;
        itr.cost_change = 0;
        itr.gradient_max_norm = last_grad_max;
        itr.step_norm = 0;
        itr.relative_decrease = 0;
      } else {
        num_consecutive_invalid = 0;
        for (int i = 0; i < n; ++i) { delta[i] = step[i] * scale[i]; x_new[i] = x[i] + delta[i]; }
        double new_cost = std::numeric_limits<double>::max();
        const double trs = now_s();
        if (!evaluate(x_new, false, &new_cost, nullptr)) new_cost = std::numeric_limits<double>::max();
        sm.residual_time_s += now_s() - trs;
        sm.num_residual_evaluations++;
        {
          double s = 0; for (int i = 0; i < n; ++i) if (active[i]) { double d = x[i] - x_new[i]; s += d * d; }
          itr.step_norm = std::sqrt(s);
        }
        const double step_size_tolerance = opts->parameter_tolerance * (x_norm + opts->parameter_tolerance);
        if (itr.step_norm <= step_size_tolerance) {
          sm.termination_type = 0;
          itr.cost = cost; itr.gradient_max_norm = last_grad_max; itr.trust_region_radius = radius;
          push(itr);
          break;
        }
        itr.cost_change = cost - new_cost;
        const double absolute_function_tolerance = opts->function_tolerance * cost;
        if (std::fabs(itr.cost_change) <= absolute_function_tolerance) {
          sm.termination_type = 0;
          itr.cost = cost; itr.gradient_max_norm = last_grad_max; itr.trust_region_radius = radius;
          push(itr);
          break;
        }
        itr.relative_decrease = itr.cost_change / model_cost_change;
        itr.step_is_successful = itr.relative_decrease > opts->min_relative_decrease;
      }

      if (itr.step_is_successful) {
        sm.num_successful_steps++;
        // StepAccepted
        radius = radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * itr.relative_decrease - 1.0, 3));
        radius = std::min(opts->max_trust_region_radius, radius);
        decrease_factor = 2.0;
        reuse_diagonal = false;
        x.swap(x_new);
        x_norm = norm_active(x);
        const double tj = now_s();
        if (!evaluate(x, true, &cost, &r)) { sm.termination_type = 2; break; }
        sm.jacobian_time_s += now_s() - tj;
        sm.num_jacobian_evaluations++;
        sm.num_residual_evaluations++;
        last_grad_max = grad_max();
        itr.gradient_max_norm = last_grad_max;
      } else {
        sm.num_unsuccessful_steps++;
        // StepRejected / StepIsInvalid
        radius = radius / decrease_factor;
        decrease_factor *= 2.0;
        reuse_diagonal = true;
        itr.gradient_max_norm = last_grad_max;
      }
      itr.cost = cost;
      itr.trust_region_radius = radius;
      push(itr);
      if (itr.step_is_successful) {
        if (itr.gradient_max_norm <= opts->gradient_tolerance) { sm.termination_type = 0; break; }
      } else {
        if (radius < opts->min_trust_region_radius) { sm.termination_type = 0; break; }
      }
    }
    sm.num_iterations = iteration;
    sm.final_cost = cost;
  }

write_back:
  if (pb.pts_var)
    for (int p = 0; p < n_pts; ++p) if (pb.pt_used[p]) std::memcpy(X + 3 * size_t(p), &x[3 * size_t(p)], 3 * sizeof(double));
  if (pb.cams_var)
    for (int c = 0; c < n_cams; ++c) if (pb.cam_used[c]) {
      std::memcpy(rot + 3 * size_t(c), &x[pb.np + 6 * size_t(c)], 3 * sizeof(double));
      std::memcpy(t + 3 * size_t(c), &x[pb.np + 6 * size_t(c) + 3], 3 * sizeof(double));
    }
  sm.wall_time_s = now_s();
  if (summary) *summary = sm;
  return 0;
}

int oracle_abi_version(void) { return 1; }

// Threads of the OpenMP loops of oracle_ba_solve (default 1; any value gives
// bitwise the same result).  Returns the previous value.
int oracle_set_threads(int threads) {
  const int prev = g_threads;
  g_threads = threads < 1 ? 1 : threads;
  return prev;
}

int oracle_set_order(int order) {
  const int prev = g_order;
  g_order = order;
  return prev;
}
}  // extern "C"

// ---------------------------------------------------------------------------
// Test helper for the landmark-sharding decomposition:
// the DENSE_SCHUR reduced camera system of a set of observations at given
// parameters, Jacobi scale and LM diagonal D (all explicit, so a shard can
// be assembled with the GLOBAL scale / D).  S [6C][6C] (full, row-major),
// rhs [6C].  The camera diagonal D_c^2 is added iff add_cam_diag.
// Also returns the unscaled squared column norms of the observations
// (colnorm_c [C][6], colnorm_p [P][3]) when those pointers are non-NULL.
extern "C" int oracle_ba_reduced_system(int64_t n_obs, const double* obs_uv, const int32_t* cam_idx,
                                        const int32_t* pt_idx, int32_t n_cams, const double* K9, const double* rot,
                                        const double* t, int32_t n_pts, const double* X, const double* scale_c,
                                        const double* scale_p, const double* D_c, const double* D_p,
                                        int32_t add_cam_diag, double* S, double* rhs, double* colnorm_c,
                                        double* colnorm_p) {
  const int C = n_cams, nf = 6 * C;
  std::vector<std::vector<int64_t>> by_pt(n_pts);
  for (int64_t i = 0; i < n_obs; ++i) by_pt[pt_idx[i]].push_back(i);
  std::memset(S, 0, sizeof(double) * size_t(nf) * nf);
  std::memset(rhs, 0, sizeof(double) * nf);
  if (colnorm_c) std::memset(colnorm_c, 0, sizeof(double) * 6 * size_t(C));
  if (colnorm_p) std::memset(colnorm_p, 0, sizeof(double) * 3 * size_t(n_pts));
  if (add_cam_diag)
    for (int i = 0; i < nf; ++i) S[size_t(i) * nf + i] += D_c[i] * D_c[i];
  std::vector<double> Ebuf;
  std::vector<int> fcams;
  for (int p = 0; p < n_pts; ++p) {
    if (by_pt[p].empty()) continue;
    double ete[9] = {0};
    for (int k = 0; k < 3; ++k) ete[4 * k] = D_p[3 * p + k] * D_p[3 * p + k];
    double g[3] = {0, 0, 0};
    fcams.clear();
    Ebuf.clear();
    std::vector<double> Es, Fs, bs;
    for (int64_t i : by_pt[p]) {
      const int c = cam_idx[i];
      double res[2], J[18];
      EvalJet(rot + 3 * size_t(c), t + 3 * size_t(c), X + 3 * size_t(p), K9 + 9 * size_t(c), obs_uv[2 * i],
              obs_uv[2 * i + 1], res, J);
      for (int row = 0; row < 2; ++row) {
        for (int k = 0; k < 6; ++k) if (colnorm_c) colnorm_c[6 * c + k] += J[9 * row + k] * J[9 * row + k];
        for (int k = 0; k < 3; ++k) if (colnorm_p) colnorm_p[3 * p + k] += J[9 * row + 6 + k] * J[9 * row + 6 + k];
      }
      int slot = -1;
      for (size_t s2 = 0; s2 < fcams.size(); ++s2) if (fcams[s2] == c) { slot = int(s2); break; }
      if (slot < 0) { slot = int(fcams.size()); fcams.push_back(c); Ebuf.resize(Ebuf.size() + 18, 0.0); }
      double E[6], F[12];
      for (int row = 0; row < 2; ++row) {
        for (int k = 0; k < 3; ++k) E[3 * row + k] = J[9 * row + 6 + k] * scale_p[3 * p + k];
        for (int k = 0; k < 6; ++k) F[6 * row + k] = J[9 * row + k] * scale_c[6 * c + k];
      }
      for (int a = 0; a < 3; ++a) {
        for (int bb = 0; bb < 3; ++bb) ete[3 * a + bb] += E[a] * E[bb] + E[3 + a] * E[3 + bb];
        g[a] += E[a] * res[0] + E[3 + a] * res[1];
        for (int k = 0; k < 6; ++k) Ebuf[18 * slot + 6 * a + k] += E[a] * F[k] + E[3 + a] * F[6 + k];
      }
      for (int a = 0; a < 6; ++a)
        for (int bb = 0; bb < 6; ++bb) S[size_t(6 * c + a) * nf + 6 * c + bb] += F[a] * F[bb] + F[6 + a] * F[6 + bb];
      Es.insert(Es.end(), E, E + 6);
      Fs.insert(Fs.end(), F, F + 12);
      bs.push_back(res[0]); bs.push_back(res[1]);
    }
    double L[9], inv[9];
    if (!Llt3(ete, L)) return -1;
    for (int col = 0; col < 3; ++col) {
      double e[3] = {0, 0, 0}; e[col] = 1.0;
      Llt3Solve(L, e);
      for (int a = 0; a < 3; ++a) inv[3 * a + col] = e[a];
    }
    double ig[3];
    for (int a = 0; a < 3; ++a) ig[a] = inv[3 * a] * g[0] + inv[3 * a + 1] * g[1] + inv[3 * a + 2] * g[2];
    for (size_t q = 0; q < by_pt[p].size(); ++q) {
      const int c = cam_idx[by_pt[p][q]];
      double sj[2];
      for (int row = 0; row < 2; ++row) {
        sj[row] = bs[2 * q + row];
        for (int k = 0; k < 3; ++k) sj[row] -= Es[6 * q + 3 * row + k] * ig[k];
      }
      for (int k = 0; k < 6; ++k) rhs[6 * c + k] += Fs[12 * q + k] * sj[0] + Fs[12 * q + 6 + k] * sj[1];
    }
    const int m = int(fcams.size());
    for (int j = 0; j < m; ++j)
      for (int k = 0; k < m; ++k)
        for (int a = 0; a < 6; ++a)
          for (int bb = 0; bb < 6; ++bb) {
            double s = 0;
            for (int u = 0; u < 3; ++u)
              for (int v = 0; v < 3; ++v) s += Ebuf[18 * j + 6 * u + a] * inv[3 * u + v] * Ebuf[18 * k + 6 * v + bb];
            S[size_t(6 * fcams[j] + a) * nf + 6 * fcams[k] + bb] -= s;
          }
  }
  return 0;
}
