// CPU sanitizer run (tests/asan/Makefile, `make -C tests/asan asan`): the host
// code of the drop-in and its checker under AddressSanitizer + UBSan, no GPU.
//
// Covered:
//   * sfm_amd/csrc/ba_host_layout.h -- set_problem's host checks and counts,
//     camera runs / chunk table, the small path's slice sizes and the camera-
//     run blob's bound -- on the C1 scene, shuffled duplicates, an empty
//     camera with single-view points, bad indices / non-finite uv, and the
//     empty problem; every output checked against a naive recount;
//   * include/sfm_ctracker_compat.hpp -- the pointer dedup / packing of
//     bundleAdjustmentStructAndPose (CSfM.cpp:321-341 gather) and its in-place
//     scatter-back, and the matchFeatures overload, with the C ABI answered by
//     the oracle (this binary links no GPU code: sfm_ba_solve /
//     sfm_match_features below are test stubs over oracle/);
//   * oracle/ (test infrastructure): the BA restatement on the same scenes in
//     all three modes, residuals/Jacobians, the matcher, KLT and GFTT.
// Any sanitizer report aborts the run (halt_on_error), so a clean exit with
// "asan: all checks passed" is the result.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <numeric>
#include <random>
#include <vector>

#include "../../include/sfm_amd.h"
#include "../../include/sfm_ctracker_compat.hpp"
#include "../../sfm_amd/csrc/ba_host_layout.h"

// ---- the oracle's C entry points (oracle/*.cpp, linked in) ----
extern "C" {
struct OOptions;
void oracle_default_options(void* o);
int oracle_ba_solve(const void* opts, int mode, int64_t n_obs, const double* obs_uv, const int32_t* cam_idx,
                    const int32_t* pt_idx, int32_t n_cams, const double* K9, double* rot, double* t, int32_t n_pts,
                    double* X, void* summary, void* trace, int32_t trace_cap, int32_t* trace_len);
int oracle_ba_residuals_jacobians(int64_t n_obs, const double* obs_uv, const int32_t* cam_idx,
                                  const int32_t* pt_idx, const double* K9, const double* rot, const double* t,
                                  const double* X, double* res, double* jac);
int oracle_match_features(const double* pts0, const uint8_t* desc0, int32_t n0, const double* pts1,
                          const uint8_t* desc1, int32_t n1, int32_t nbytes, double ratio_test, double min_distance,
                          double max_distance, int32_t* idx0, int32_t* idx1);
void oracle_min_eigen(const uint8_t* img, int32_t w, int32_t h, float* eig);
void oracle_pyr_down(const uint8_t* src, int32_t w, int32_t h, uint8_t* dst);
void oracle_scharr(const uint8_t* src, int32_t w, int32_t h, int16_t* dxy);
// scene generator (sfm_amd/csrc/scene.cpp, plain C++)
int sfm_scene_generate(int32_t n_cams, int32_t n_pts_total, int32_t p_begin, int32_t p_end, int32_t views,
                       uint64_t seed, double pixel_sigma, double pt_sigma, double rot_sigma, double t_sigma,
                       double* K9, double* rot_true, double* t_true, double* X_true, double* rot_init,
                       double* t_init, double* X_init, double* obs_uv, int32_t* cam_idx, int32_t* pt_idx);

// ---- test stubs of the C ABI the compat header calls (oracle-backed) ----
void sfm_ba_default_options(sfm_ba_options* o) { oracle_default_options(o); }
int sfm_ba_solve(const sfm_ba_options* opts, int32_t mode, int64_t n_obs, const double* obs_uv,
                 const int32_t* cam_idx, const int32_t* pt_idx, int32_t n_cams, const double* K9, double* rot,
                 double* t, int32_t n_pts, double* X, sfm_ba_summary* summary, sfm_ba_iteration* trace,
                 int32_t trace_cap, int32_t* trace_len) {
  return oracle_ba_solve(opts, mode, n_obs, obs_uv, cam_idx, pt_idx, n_cams, K9, rot, t, n_pts, X, summary, trace,
                         trace_cap, trace_len);
}
int sfm_match_features(int32_t, const double* pts0, const uint8_t* desc0, int32_t n0, const double* pts1,
                       const uint8_t* desc1, int32_t n1, int32_t desc_bytes, double ratio_test, double min_distance,
                       double max_distance, int32_t* idx0, int32_t* idx1, int32_t* n_matches) {
  const int r = oracle_match_features(pts0, desc0, n0, pts1, desc1, n1, desc_bytes, ratio_test, min_distance,
                                      max_distance, idx0, idx1);
  if (r < 0) return r;
  *n_matches = r;
  return 0;
}
}

static int g_checks = 0;
#define CHECK(cond)                                                              \
  do {                                                                           \
    ++g_checks;                                                                  \
    if (!(cond)) {                                                               \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

struct Scene {
  int C = 0, P = 0;
  std::vector<double> K9, rot, t, X, uv;
  std::vector<int32_t> cam, pt;
  int64_t N() const { return int64_t(cam.size()); }
};

static Scene make_scene(int C, int P, int views, uint64_t seed) {
  Scene s;
  s.C = C;
  s.P = P;
  const int64_t N = int64_t(P) * views;
  s.K9.resize(9 * size_t(C));
  s.rot.resize(3 * size_t(C));
  s.t.resize(3 * size_t(C));
  s.X.resize(3 * size_t(P));
  s.uv.resize(2 * size_t(N));
  s.cam.resize(size_t(N));
  s.pt.resize(size_t(N));
  std::vector<double> rt(3 * size_t(C)), tt(3 * size_t(C)), Xt(3 * size_t(P));
  const int rc = sfm_scene_generate(C, P, 0, P, views, seed, 0.5, 0.01, 1e-3, 0.01, s.K9.data(), rt.data(),
                                    tt.data(), Xt.data(), s.rot.data(), s.t.data(), s.X.data(), s.uv.data(),
                                    s.cam.data(), s.pt.data());
  CHECK(rc == 0);
  return s;
}

// A naive restatement of hostlayout's outputs, for comparison.
static void check_layout(const Scene& s, const char* name) {
  const int C = s.C, P = s.P;
  const int64_t N = s.N();
  std::vector<int32_t> cam_cnt(size_t(C) + 4), pc(size_t(P) + 1);
  std::vector<int32_t> cam_slice;
  int64_t pairs_est = -1;
  sfm::hostlayout::check_and_count(N, s.uv.data(), s.cam.data(), s.pt.data(), C, P, C <= 127, cam_cnt.data(),
                                   pc.data(), &cam_slice, &pairs_est);
  // first bad observation per kind
  int32_t f[3] = {INT32_MAX, INT32_MAX, INT32_MAX};
  for (int64_t i = 0; i < N; ++i) {
    if ((s.cam[i] < 0 || s.cam[i] >= C) && f[0] == INT32_MAX) f[0] = int32_t(i);
    if ((s.pt[i] < 0 || s.pt[i] >= P) && f[1] == INT32_MAX) f[1] = int32_t(i);
    if (!(std::isfinite(s.uv[2 * i]) && std::isfinite(s.uv[2 * i + 1])) && f[2] == INT32_MAX) f[2] = int32_t(i);
  }
  CHECK(cam_cnt[0] == f[0] && cam_cnt[1] == f[1] && cam_cnt[2] == f[2] && cam_cnt[3] == INT32_MAX);
  const bool bad = f[0] != INT32_MAX || f[1] != INT32_MAX || f[2] != INT32_MAX;
  if (bad) {
    std::printf("  %-14s N=%-7lld C=%-4d P=%-6d rejected at observation %d (as the device validation reports)\n",
                name, (long long)N, C, P, std::min({f[0], f[1], f[2]}));
    return;
  }
  std::vector<int32_t> cc(size_t(C), 0), pp(size_t(P) + 1, 0);
  for (int64_t i = 0; i < N; ++i) {
    ++cc[size_t(s.cam[i])];
    ++pp[size_t(s.pt[i])];
  }
  for (int c = 0; c < C; ++c) CHECK(cam_cnt[4 + size_t(c)] == cc[size_t(c)]);
  CHECK(std::equal(pp.begin(), pp.end(), pc.begin()));
  int64_t pe = 0;
  for (int p = 0; p < P; ++p) pe += int64_t(pp[size_t(p)]) * (pp[size_t(p)] - 1) / 2;
  CHECK(pe == pairs_est);
  // camera runs and the chunk table
  sfm::hostlayout::Runs r;
  sfm::hostlayout::camera_runs(C, cam_cnt.data() + 4, &r);
  int64_t np = 0, nch = 0;
  for (int c = 0; c < C; ++c) {
    CHECK(r.cam_off[size_t(c) + 1] - r.cam_off[size_t(c)] == cc[size_t(c)]);
    CHECK(r.cam_rng[2 * size_t(c)] == np && r.cam_rng[2 * size_t(c) + 1] == np + cc[size_t(c)]);
    for (int64_t w = np / 64; w < (np + cc[size_t(c)] + 63) / 64; ++w) CHECK(r.wcam[size_t(w)] == c);
    np += (cc[size_t(c)] + 63) / 64 * 64;
    nch += (cc[size_t(c)] + 63) / 64;
  }
  CHECK(r.npad == np && int64_t(r.chunks.size()) == nch);
  int64_t covered = 0;
  for (const auto& ch : r.chunks) {
    CHECK(ch.cnt >= 1 && ch.cnt <= 64 && ch.pos % 64 == 0);
    CHECK(ch.pos >= r.cam_rng[2 * size_t(ch.cam)] && ch.pos + ch.cnt <= r.cam_rng[2 * size_t(ch.cam) + 1]);
    CHECK(ch.first == r.cam_off[size_t(ch.cam)] + (ch.pos - r.cam_rng[2 * size_t(ch.cam)]));
    covered += ch.cnt;
  }
  CHECK(covered == N);
  // the camera-run blob (cam_rng | wcam | cam_off | chunks | pt_off | fill)
  // within its bound, each part 256-aligned as StageLayout adds it
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t blob = al(4 * r.cam_rng.size()) + al(4 * r.wcam.size()) + al(4 * r.cam_off.size()) +
                      al(16 * r.chunks.size()) + al(4 * (size_t(P) + 1)) + al(4 * (size_t(P) + size_t(C)));
  CHECK(blob <= sfm::hostlayout::runs_blob_bound(C, N, P));
  // small path: slice sizes vs a point-order walk of every camera's run
  if (C <= 127 && P > 0) {
    CHECK(cam_slice.size() == 8 * size_t(C));
    std::vector<std::vector<int32_t>> per(static_cast<size_t>(C));
    std::vector<int64_t> ids(static_cast<size_t>(N));
    std::iota(ids.begin(), ids.end(), 0);
    std::stable_sort(ids.begin(), ids.end(), [&](int64_t a, int64_t b) { return s.pt[a] < s.pt[b]; });
    for (int64_t i : ids) per[size_t(s.cam[i])].push_back(s.pt[i]);
    std::vector<int32_t> jc(8, 0);
    for (int c = 0; c < C; ++c)
      for (size_t k = 0; k < per[size_t(c)].size(); k += 64) ++jc[size_t(int64_t(per[size_t(c)][k]) * 8 / P)];
    CHECK(sfm::hostlayout::small_slice_max(C, cam_cnt.data() + 4, cam_slice) ==
          *std::max_element(jc.begin(), jc.end()));
  }
  std::printf("  %-14s N=%-7lld C=%-4d P=%-6d layout ok (%lld chunks, %lld pairs est.)\n", name, (long long)N, C, P,
              (long long)nch, (long long)pairs_est);
}

struct Pt2 {
  double x, y;
};
struct M33 {
  double val[9];
};
struct Desc {
  int rows, cols;
  const uint8_t* data;
};

// compat: gather through aliased per-observation pointers, solve (oracle),
// scatter back; compare with the oracle on the packed arrays directly
static void check_compat(const Scene& s, int mode) {
  const int64_t N = s.N();
  std::vector<double> Xw(s.X), rw(s.rot), tw(s.t);
  std::vector<Pt2> obs(static_cast<size_t>(N));
  std::vector<int> camIdx(static_cast<size_t>(N));
  std::vector<double*> pts(static_cast<size_t>(N)), R(size_t(s.C)), T(size_t(s.C));
  std::vector<M33> K(size_t(s.C));
  for (int64_t i = 0; i < N; ++i) {
    obs[size_t(i)] = Pt2{s.uv[2 * i], s.uv[2 * i + 1]};
    camIdx[size_t(i)] = s.cam[size_t(i)];
    pts[size_t(i)] = &Xw[3 * size_t(s.pt[size_t(i)])];
  }
  for (int c = 0; c < s.C; ++c) {
    R[size_t(c)] = &rw[3 * size_t(c)];
    T[size_t(c)] = &tw[3 * size_t(c)];
    std::memcpy(K[size_t(c)].val, &s.K9[9 * size_t(c)], sizeof(double) * 9);
  }
  sfm_ba_summary sm{};
  const int rc = sfm_compat::bundleAdjustmentStructAndPose(obs, camIdx, K, R, T, pts, mode, nullptr, &sm);
  CHECK(rc == 0);
  // the same solve on the caller's own arrays
  std::vector<double> Xo(s.X), ro(s.rot), to(s.t);
  sfm_ba_options o;
  sfm_ba_default_options(&o);
  sfm_ba_summary so{};
  CHECK(sfm_ba_solve(&o, mode, N, s.uv.data(), s.cam.data(), s.pt.data(), s.C, s.K9.data(), ro.data(), to.data(),
                     s.P, Xo.data(), &so, nullptr, 0, nullptr) == 0);
  // the compat layer renumbers points in first-seen order, which changes the
  // Schur summation order: the same solve up to rounding
  CHECK(so.num_iterations == sm.num_iterations && so.termination_type == sm.termination_type);
  CHECK(std::fabs(so.final_cost - sm.final_cost) <= 1e-9 * std::max(1.0, so.final_cost));
  auto close = [](double a, double b) { return std::fabs(a - b) <= 1e-6 * std::max(1.0, std::fabs(b)); };
  for (int64_t i = 0; i < N; ++i)
    for (int k = 0; k < 3; ++k) CHECK(close(pts[size_t(i)][k], Xo[3 * size_t(s.pt[size_t(i)]) + k]));
  for (size_t k = 0; k < rw.size(); ++k) CHECK(close(rw[k], ro[k]) && close(tw[k], to[k]));
  // unobserved points are never written (no pointer reaches them)
}

int main() {
  std::printf("asan: host layout (ba_host_layout.h)\n");
  Scene c1 = make_scene(20, 2000, 10, 0x5F3D2017ull + 1);  // C1: 20 cams / 2000 points / 20000 obs
  check_layout(c1, "C1");
  Scene dup = make_scene(12, 400, 4, 23);  // shuffled caller order with duplicates
  {
    std::mt19937_64 g(7);
    for (int k = 0; k < 40; ++k) {
      const size_t i = size_t(g() % dup.cam.size());
      dup.cam.push_back(dup.cam[i]);
      dup.pt.push_back(dup.pt[i]);
      dup.uv.push_back(dup.uv[2 * i] + 0.1);
      dup.uv.push_back(dup.uv[2 * i + 1] - 0.1);
    }
    std::vector<size_t> perm(dup.cam.size());
    std::iota(perm.begin(), perm.end(), 0);
    std::shuffle(perm.begin(), perm.end(), g);
    Scene sh = dup;
    for (size_t i = 0; i < perm.size(); ++i) {
      sh.cam[i] = dup.cam[perm[i]];
      sh.pt[i] = dup.pt[perm[i]];
      sh.uv[2 * i] = dup.uv[2 * perm[i]];
      sh.uv[2 * i + 1] = dup.uv[2 * perm[i] + 1];
    }
    dup = sh;
  }
  check_layout(dup, "dup-shuffled");
  Scene emp = make_scene(40, 3000, 6, 31);  // an empty camera and single-view points
  {
    Scene e = emp;
    e.cam.clear();
    e.pt.clear();
    e.uv.clear();
    std::vector<int> seen(size_t(e.P), 0);
    for (size_t i = 0; i < emp.cam.size(); ++i) {
      if (emp.cam[i] == 17) continue;                        // camera 17 sees nothing
      if (emp.pt[i] % 50 == 0 && seen[size_t(emp.pt[i])]++) continue;  // every 50th point: one view
      e.cam.push_back(emp.cam[i]);
      e.pt.push_back(emp.pt[i]);
      e.uv.push_back(emp.uv[2 * i]);
      e.uv.push_back(emp.uv[2 * i + 1]);
    }
    emp = e;
  }
  check_layout(emp, "empty-camera");
  Scene badc = c1;
  badc.cam[777] = badc.C;
  check_layout(badc, "bad-camera");
  Scene badp = c1;
  badp.pt[123] = -1;
  badp.cam[5000] = -3;
  check_layout(badp, "bad-point");
  Scene nanuv = c1;
  nanuv.uv[2 * 999 + 1] = std::nan("");
  nanuv.uv[2 * 4000] = INFINITY;
  check_layout(nanuv, "non-finite-uv");
  Scene none;
  none.C = 3;
  none.P = 0;
  none.K9.assign(27, 0.0);
  check_layout(none, "empty");
  Scene big = make_scene(130, 500, 8, 99);  // above the small path's 127 cameras: no slices
  check_layout(big, "C>127");

  std::printf("asan: compat header over the oracle (gather, solve, scatter-back)\n");
  for (int mode = 0; mode < 3; ++mode) {
    check_compat(c1, mode);
    check_compat(dup, mode);
    check_compat(emp, mode);
    std::printf("  mode %d: C1, dup-shuffled, empty-camera ok\n", mode);
  }
  {
    std::vector<double> res(2 * size_t(c1.N())), jac(18 * size_t(c1.N()));
    CHECK(oracle_ba_residuals_jacobians(c1.N(), c1.uv.data(), c1.cam.data(), c1.pt.data(), c1.K9.data(),
                                        c1.rot.data(), c1.t.data(), c1.X.data(), res.data(), jac.data()) == 0);
    for (double v : res) CHECK(std::isfinite(v));
  }

  std::printf("asan: matcher (compat overload over the oracle), KLT / GFTT oracle kernels\n");
  {
    std::mt19937_64 g(11);
    const int n0 = 500, n1 = 520;
    std::vector<uint8_t> d0(64 * size_t(n0)), d1(64 * size_t(n1));
    for (auto& b : d0) b = uint8_t(g());
    for (auto& b : d1) b = uint8_t(g());
    for (int i = 0; i < n0; ++i) std::memcpy(&d1[64 * size_t(i)], &d0[64 * size_t(i)], 64), d1[64 * size_t(i)] ^= 1;
    std::vector<Pt2> p0(static_cast<size_t>(n0)), p1(static_cast<size_t>(n1));
    std::uniform_real_distribution<double> U(0, 1280), D(-5, 5);
    for (int i = 0; i < n0; ++i) p0[size_t(i)] = Pt2{U(g), U(g) * 0.5625};
    for (int i = 0; i < n1; ++i) p1[size_t(i)] = i < n0 ? Pt2{p0[size_t(i)].x + D(g), p0[size_t(i)].y + D(g)} : Pt2{U(g), U(g)};
    Desc a{n0, 64, d0.data()}, b{n1, 64, d1.data()};
    std::vector<int> m0{-7}, m1{-7};  // the overload APPENDS (push_back), as the reference
    CHECK(sfm_compat::matchFeatures(p0, a, p1, b, m0, m1) == 0);
    CHECK(m0.size() == m1.size() && m0.size() > 100 && m0[0] == -7);
    std::printf("  matcher: %zu matches appended\n", m0.size() - 1);
    const int w = 320, h = 240;
    std::vector<uint8_t> img(size_t(w) * h), half(size_t(w / 2) * (h / 2));
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) img[size_t(y) * w + x] = uint8_t((x * 7 + y * 13 + ((x / 16 + y / 16) & 1) * 90) & 255);
    std::vector<float> eig(size_t(w) * h);
    oracle_min_eigen(img.data(), w, h, eig.data());
    oracle_pyr_down(img.data(), w, h, half.data());
    std::vector<int16_t> dxy(2 * size_t(w) * h);
    oracle_scharr(img.data(), w, h, dxy.data());
    std::printf("  gftt / pyramid / scharr ok\n");
  }
  std::printf("asan: all checks passed (%d checks)\n", g_checks);
  return 0;
}
