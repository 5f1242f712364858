// Synthetic bundle-adjustment scenes.
//
// The reference ships no data: its only camera model is the hard-coded
// iPhone-6s intrinsics of main/main.cpp:47-50 and its only scene is a
// developer's local video (main/main.cpp:39).  Benchmarks and parity tests
// therefore run on seeded synthetic object-scanning scenes that mimic what
// CSfM::bundleAdjustment (CSfM.cpp:310-348) hands to
// CTracker::bundleAdjustmentStructAndPose (CTracker.cpp:670-702):
//   * identical undistorted intrinsics per keyframe (K == Kopt, no distortion),
//   * the first keyframe at exactly rot = 0 (CFrame.cpp:229-235 setPose()),
//   * points of a small object inside [-1,1]^3 seen by many keyframes.
//
// Streams (fixed, so any re-implementation reproduces the same bytes):
//   * camera geometry: SplitMix64(seed); cameras 1..C-1 draw polar u, azimuth u
//   * camera initial guess: SplitMix64(seed ^ 0xA5A5A5A5DEADBEEF); per camera
//     3 rot normals (camera 0 skips them and keeps rot exactly 0), 3 t normals
//   * point p: SplitMix64(hash(seed ^ hash(p + 1))); x,y,z uniforms in [-1,1],
//     `views` partial Fisher-Yates draws over the identity camera permutation,
//     2 pixel-noise normals per view in ascending camera order, then 3
//     initial-guess normals.
// Per-point streams make any point range [p_begin, p_end) reproducible on
// its own, so landmark shards are generated where they are solved.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include <algorithm>

namespace {

inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct SplitMix64 {
  uint64_t s;
  explicit SplitMix64(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uniform() { return double(next() >> 11) * (1.0 / 9007199254740992.0); }
  // Box-Muller, one value per call (the sine partner is discarded so that the
  // number of draws per normal is always exactly two).
  double normal() {
    double u1 = 1.0 - uniform();  // (0, 1]
    double u2 = uniform();
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586476925 * u2);
  }
};

void cross3(const double a[3], const double b[3], double o[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

void normalize3(double v[3]) {
  double n = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  v[0] /= n; v[1] /= n; v[2] /= n;
}

// Rotation matrix (row-major) -> angle-axis through a unit quaternion
// (Shepperd's method), well conditioned for every angle in [0, pi].
void rotmat_to_angle_axis(const double R[9], double aa[3]) {
  double tr = R[0] + R[4] + R[8];
  double q[4];  // w x y z
  if (tr > 0) {
    double s = std::sqrt(tr + 1.0) * 2;
    q[0] = 0.25 * s; q[1] = (R[7] - R[5]) / s; q[2] = (R[2] - R[6]) / s; q[3] = (R[3] - R[1]) / s;
  } else if (R[0] > R[4] && R[0] > R[8]) {
    double s = std::sqrt(1.0 + R[0] - R[4] - R[8]) * 2;
    q[0] = (R[7] - R[5]) / s; q[1] = 0.25 * s; q[2] = (R[1] + R[3]) / s; q[3] = (R[2] + R[6]) / s;
  } else if (R[4] > R[8]) {
    double s = std::sqrt(1.0 + R[4] - R[0] - R[8]) * 2;
    q[0] = (R[2] - R[6]) / s; q[1] = (R[1] + R[3]) / s; q[2] = 0.25 * s; q[3] = (R[5] + R[7]) / s;
  } else {
    double s = std::sqrt(1.0 + R[8] - R[0] - R[4]) * 2;
    q[0] = (R[3] - R[1]) / s; q[1] = (R[2] + R[6]) / s; q[2] = (R[5] + R[7]) / s; q[3] = 0.25 * s;
  }
  if (q[0] < 0) { q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3]; }
  double sn = std::sqrt(q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (sn < 1e-300) { aa[0] = aa[1] = aa[2] = 0; return; }
  double angle = 2.0 * std::atan2(sn, q[0]);
  aa[0] = q[1] / sn * angle; aa[1] = q[2] / sn * angle; aa[2] = q[3] / sn * angle;
}

}  // namespace

extern "C" {

// Intrinsics of main/main.cpp:47-50 (undistorted == Kopt here, skew 0).
void sfm_scene_default_intrinsics(double K9[9]) {
  const double fx = 1072.606693272117800, fy = 1067.197515608619600;
  const double cx = 648.780750477178910, cy = 364.503435962496890;
  const double k[9] = {fx, 0, cx, 0, fy, cy, 0, 0, 1};
  std::memcpy(K9, k, sizeof(k));
}

// Generates points [p_begin, p_end) of a scene with n_pts_total points and
// all of its cameras; n_obs = (p_end - p_begin) * views observations sorted
// by (point, camera), pt_idx relative to p_begin.  All output arrays are
// caller-owned: K9 [C][9], rot/t [C][3], X [P][3], obs_uv [N][2],
// cam_idx/pt_idx [N]; *_true / *_init may be NULL.  Returns 0 or -22.
int sfm_scene_generate(int32_t n_cams, int32_t n_pts_total, int32_t p_begin, int32_t p_end, int32_t views,
                       uint64_t seed, double pixel_sigma, double pt_sigma, double rot_sigma, double t_sigma,
                       double* K9, double* rot_true, double* t_true, double* X_true,
                       double* rot_init, double* t_init, double* X_init,
                       double* obs_uv, int32_t* cam_idx, int32_t* pt_idx) {
  if (n_cams < 1 || n_pts_total < 0 || p_begin < 0 || p_end < p_begin || p_end > n_pts_total || views < 1 ||
      views > n_cams || !K9 || !obs_uv || !cam_idx || !pt_idx)
    return -22;
  double Kd[9];
  sfm_scene_default_intrinsics(Kd);
  std::vector<double> R(size_t(n_cams) * 9), rot(size_t(n_cams) * 3), t(size_t(n_cams) * 3);
  SplitMix64 crng(seed);
  for (int c = 0; c < n_cams; ++c) {
    std::memcpy(K9 + 9 * size_t(c), Kd, sizeof(Kd));
    double* Rc = &R[9 * size_t(c)];
    if (c == 0) {
      // first keyframe: identity rotation, centre (0,0,-8) -> t = (0,0,8)
      const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
      std::memcpy(Rc, I, sizeof(I));
      rot[0] = rot[1] = rot[2] = 0;
      t[0] = 0; t[1] = 0; t[2] = 8;
      continue;
    }
    const double kPi = 3.14159265358979323846;
    double polar = (30.0 + 60.0 * crng.uniform()) * kPi / 180.0;
    double az = 2.0 * kPi * crng.uniform();
    double C[3] = {8 * std::sin(polar) * std::cos(az), 8 * std::sin(polar) * std::sin(az), 8 * std::cos(polar)};
    double z[3] = {-C[0], -C[1], -C[2]};
    normalize3(z);
    const double up[3] = {0, 0, 1};
    double x[3], y[3];
    cross3(z, up, x);
    normalize3(x);
    cross3(z, x, y);
    for (int k = 0; k < 3; ++k) { Rc[k] = x[k]; Rc[3 + k] = y[k]; Rc[6 + k] = z[k]; }
    for (int r = 0; r < 3; ++r)
      t[3 * size_t(c) + r] = -(Rc[3 * r] * C[0] + Rc[3 * r + 1] * C[1] + Rc[3 * r + 2] * C[2]);
    rotmat_to_angle_axis(Rc, &rot[3 * size_t(c)]);
  }
  if (rot_true) std::memcpy(rot_true, rot.data(), rot.size() * sizeof(double));
  if (t_true) std::memcpy(t_true, t.data(), t.size() * sizeof(double));
  {
    SplitMix64 irng(seed ^ 0xA5A5A5A5DEADBEEFull);
    std::vector<double> ri(rot), ti(t);
    for (int c = 0; c < n_cams; ++c) {
      if (c != 0)
        for (int k = 0; k < 3; ++k) ri[3 * size_t(c) + k] += rot_sigma * irng.normal();
      for (int k = 0; k < 3; ++k) ti[3 * size_t(c) + k] += t_sigma * irng.normal();
    }
    if (rot_init) std::memcpy(rot_init, ri.data(), ri.size() * sizeof(double));
    if (t_init) std::memcpy(t_init, ti.data(), ti.size() * sizeof(double));
  }
  // sparse partial Fisher-Yates: only the (<= 2*views) touched slots are stored
  std::vector<int32_t> key(2 * views), val(2 * views), sel(views);
  int64_t o = 0;
  for (int64_t p = p_begin; p < p_end; ++p) {
    SplitMix64 prng(mix64(seed ^ mix64(uint64_t(p) + 1)));
    double Xp[3];
    for (int k = 0; k < 3; ++k) Xp[k] = 2.0 * prng.uniform() - 1.0;
    int nk = 0;
    auto get = [&](int32_t i) { for (int s2 = 0; s2 < nk; ++s2) if (key[s2] == i) return val[s2]; return i; };
    auto put = [&](int32_t i, int32_t v) {
      for (int s2 = 0; s2 < nk; ++s2) if (key[s2] == i) { val[s2] = v; return; }
      key[nk] = i; val[nk] = v; ++nk;
    };
    for (int i = 0; i < views; ++i) {
      int64_t j = i + int64_t(prng.uniform() * double(n_cams - i));
      if (j >= n_cams) j = n_cams - 1;
      const int32_t vi = get(i), vj = get(int32_t(j));
      put(i, vj); put(int32_t(j), vi);
      sel[i] = vj;
    }
    std::sort(sel.begin(), sel.end());
    for (int i = 0; i < views; ++i) {
      int c = sel[i];
      const double* Rc = &R[9 * size_t(c)];
      double pc[3];
      for (int r = 0; r < 3; ++r)
        pc[r] = Rc[3 * r] * Xp[0] + Rc[3 * r + 1] * Xp[1] + Rc[3 * r + 2] * Xp[2] + t[3 * size_t(c) + r];
      double xp = pc[0] / pc[2], yp = pc[1] / pc[2];
      double u = Kd[0] * xp + Kd[1] * yp + Kd[2];
      double v = Kd[4] * yp + Kd[5];
      u += pixel_sigma * prng.normal();
      v += pixel_sigma * prng.normal();
      obs_uv[2 * o] = u; obs_uv[2 * o + 1] = v;
      cam_idx[o] = c; pt_idx[o] = int32_t(p - p_begin);
      ++o;
    }
    const int64_t lp = p - p_begin;
    if (X_true) for (int k = 0; k < 3; ++k) X_true[3 * lp + k] = Xp[k];
    for (int k = 0; k < 3; ++k) {
      const double e = pt_sigma * prng.normal();
      if (X_init) X_init[3 * lp + k] = Xp[k] + e;
    }
  }
  return 0;
}

}  // extern "C"
