// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY (see ba_oracle.cpp header).  Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
//
// Restatement of the reference's corner detector for the optical-flow
// tracker:
//   CTracker::detectFeaturesOpticalFlow   /root/reference/CTracker.cpp:252-272
//     goodFeaturesToTrack(grey, pts, 500, 0.05, 10)            (:262)
//     cornerSubPix(grey, pts, Size(5,5), Size(-1,-1),
//                  TermCriteria(COUNT|EPS, 20, 0.03))          (:265)
//     pts.size() < _minFeatures (5, CTracker.cpp:32) -> false  (:267)
// The arithmetic lives in OpenCV 3.0 (README.md:28; not vendored, SURVEY.md
// §8c).  Restated published semantics (modules/imgproc/src/featureselect.cpp,
// corner.cpp, cornersubpix.cpp, samplers.cpp), blockSize 3, Sobel aperture 3,
// no Harris, no mask:
//   * response: Sobel 3x3 derivatives of the u8 frame (BORDER_REFLECT_101),
//     scaled by 1/(4*3*255) (cornerEigenValsVecs' scale); per pixel the
//     products Ix^2, IxIy, Iy^2 (float); unnormalised 3x3 box sums
//     (BORDER_REFLECT_101); min eigenvalue
//     (a+c) - sqrt((a-c)^2 + b^2), a = sxx/2, c = syy/2, b = sxy (float).
//   * threshold TOZERO at (float)(max * qualityLevel); 3x3 dilate (border
//     ignored); candidates = interior pixels (1..w-2, 1..h-2) with
//     v != 0 && v == dilated.
//   * order: response descending; ties -> larger raster index first (the
//     address tie-break of OpenCV's greaterThanPtr).
//   * greedy: accept a candidate unless an accepted corner lies at squared
//     distance < minDistance^2; stop at maxCorners (the cell grid OpenCV
//     uses is only an index over the same test).
//   * cornerSubPix: 11x11 window, Gaussian weights exp(-x^2)exp(-y^2) over
//     x,y in [-1,1] (float), 13x13 bilinear resample around the estimate
//     (float weights; taps clamped to the frame outside it), central
//     differences, 2x2 normal equations in double, update in float, stop
//     on 20 iterations or squared step <= 0.03^2 or leaving the frame;
//     a result more than 5 px from the start reverts to the start.
// Deliberate definitions where OpenCV's float/double rounding order is an
// implementation detail (its box filter slides a running sum, its 8u->32f
// subpixel sampler uses an incremental form): box sums are the direct
// (left + centre) + right sums, Sobel output is the double product rounded
// once to float, and the five double window sums of cornerSubPix are
// reduced in a fixed 64-lane order (lane L sums pixels L, L + 64, ... in
// turn, then an xor butterfly 32..1), which the device kernel reproduces bit for bit.
//
// PARITY UNPINNED against OpenCV: it is absent here and the reference holds
// no test or fixture for this path (its only tests are empty XCTest
// templates).  tests/gftt_ref.py pins this restatement with an independent
// numpy one.
// ============================================================================
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

inline int r101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
  }
  return i;
}

void min_eigen(const uint8_t* img, int w, int h, float* eig) {
  const double scale = 1.0 / (4.0 * 3.0 * 255.0);
  std::vector<float> cxx(size_t(w) * h), cxy(size_t(w) * h), cyy(size_t(w) * h);
  auto P = [&](int x, int y) { return int(img[size_t(r101(y, h)) * w + r101(x, w)]); };
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const int dx = (P(x + 1, y - 1) - P(x - 1, y - 1)) + 2 * (P(x + 1, y) - P(x - 1, y)) +
                     (P(x + 1, y + 1) - P(x - 1, y + 1));
      const int dy = (P(x - 1, y + 1) - P(x - 1, y - 1)) + 2 * (P(x, y + 1) - P(x, y - 1)) +
                     (P(x + 1, y + 1) - P(x + 1, y - 1));
      const float ix = float(double(dx) * scale), iy = float(double(dy) * scale);
      const size_t o = size_t(y) * w + x;
      cxx[o] = ix * ix;
      cxy[o] = ix * iy;
      cyy[o] = iy * iy;
    }
  std::vector<float> rxx(size_t(w) * h), rxy(size_t(w) * h), ryy(size_t(w) * h);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const size_t a = size_t(y) * w + r101(x - 1, w), b = size_t(y) * w + x, c = size_t(y) * w + r101(x + 1, w);
      rxx[b] = (cxx[a] + cxx[b]) + cxx[c];
      rxy[b] = (cxy[a] + cxy[b]) + cxy[c];
      ryy[b] = (cyy[a] + cyy[b]) + cyy[c];
    }
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const size_t a = size_t(r101(y - 1, h)) * w + x, b = size_t(y) * w + x, c = size_t(r101(y + 1, h)) * w + x;
      const float sxx = (rxx[a] + rxx[b]) + rxx[c];
      const float sxy = (rxy[a] + rxy[b]) + rxy[c];
      const float syy = (ryy[a] + ryy[b]) + ryy[c];
      const float A = sxx * 0.5f, B = sxy, Cc = syy * 0.5f;
      eig[b] = (A + Cc) - std::sqrt((A - Cc) * (A - Cc) + B * B);
    }
}

// Candidates (raster order) after threshold + dilate; returns the threshold.
float candidates(const float* eig, int w, int h, double quality, std::vector<uint64_t>& keys) {
  float mx = -FLT_MAX;
  for (size_t i = 0; i < size_t(w) * h; ++i) mx = std::max(mx, eig[i]);
  const float thr = float(double(mx) * quality);
  auto T = [&](int x, int y) {
    const float v = eig[size_t(y) * w + x];
    return v > thr ? v : 0.0f;
  };
  keys.clear();
  for (int y = 1; y < h - 1; ++y)
    for (int x = 1; x < w - 1; ++x) {
      const float v = T(x, y);
      if (v == 0.0f) continue;
      float d = v;
      for (int yy = y - 1; yy <= y + 1; ++yy)
        for (int xx = x - 1; xx <= x + 1; ++xx) d = std::max(d, T(xx, yy));
      if (v == d) {
        uint32_t bits;
        std::memcpy(&bits, &v, 4);
        keys.push_back((uint64_t(bits) << 32) | uint32_t(y * w + x));
      }
    }
  return thr;
}

int select_corners(std::vector<uint64_t>& keys, int w, int max_corners, double min_distance, float* out) {
  // response descending, then raster index descending (v > 0: the float
  // bits order like the values)
  std::sort(keys.begin(), keys.end(), [](uint64_t a, uint64_t b) { return a > b; });
  const double md2 = min_distance * min_distance;
  std::vector<int> ax, ay;
  int n = 0;
  for (uint64_t k : keys) {
    const int lin = int(uint32_t(k));
    const int x = lin % w, y = lin / w;
    bool good = true;
    if (min_distance >= 1.0)
      for (size_t j = 0; j < ax.size() && good; ++j) {
        const float dx = float(x - ax[j]), dy = float(y - ay[j]);
        if (double(dx * dx + dy * dy) < md2) good = false;
      }
    if (!good) continue;
    ax.push_back(x);
    ay.push_back(y);
    out[2 * n] = float(x);
    out[2 * n + 1] = float(y);
    if (++n == max_corners) break;
  }
  return n;
}

// Fixed-order reduction of the 121 window terms (see header).
double lane_sum(const double* t, int n) {
  double v[64];
  for (int L = 0; L < 64; ++L) {
    v[L] = L < n ? t[L] : 0.0;
    for (int k = L + 64; k < n; k += 64) v[L] = v[L] + t[k];
  }
  for (int off = 32; off >= 1; off >>= 1) {
    double nv[64];
    for (int L = 0; L < 64; ++L) nv[L] = v[L] + v[L ^ off];
    for (int L = 0; L < 64; ++L) v[L] = nv[L];
  }
  return v[0];
}

void corner_subpix(const uint8_t* img, int w, int h, float* pts, int n, int win, int max_iter, double eps) {
  const int ww = 2 * win + 1, sw = ww + 2;  // 11, 13
  std::vector<float> mask(size_t(ww) * ww);
  for (int i = 0; i < ww; ++i) {
    const float y = float(i - win) / float(win);
    const float vy = std::exp(-y * y);
    for (int j = 0; j < ww; ++j) {
      const float x = float(j - win) / float(win);
      mask[size_t(i) * ww + j] = vy * std::exp(-x * x);
    }
  }
  max_iter = std::min(std::max(max_iter, 1), 100);
  const double eps2 = std::max(eps, 0.0) * std::max(eps, 0.0);
  std::vector<float> sub(size_t(sw) * sw);
  std::vector<double> t[5];
  for (auto& v : t) v.resize(size_t(ww) * ww);
  auto px = [&](int x, int y) {
    x = std::min(std::max(x, 0), w - 1);
    y = std::min(std::max(y, 0), h - 1);
    return float(img[size_t(y) * w + x]);
  };
  for (int p = 0; p < n; ++p) {
    const float tx = pts[2 * p], ty = pts[2 * p + 1];
    float cx = tx, cy = ty;
    int iter = 0;
    double err = 0.0;
    do {
      // 13x13 bilinear resample centred on (cx, cy)
      const float ox = cx - float(sw - 1) * 0.5f, oy = cy - float(sw - 1) * 0.5f;
      const int ix = int(std::floor(ox)), iy = int(std::floor(oy));
      const float a = ox - float(ix), b = oy - float(iy);
      const float a11 = (1.f - a) * (1.f - b), a12 = a * (1.f - b), a21 = (1.f - a) * b, a22 = a * b;
      for (int i = 0; i < sw; ++i)
        for (int j = 0; j < sw; ++j) {
          const int X = ix + j, Y = iy + i;
          sub[size_t(i) * sw + j] =
              ((px(X, Y) * a11 + px(X + 1, Y) * a12) + px(X, Y + 1) * a21) + px(X + 1, Y + 1) * a22;
        }
      for (int i = 0, k = 0; i < ww; ++i) {
        const double py = double(i - win);
        const float* s = &sub[size_t(i + 1) * sw + 1];
        for (int j = 0; j < ww; ++j, ++k) {
          const double m = mask[k];
          const double tgx = double(s[j + 1] - s[j - 1]);
          const double tgy = double(s[j + sw] - s[j - sw]);
          const double gxx = tgx * tgx * m, gxy = tgx * tgy * m, gyy = tgy * tgy * m;
          const double pxx = double(j - win);
          t[0][k] = gxx;
          t[1][k] = gxy;
          t[2][k] = gyy;
          t[3][k] = gxx * pxx + gxy * py;
          t[4][k] = gxy * pxx + gyy * py;
        }
      }
      const int nk = ww * ww;
      const double A = lane_sum(t[0].data(), nk), B = lane_sum(t[1].data(), nk), C = lane_sum(t[2].data(), nk),
                   bb1 = lane_sum(t[3].data(), nk), bb2 = lane_sum(t[4].data(), nk);
      const double det = A * C - B * B;
      if (std::fabs(det) <= DBL_EPSILON * DBL_EPSILON) break;
      const double sc = 1.0 / det;
      const float nx = float(cx + C * sc * bb1 - B * sc * bb2);
      const float ny = float(cy - B * sc * bb1 + A * sc * bb2);
      err = double((nx - cx) * (nx - cx) + (ny - cy) * (ny - cy));
      cx = nx;
      cy = ny;
      if (cx < 0 || cx >= float(w) || cy < 0 || cy >= float(h)) break;
    } while (++iter < max_iter && err > eps2);
    if (std::fabs(cx - tx) > float(win) || std::fabs(cy - ty) > float(win)) {
      cx = tx;
      cy = ty;
    }
    pts[2 * p] = cx;
    pts[2 * p + 1] = cy;
  }
}

}  // namespace

extern "C" {

void oracle_min_eigen(const uint8_t* img, int32_t w, int32_t h, float* eig) { min_eigen(img, w, h, eig); }

// goodFeaturesToTrack (integer corners, before cornerSubPix); returns the count.
int32_t oracle_good_features(const uint8_t* img, int32_t w, int32_t h, int32_t max_corners, double quality,
                             double min_distance, float* out) {
  if (w < 3 || h < 3 || max_corners < 1) return 0;
  std::vector<float> eig(size_t(w) * h);
  min_eigen(img, w, h, eig.data());
  std::vector<uint64_t> keys;
  candidates(eig.data(), w, h, quality, keys);
  return select_corners(keys, w, max_corners, min_distance, out);
}

void oracle_corner_subpix(const uint8_t* img, int32_t w, int32_t h, float* pts, int32_t n, int32_t win,
                          int32_t max_iter, double eps) {
  corner_subpix(img, w, h, pts, n, win, max_iter, eps);
}

// CTracker::detectFeaturesOpticalFlow minus setPoints: corners after
// cornerSubPix; the reference's bool is (count >= min_features).
int32_t oracle_detect_features_of(const uint8_t* img, int32_t w, int32_t h, int32_t max_corners, double quality,
                                  double min_distance, int32_t win, int32_t max_iter, double eps, float* out) {
  const int n = oracle_good_features(img, w, h, max_corners, quality, min_distance, out);
  corner_subpix(img, w, h, out, n, win, max_iter, eps);
  return n;
}

}  // extern "C"
