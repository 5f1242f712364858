// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY (see ba_oracle.cpp header).  Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
//
// Restatement of the reference's optical-flow tracker:
//   CTracker::computeOpticalFlow          /root/reference/CTracker.cpp:480-562
//   CFrame::findClosestPointIndexDistorted /root/reference/CFrame.cpp:437-450
// and of the external call it makes at CTracker.cpp:513,
//   cv::calcOpticalFlowPyrLK(prev, next, prevPts, currPts, status, err,
//                            Size(21,21), 3, TermCriteria(COUNT|EPS, 20, 0.03),
//                            0, 0.001)
// whose library (OpenCV 3.0, README.md:28) is not vendored.
// Restated OpenCV semantics (modules/video/src/lkpyramid.cpp, published):
//   * pyramid: level 0 = the frame; level l = pyrDown(level l-1), size
//     ((w+1)/2, (h+1)/2), 5x5 kernel [1 4 6 4 1]^2 / 256 with +128 rounding,
//     BORDER_REFLECT_101; every level is read through a reflect-101 border
//     (copyMakeBorder of winSize); derivatives read as 0 outside the level.
//   * derivatives (calcSharrDeriv): t0 = 3(s[y-1]+s[y+1]) + 10 s[y],
//     t1 = s[y+1]-s[y-1] (rows reflect-101), Ix = t0[x+1]-t0[x-1],
//     Iy = 3(t1[x-1]+t1[x+1]) + 10 t1[x] (columns reflect-101), int16.
//   * per point, levels maxLevel..0 (LKTrackerInvoker): patch and gradients
//     by 14-bit fixed-point bilinear weights (cvRound, iw11 = 2^14 - rest),
//     I descaled by 9 bits (x32), gradients by 14; A = sum of gradient
//     products * 2^-20; minEig gate; up to maxCount Newton steps with the
//     eps^2 and oscillation (|d + d_prev| < 0.01, half-step back) stops.
//   * one deliberate difference: the integer products are summed exactly
//     (int64) and converted to float once; OpenCV sums them in float (SSE
//     lanes), which differs only by float rounding of the partial sums.
// The reference converts its Point2d points to Point2f for the call
// (CTracker.cpp:498-503) — restated as a float cast.
//
// PARITY UNPINNED: OpenCV is absent here and the reference holds no test or
// fixture for this path (its only tests are empty XCTest templates).
// ============================================================================
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

struct Level {
  int w = 0, h = 0;
  std::vector<uint8_t> img;
  std::vector<int16_t> dxy;  // [h][w][2]
};

void pyr_down(const uint8_t* s, int w, int h, uint8_t* d) {
  static const int k[5] = {1, 4, 6, 4, 1};
  const int dw = (w + 1) / 2, dh = (h + 1) / 2;
  for (int y = 0; y < dh; ++y)
    for (int x = 0; x < dw; ++x) {
      int acc = 0;
      for (int i = 0; i < 5; ++i) {
        const uint8_t* row = s + size_t(r101(2 * y + i - 2, h)) * w;
        int hs = 0;
        for (int j = 0; j < 5; ++j) hs += k[j] * row[r101(2 * x + j - 2, w)];
        acc += k[i] * hs;
      }
      d[size_t(y) * dw + x] = uint8_t((acc + 128) >> 8);
    }
}

void scharr(const uint8_t* s, int w, int h, int16_t* d) {
  std::vector<int> t0(w), t1(w);
  for (int y = 0; y < h; ++y) {
    const uint8_t* s0 = s + size_t(y > 0 ? y - 1 : (h > 1 ? 1 : 0)) * w;
    const uint8_t* s1 = s + size_t(y) * w;
    const uint8_t* s2 = s + size_t(y < h - 1 ? y + 1 : (h > 1 ? h - 2 : 0)) * w;
    for (int x = 0; x < w; ++x) {
      t0[x] = (s0[x] + s2[x]) * 3 + s1[x] * 10;
      t1[x] = s2[x] - s0[x];
    }
    for (int x = 0; x < w; ++x) {
      const int xl = x > 0 ? x - 1 : (w > 1 ? 1 : 0), xr = x < w - 1 ? x + 1 : (w > 1 ? w - 2 : 0);
      d[(size_t(y) * w + x) * 2] = int16_t(t0[xr] - t0[xl]);
      d[(size_t(y) * w + x) * 2 + 1] = int16_t((t1[xr] + t1[xl]) * 3 + t1[x] * 10);
    }
  }
}

std::vector<Level> build_pyramid(const uint8_t* img, int w, int h, int max_level, int win, bool derivs) {
  std::vector<Level> L;
  Level l0;
  l0.w = w;
  l0.h = h;
  l0.img.assign(img, img + size_t(w) * h);
  L.push_back(std::move(l0));
  // buildOpticalFlowPyramid stops once a level would not exceed the window.
  for (int l = 1; l <= max_level; ++l) {
    const Level& p = L.back();
    const int nw = (p.w + 1) / 2, nh = (p.h + 1) / 2;
    if (nw <= win || nh <= win) break;
    Level n;
    n.w = nw;
    n.h = nh;
    n.img.resize(size_t(nw) * nh);
    pyr_down(p.img.data(), p.w, p.h, n.img.data());
    L.push_back(std::move(n));
  }
  if (derivs)
    for (Level& l : L) {
      l.dxy.resize(size_t(l.w) * l.h * 2);
      scharr(l.img.data(), l.w, l.h, l.dxy.data());
    }
  return L;
}

inline int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }
inline int pix(const Level& l, int x, int y) { return l.img[size_t(r101(y, l.h)) * l.w + r101(x, l.w)]; }
inline int der(const Level& l, int x, int y, int c) {
  if (x < 0 || y < 0 || x >= l.w || y >= l.h) return 0;
  return l.dxy[(size_t(y) * l.w + x) * 2 + c];
}

struct LkParams {
  int win, max_level, max_count;
  double eps2;
  double min_eig;
};

// LKTrackerInvoker::operator() for one point over every level.
void track_point(const std::vector<Level>& I, const std::vector<Level>& J, int maxLevel, const LkParams& P,
                 float px, float py, float* out_x, float* out_y, uint8_t* status) {
  const int win = P.win, area = win * win;
  const float half = (win - 1) * 0.5f;
  const int W_BITS = 14;
  const float FLT_SCALE = 1.f / (1 << 20);
  std::vector<int> Ip(area), Dx(area), Dy(area);
  float nx = 0.f, ny = 0.f;  // nextPts[ptidx]
  *status = 1;
  for (int level = maxLevel; level >= 0; --level) {
    const Level& Li = I[level];
    const Level& Lj = J[level];
    const float sc = (float)(1. / (1 << level));
    float ppx = px * sc, ppy = py * sc;
    float npx, npy;
    if (level == maxLevel) { npx = ppx; npy = ppy; }
    else { npx = nx * 2.f; npy = ny * 2.f; }
    nx = npx;
    ny = npy;
    ppx -= half;
    ppy -= half;
    const int ipx = (int)std::floor(ppx), ipy = (int)std::floor(ppy);
    if (ipx < -win || ipx >= Li.w || ipy < -win || ipy >= Li.h) {
      if (level == 0) *status = 0;
      continue;
    }
    float a = ppx - ipx, b = ppy - ipy;
    int iw00 = (int)std::nearbyint((1.f - a) * (1.f - b) * (1 << W_BITS));
    int iw01 = (int)std::nearbyint(a * (1.f - b) * (1 << W_BITS));
    int iw10 = (int)std::nearbyint((1.f - a) * b * (1 << W_BITS));
    int iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
    int64_t iA11 = 0, iA12 = 0, iA22 = 0;
    for (int y = 0; y < win; ++y)
      for (int x = 0; x < win; ++x) {
        const int X = ipx + x, Y = ipy + y;
        const int ival = descale(pix(Li, X, Y) * iw00 + pix(Li, X + 1, Y) * iw01 + pix(Li, X, Y + 1) * iw10 +
                                     pix(Li, X + 1, Y + 1) * iw11, W_BITS - 5);
        const int ixv = descale(der(Li, X, Y, 0) * iw00 + der(Li, X + 1, Y, 0) * iw01 + der(Li, X, Y + 1, 0) * iw10 +
                                    der(Li, X + 1, Y + 1, 0) * iw11, W_BITS);
        const int iyv = descale(der(Li, X, Y, 1) * iw00 + der(Li, X + 1, Y, 1) * iw01 + der(Li, X, Y + 1, 1) * iw10 +
                                    der(Li, X + 1, Y + 1, 1) * iw11, W_BITS);
        const int k = y * win + x;
        Ip[k] = ival;
        Dx[k] = ixv;
        Dy[k] = iyv;
        iA11 += int64_t(ixv) * ixv;
        iA12 += int64_t(ixv) * iyv;
        iA22 += int64_t(iyv) * iyv;
      }
    const float A11 = (float)iA11 * FLT_SCALE, A12 = (float)iA12 * FLT_SCALE, A22 = (float)iA22 * FLT_SCALE;
    float D = A11 * A22 - A12 * A12;
    const float minEig = (A22 + A11 - std::sqrt((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * area);
    if ((double)minEig < P.min_eig || D < FLT_EPSILON) {
      if (level == 0) *status = 0;
      continue;
    }
    D = 1.f / D;
    npx -= half;
    npy -= half;
    float pdx = 0.f, pdy = 0.f;
    for (int j = 0; j < P.max_count; ++j) {
      const int inx = (int)std::floor(npx), iny = (int)std::floor(npy);
      if (inx < -win || inx >= Lj.w || iny < -win || iny >= Lj.h) {
        if (level == 0) *status = 0;
        break;
      }
      a = npx - inx;
      b = npy - iny;
      iw00 = (int)std::nearbyint((1.f - a) * (1.f - b) * (1 << W_BITS));
      iw01 = (int)std::nearbyint(a * (1.f - b) * (1 << W_BITS));
      iw10 = (int)std::nearbyint((1.f - a) * b * (1 << W_BITS));
      iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
      int64_t ib1 = 0, ib2 = 0;
      for (int y = 0; y < win; ++y)
        for (int x = 0; x < win; ++x) {
          const int X = inx + x, Y = iny + y, k = y * win + x;
          const int diff = descale(pix(Lj, X, Y) * iw00 + pix(Lj, X + 1, Y) * iw01 + pix(Lj, X, Y + 1) * iw10 +
                                       pix(Lj, X + 1, Y + 1) * iw11, W_BITS - 5) - Ip[k];
          ib1 += int64_t(diff) * Dx[k];
          ib2 += int64_t(diff) * Dy[k];
        }
      const float b1 = (float)ib1 * FLT_SCALE, b2 = (float)ib2 * FLT_SCALE;
      const float dx = (float)((A12 * b2 - A22 * b1) * D);
      const float dy = (float)((A12 * b1 - A11 * b2) * D);
      npx += dx;
      npy += dy;
      nx = npx + half;
      ny = npy + half;
      if ((double)dx * dx + (double)dy * dy <= P.eps2) break;
      if (j > 0 && std::fabs(dx + pdx) < 0.01 && std::fabs(dy + pdy) < 0.01) {
        nx -= dx * 0.5f;
        ny -= dy * 0.5f;
        break;
      }
      pdx = dx;
      pdy = dy;
    }
  }
  *out_x = nx;
  *out_y = ny;
}

int klt_levels(int w, int h, int max_level, int win) {
  int l = 0;
  while (l < max_level) {
    w = (w + 1) / 2;
    h = (h + 1) / 2;
    if (w <= win || h <= win) break;
    ++l;
  }
  return l;
}

}  // namespace

extern "C" {

// Building blocks, exposed for the per-stage parity tests.
void oracle_pyr_down(const uint8_t* src, int32_t w, int32_t h, uint8_t* dst) { pyr_down(src, w, h, dst); }
void oracle_scharr(const uint8_t* src, int32_t w, int32_t h, int16_t* dxy) { scharr(src, w, h, dxy); }

// cv::calcOpticalFlowPyrLK (flags 0, no initial flow) as called at
// CTracker.cpp:513: prev_pts/next_pts [n][2] float, status [n].
// eps is the TermCriteria epsilon (squared internally, lkpyramid.cpp).
int oracle_calc_optical_flow_pyr_lk(const uint8_t* prev, const uint8_t* next, int32_t w, int32_t h,
                                    const float* prev_pts, int32_t n, float* next_pts, uint8_t* status, int32_t win,
                                    int32_t max_level, int32_t max_count, double eps, double min_eig) {
  if (w <= 0 || h <= 0 || n < 0 || win < 3 || (win & 1) == 0 || max_level < 0) return -22;
  if (n == 0) return 0;
  const int maxLevel = klt_levels(w, h, max_level, win);
  std::vector<Level> I = build_pyramid(prev, w, h, maxLevel, win, true);
  std::vector<Level> J = build_pyramid(next, w, h, maxLevel, win, false);
  LkParams P{win, maxLevel, std::min(std::max(max_count, 0), 100), 0.0, min_eig};
  const double e = std::min(std::max(eps, 0.), 10.);
  P.eps2 = e * e;
  for (int i = 0; i < n; ++i)
    track_point(I, J, maxLevel, P, prev_pts[2 * i], prev_pts[2 * i + 1], &next_pts[2 * i], &next_pts[2 * i + 1],
                &status[i]);
  return 0;
}

// CTracker::computeOpticalFlow (CTracker.cpp:480-562) after the LK call:
// association of every flowed point with the nearest detected point of the
// current frame (CFrame::findClosestPointIndexDistorted, CFrame.cpp:437-450,
// double distances, first minimum), the gates of CTracker.cpp:525 (float
// squared distances d, e against max/min match distance and the maximum
// distance to a detected feature), and the better-or-equal replacement of
// CTracker.cpp:525-545.  Returns the match count; prev_idx/curr_idx
// capacity >= n.  An empty detected set yields no matches (the reference
// would index position -1).
int32_t oracle_klt_associate(const float* prev_pts, const float* flowed, const uint8_t* status, int32_t n,
                             const double* curr_pts, int32_t m, double max_match_distance,
                             double min_match_distance, double max_org_feat_dist, int32_t* prev_idx,
                             int32_t* curr_idx) {
  if (m <= 0 || n <= 0) return 0;
  const double maxDistSq = max_match_distance * max_match_distance;
  const double maxFeatDistSq = max_org_feat_dist * max_org_feat_dist;
  const double minDistSq = min_match_distance * min_match_distance;
  std::vector<double> matchDistance(m, -1.0);
  std::vector<char> matchStatus(m, 0);
  std::vector<int> matchedIdx(m, -1);
  int matchCount = 0;
  for (int i = 0; i < n; ++i) {
    if (!status[i]) continue;
    const float cx = flowed[2 * i], cy = flowed[2 * i + 1];
    int idx = -1;
    double best = DBL_MAX;
    for (int k = 0; k < m; ++k) {
      const double d = (curr_pts[2 * k] - cx) * (curr_pts[2 * k] - cx) +
                       (curr_pts[2 * k + 1] - cy) * (curr_pts[2 * k + 1] - cy);
      if (d < best) { best = d; idx = k; }
    }
    if (idx < 0) continue;
    const float qx = (float)curr_pts[2 * idx], qy = (float)curr_pts[2 * idx + 1];
    const float e = (cx - qx) * (cx - qx) + (cy - qy) * (cy - qy);
    const float d = (prev_pts[2 * i] - cx) * (prev_pts[2 * i] - cx) + (prev_pts[2 * i + 1] - cy) * (prev_pts[2 * i + 1] - cy);
    if ((d < maxDistSq) && (e < maxFeatDistSq) && (d > minDistSq) &&
        ((matchDistance[idx] >= e) || (matchDistance[idx] == -1))) {
      if (matchStatus[idx]) {
        prev_idx[matchedIdx[idx]] = i;
      } else {
        prev_idx[matchCount] = i;
        curr_idx[matchCount] = idx;
        matchStatus[idx] = 1;
        matchedIdx[idx] = matchCount;
        ++matchCount;
      }
      matchDistance[idx] = e;
    }
  }
  return matchCount;
}

}  // extern "C"
