// BRISK on the device (CTracker::detectFeatures,
// /root/reference/CTracker.cpp:275-287; constructed at :43-45).
//
// The reference links the ethz-asl BRISK 2 library, which is not in the
// tree: what is built is BRISK as published (Leutenegger et al., ICCV 2011)
// in its reference implementation's form (the code OpenCV ships as
// cv::BRISK), restated in oracle/brisk_oracle.py; parity against the
// reference's library is unpinned.
//
// Descriptor: the 60-point pattern (4 rings), 64 scales x 1024 rotations
// generated on the host with the same float / double steps as the
// restatement and uploaded once per device; one wave per keypoint: lane p
// < 60 takes the smoothed intensity of pattern point p (box filter of side
// 2 sigma with fixed-point border weights over the integral image), the
// 870 long pairs give the orientation by exact integer sums, and lane l
// writes descriptor byte l (short pairs 8l .. 8l + 7).  Float work is
// compiled without contraction (-ffp-contract=off), so it is IEEE step for
// step the restatement's.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>
#include "../../include/sfm_amd.h"

void sfm_internal_set_error(const std::string& msg);  // ba_solver.hip

namespace sfm {
namespace {

constexpr int kRot = 1024, kScales = 64, kPts = 60;
constexpr float kScaleRange = 30.0f, kBasicSize = 12.0f;

int bfail(int code, const std::string& m) {
  sfm_internal_set_error("brisk: " + m);
  return code;
}

struct BriskPattern {
  std::vector<float> xy;      // [scales][rot][points][2]
  std::vector<float> sigma;   // [scales][points]
  int size_list[kScales];
  std::vector<int32_t> shortp;  // [n][2]
  std::vector<int32_t> longp;   // [n][4]: i, j, weighted dx, weighted dy
};

// BRISK_Impl::generateKernel with the standard pattern (patternScale 1)
BriskPattern make_pattern() {
  BriskPattern P;
  const double f = 0.85;
  const float r_list[5] = {float(f * 0.0), float(f * 2.9), float(f * 4.9), float(f * 7.4), float(f * 10.8)};
  const int n_list[5] = {1, 10, 14, 15, 20};
  const float d_max = 5.85f, d_min = 8.2f;
  const float lb_scale = float(std::log(double(kScaleRange)) / std::log(2.0));
  const float lb_scale_step = lb_scale / float(kScales);
  const float sigma_scale = 1.3f;
  P.xy.resize(size_t(kScales) * kRot * kPts * 2);
  P.sigma.resize(size_t(kScales) * kPts);
  for (int sc = 0; sc < kScales; ++sc) {
    const float s = float(std::pow(2.0, double(float(sc) * lb_scale_step)));
    P.size_list[sc] = 0;
    for (int rot = 0; rot < kRot; ++rot) {
      const double theta = double(rot) * 2 * M_PI / double(kRot);
      int k = 0;
      for (int ring = 0; ring < 5; ++ring)
        for (int num = 0; num < n_list[ring]; ++num, ++k) {
          const double alpha = double(num) * 2 * M_PI / double(n_list[ring]);
          const float sr = s * r_list[ring];
          float* q = &P.xy[((size_t(sc) * kRot + rot) * kPts + k) * 2];
          q[0] = float(double(sr) * std::cos(alpha + theta));
          q[1] = float(double(sr) * std::sin(alpha + theta));
          float sig;
          if (ring == 0) sig = sigma_scale * s * 0.5f;
          else sig = float(double(sigma_scale * s) * double(r_list[ring]) * std::sin(M_PI / n_list[ring]));
          if (rot == 0) {
            P.sigma[size_t(sc) * kPts + k] = sig;
            const int size = int(std::ceil(double(sr + sig))) + 1;
            P.size_list[sc] = std::max(P.size_list[sc], size);
          }
        }
    }
  }
  const float* p0 = &P.xy[0];
  for (int i = 1; i < kPts; ++i)
    for (int j = 0; j < i; ++j) {
      const float dx = p0[2 * j] - p0[2 * i], dy = p0[2 * j + 1] - p0[2 * i + 1];
      const float nsq = dx * dx + dy * dy;
      if (nsq > d_min * d_min) {
        P.longp.insert(P.longp.end(), {i, j, int(double(dx / nsq) * 2048.0 + 0.5), int(double(dy / nsq) * 2048.0 + 0.5)});
      } else if (nsq < d_max * d_max) {
        P.shortp.insert(P.shortp.end(), {i, j});
      }
    }
  return P;
}

struct DevPattern {
  float2* xy = nullptr;
  float* sigma = nullptr;
  int32_t* size_list = nullptr;
  int4* longp = nullptr;
  int2* shortp = nullptr;
  int n_long = 0, n_short = 0;
};

// one copy per device, built on first use
DevPattern* device_pattern(int device, int* rc) {
  static std::mutex mu;
  static std::vector<DevPattern*> per_dev(64, nullptr);
  std::lock_guard<std::mutex> lock(mu);
  if (device < 0 || device >= 64) { *rc = bfail(SFM_ENODEV, "device index"); return nullptr; }
  if (per_dev[device]) return per_dev[device];
  static BriskPattern host = make_pattern();
  auto* d = new DevPattern;
  d->n_long = int(host.longp.size() / 4);
  d->n_short = int(host.shortp.size() / 2);
  bool ok = hipMalloc(&d->xy, host.xy.size() * sizeof(float)) == hipSuccess &&
            hipMalloc(&d->sigma, host.sigma.size() * sizeof(float)) == hipSuccess &&
            hipMalloc(&d->size_list, sizeof(int32_t) * kScales) == hipSuccess &&
            hipMalloc(&d->longp, host.longp.size() * sizeof(int32_t)) == hipSuccess &&
            hipMalloc(&d->shortp, host.shortp.size() * sizeof(int32_t)) == hipSuccess;
  ok = ok && hipMemcpy(d->xy, host.xy.data(), host.xy.size() * sizeof(float), hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(d->sigma, host.sigma.data(), host.sigma.size() * sizeof(float), hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(d->size_list, host.size_list, sizeof(int32_t) * kScales, hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(d->longp, host.longp.data(), host.longp.size() * sizeof(int32_t), hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(d->shortp, host.shortp.data(), host.shortp.size() * sizeof(int32_t), hipMemcpyHostToDevice) == hipSuccess;
  if (!ok) { *rc = bfail(SFM_ENOMEM, "pattern upload failed"); return nullptr; }
  per_dev[device] = d;
  return d;
}

// integral image [h+1][w+1] (int32: 255 * 1280 * 720 < 2^31)
__global__ void k_integral_rows(const uint8_t* __restrict__ img, int w, int h, int32_t* __restrict__ ii) {
  const int y = blockIdx.x * blockDim.x + threadIdx.x;
  if (y > h) return;
  int32_t* row = ii + size_t(y) * (w + 1);
  row[0] = 0;
  int32_t s = 0;
  if (y == 0) {
    for (int x = 0; x < w; ++x) row[x + 1] = 0;
    return;
  }
  const uint8_t* src = img + size_t(y - 1) * w;
  for (int x = 0; x < w; ++x) {
    s += src[x];
    row[x + 1] = s;
  }
}
__global__ void k_integral_cols(int w, int h, int32_t* __restrict__ ii) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x > w) return;
  int32_t s = 0;
  for (int y = 1; y <= h; ++y) {
    s += ii[size_t(y) * (w + 1) + x];
    ii[size_t(y) * (w + 1) + x] = s;
  }
}

// BRISK_Impl::smoothedIntensity for one pattern point
__device__ int smoothed(const uint8_t* __restrict__ img, const int32_t* __restrict__ ii, int cols, float key_x,
                        float key_y, float px, float py, float sigma_half) {
  const float xf = px + key_x, yf = py + key_y;
  const int x = int(xf), y = int(yf);
  const float area = 4.0f * sigma_half * sigma_half;
  if (sigma_half < 0.5f) {
    const int r_x = int((xf - float(x)) * 1024), r_y = int((yf - float(y)) * 1024);
    const int r_x_1 = 1024 - r_x, r_y_1 = 1024 - r_y;
    const uint8_t* p = img + size_t(y) * cols + x;
    const int v = r_x_1 * r_y_1 * int(p[0]) + r_x * r_y_1 * int(p[1]) + r_x * r_y * int(p[cols + 1]) +
                  r_x_1 * r_y * int(p[cols]);
    return (v + 512) / 1024;
  }
  const int scaling = int(4194304.0 / double(area));
  const int scaling2 = int(double(float(scaling) * area) / 1024.0);
  const float x_1 = xf - sigma_half, x1 = xf + sigma_half, y_1 = yf - sigma_half, y1 = yf + sigma_half;
  const int x_left = int(x_1 + 0.5f), y_top = int(y_1 + 0.5f), x_right = int(x1 + 0.5f), y_bottom = int(y1 + 0.5f);
  const float r_x_1 = float(x_left) - x_1 + 0.5f, r_y_1 = float(y_top) - y_1 + 0.5f;
  const float r_x1 = x1 - float(x_right) + 0.5f, r_y1 = y1 - float(y_bottom) + 0.5f;
  const int dx = x_right - x_left - 1, dy = y_bottom - y_top - 1;
  const int A = int((r_x_1 * r_y_1) * float(scaling)), B = int((r_x1 * r_y_1) * float(scaling));
  const int C = int((r_x1 * r_y1) * float(scaling)), D = int((r_x_1 * r_y1) * float(scaling));
  const int r_x_1_i = int(r_x_1 * float(scaling)), r_y_1_i = int(r_y_1 * float(scaling));
  const int r_x1_i = int(r_x1 * float(scaling)), r_y1_i = int(r_y1 * float(scaling));
  const uint8_t* p = img + size_t(y_top) * cols + x_left;
  int v = A * int(p[0]) + B * int(p[dx + 1]) + C * int(p[size_t(dy + 1) * cols + dx + 1]) +
          D * int(p[size_t(dy + 1) * cols]);
  if (dx + dy > 2) {
    const int ic = cols + 1;
    auto S = [&](int r0, int r1, int c0, int c1) {
      return ii[size_t(r1) * ic + c1] - ii[size_t(r0) * ic + c1] - ii[size_t(r1) * ic + c0] + ii[size_t(r0) * ic + c0];
    };
    const int xl = x_left, yt = y_top;
    const int upper = S(yt, yt + 1, xl + 1, xl + 1 + dx) * r_y_1_i;
    const int middle = S(yt + 1, yt + 1 + dy, xl + 1, xl + 1 + dx) * scaling;
    const int left = S(yt + 1, yt + 1 + dy, xl, xl + 1) * r_x_1_i;
    const int right = S(yt + 1, yt + 1 + dy, xl + dx + 1, xl + dx + 2) * r_x1_i;
    const int bottom = S(yt + dy + 1, yt + dy + 2, xl + 1, xl + 1 + dx) * r_y1_i;
    return (v + upper + middle + left + right + bottom + scaling2 / 2) / scaling2;
  }
  for (int c = 1; c <= dx; ++c) v += r_y_1_i * int(p[c]) + r_y1_i * int(p[size_t(dy + 1) * cols + c]);
  for (int r = 1; r <= dy; ++r) {
    const uint8_t* q = p + size_t(r) * cols;
    v += r_x_1_i * int(q[0]) + r_x1_i * int(q[dx + 1]);
    for (int c = 1; c <= dx; ++c) v += int(q[c]) * scaling;
  }
  return (v + scaling2 / 2) / scaling2;
}

__device__ __forceinline__ int wave_isum(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// one wave per keypoint
__global__ __launch_bounds__(64) void k_brisk_describe(const uint8_t* __restrict__ img, int w, int h,
                                                       const int32_t* __restrict__ ii, DevPattern P,
                                                       const float* __restrict__ kps, int n,
                                                       int32_t* __restrict__ keep, float* __restrict__ angle_out,
                                                       uint8_t* __restrict__ desc) {
  __shared__ int vals[kPts];
  const int i = blockIdx.x, l = threadIdx.x;
  if (i >= n) return;
  const float x = kps[3 * i], y = kps[3 * i + 1], size = kps[3 * i + 2];
  // scale index (computeDescriptorsAndOrOrientation)
  const float ln2 = 0.693147180559945f;
  const float lb_scalerange = float(log(double(kScaleRange)) / double(ln2));
  const float basic06 = kBasicSize * 0.6f;
  const float lg = float(log(double(size / basic06))) / ln2;
  int sc = int(double(float(kScales) / lb_scalerange * lg) + 0.5);
  sc = sc < 0 ? 0 : sc;
  if (sc >= kScales) sc = kScales - 1;
  const int border = P.size_list[sc];
  if (x < float(border) || x >= float(w - border) || y < float(border) || y >= float(h - border)) {
    if (l == 0) keep[i] = 0;
    return;
  }
  if (l < kPts) {
    const float2 q = P.xy[(size_t(sc) * kRot) * kPts + l];
    vals[l] = smoothed(img, ii, w, x, y, q.x, q.y, P.sigma[sc * kPts + l]);
  }
  __syncthreads();
  int d0 = 0, d1 = 0;
  for (int k = l; k < P.n_long; k += 64) {
    const int4 lp = P.longp[k];
    const int dt = vals[lp.x] - vals[lp.y];
    d0 += dt * lp.z / 1024;
    d1 += dt * lp.w / 1024;
  }
  d0 = wave_isum(d0);
  d1 = wave_isum(d1);
  float ang = float(atan2(double(float(d1)), double(float(d0))) / M_PI * 180.0);
  int theta = int(double(kRot) * (double(ang) / 360.0) + 0.5);
  if (theta < 0) theta += kRot;
  if (theta >= kRot) theta -= kRot;
  if (ang < 0) ang += 360.0f;
  __syncthreads();
  if (l < kPts) {
    const float2 q = P.xy[(size_t(sc) * kRot + theta) * kPts + l];
    vals[l] = smoothed(img, ii, w, x, y, q.x, q.y, P.sigma[sc * kPts + l]);
  }
  __syncthreads();
  // byte l: short pairs 8 l .. 8 l + 7 (bit b of the descriptor's b / 32-th
  // little-endian word, as the reference's UINT32 writes)
  unsigned byte = 0;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const int k = 8 * l + b;
    if (k < P.n_short) {
      const int2 sp = P.shortp[k];
      byte |= unsigned(vals[sp.x] > vals[sp.y]) << b;
    }
  }
  const int n_bytes = ((P.n_short + 127) / 128) * 16;
  if (l < n_bytes) desc[size_t(i) * n_bytes + l] = uint8_t(byte);
  if (l == 0) {
    keep[i] = 1;
    angle_out[i] = ang;
  }
}

// ---------------------------------------------------------------------------
// Detector (BriskScaleSpace): layers c_i / d_i, FAST 9-16 scores, 2-D
// maxima with isMax2D's tie-break, the scale test against the adjacent
// layers, subpixel2D (see oracle/brisk_oracle.py for the simplifications).
constexpr int kMaxLayers = 16;
__constant__ int2 kCircle[16] = {{0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
                                 {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

struct Layer {
  const uint8_t* img;
  const uint8_t* R;  // scores (cornerScore when >= 1, else 0)
  int w, h;
  float scale, offset;
};
struct Layers {
  Layer l[kMaxLayers];
  int n;
};

__global__ void k_halfsample(const uint8_t* __restrict__ src, int sw, uint8_t* __restrict__ dst, int dw, int dh) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= dw || y >= dh) return;
  const uint8_t* a = src + size_t(2 * y) * sw + 2 * x;
  dst[size_t(y) * dw + x] = uint8_t((int(a[0]) + a[1] + a[sw] + a[sw + 1] + 2) >> 2);
}
__global__ void k_twothirdsample(const uint8_t* __restrict__ src, int sw, uint8_t* __restrict__ dst, int dw, int dh) {
  const int bx = blockIdx.x * blockDim.x + threadIdx.x, by = blockIdx.y;  // 3x3 block -> 2x2
  if (2 * bx >= dw || 2 * by >= dh) return;
  const uint8_t* a = src + size_t(3 * by) * sw + 3 * bx;
  const int p00 = a[0], p01 = a[1], p02 = a[2], p10 = a[sw], p11 = a[sw + 1], p12 = a[sw + 2];
  const int p20 = a[2 * sw], p21 = a[2 * sw + 1], p22 = a[2 * sw + 2];
  uint8_t* o = dst + size_t(2 * by) * dw + 2 * bx;
  o[0] = uint8_t((4 * p00 + 2 * p01 + 2 * p10 + p11 + 4) / 9);
  o[1] = uint8_t((4 * p02 + 2 * p01 + 2 * p12 + p11 + 4) / 9);
  o[dw] = uint8_t((4 * p20 + 2 * p10 + 2 * p21 + p11 + 4) / 9);
  o[dw + 1] = uint8_t((4 * p22 + 2 * p12 + 2 * p21 + p11 + 4) / 9);
}

// cornerScore<16>(p, 0) = max(0, darkest / brightest 9-arc contrast) - 1,
// kept when >= 1 (getAgastScore(x, y, 1)); 0 within 3 pixels of the border
__global__ void k_fast_score(const uint8_t* __restrict__ img, int w, int h, uint8_t* __restrict__ R) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w || y >= h) return;
  int out = 0;
  if (x >= 3 && y >= 3 && x < w - 3 && y < h - 3) {
    const int v = img[size_t(y) * w + x];
    int d[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = v - int(img[size_t(y + kCircle[k].y) * w + x + kCircle[k].x]);
    int dark = -1000000, bright = -1000000;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      int mn = 1000000, mx = -1000000;
#pragma unroll
      for (int m = 0; m < 9; ++m) {
        mn = min(mn, d[(s + m) & 15]);
        mx = max(mx, d[(s + m) & 15]);
      }
      dark = max(dark, mn);
      bright = max(bright, -mx);
    }
    const int sc = max(max(dark, bright), 0) - 1;
    out = sc >= 1 ? sc : 0;
  }
  R[size_t(y) * w + x] = uint8_t(out);
}

__device__ __forceinline__ int s_at(const Layer& L, int x, int y, int thr) {
  if (x < 0 || y < 0 || x >= L.w || y >= L.h) return 0;
  const int r = L.R[size_t(y) * L.w + x];
  return r >= thr ? r : 0;
}

// BriskScaleSpace::subpixel2D (float step for step; the reference's
// delta_y = delta_x1 / _x2 in the clamped branch kept)
__device__ float subpixel2d(const int s[3][3], float& dx_out, float& dy_out) {
  const int s_0_0 = s[0][0], s_0_1 = s[0][1], s_0_2 = s[0][2], s_1_0 = s[1][0], s_1_1 = s[1][1], s_1_2 = s[1][2];
  const int s_2_0 = s[2][0], s_2_1 = s[2][1], s_2_2 = s[2][2];
  const int tmp1 = s_0_0 + s_0_2 - 2 * s_1_1 + s_2_0 + s_2_2;
  const int coeff1 = 3 * (tmp1 + s_0_1 - ((s_1_0 + s_1_2) << 1) + s_2_1);
  const int coeff2 = 3 * (tmp1 - ((s_0_1 + s_2_1) << 1) + s_1_0 + s_1_2);
  const int tmp2 = s_0_2 - s_2_0;
  const int tmp3 = s_0_0 + tmp2 - s_2_2;
  const int tmp4 = tmp3 - 2 * tmp2;
  const int coeff3 = -3 * (tmp3 + s_0_1 - s_2_1);
  const int coeff4 = -3 * (tmp4 + s_1_0 - s_1_2);
  const int coeff5 = (s_0_0 - s_0_2 - s_2_0 + s_2_2) << 2;
  const int coeff6 = -((s_0_0 + s_0_2 - ((s_1_0 + s_0_1 + s_1_2 + s_2_1) << 1) - 5 * s_1_1 + s_2_0 + s_2_2) << 1);
  const int H_det = 4 * coeff1 * coeff2 - coeff5 * coeff5;
  auto quad = [&](float dx, float dy) {
    return (coeff1 * dx * dx + coeff2 * dy * dy + coeff3 * dx + coeff4 * dy + coeff5 * dx * dy + coeff6) / 18.0f;
  };
  if (H_det == 0) {
    dx_out = 0.0f;
    dy_out = 0.0f;
    return float(coeff6) / 18.0f;
  }
  if (!(H_det > 0 && coeff1 < 0)) {
    int tmp_max = coeff3 + coeff4 + coeff5;
    float dx = 1.0f, dy = 1.0f;
    int t = -coeff3 + coeff4 - coeff5;
    if (t > tmp_max) { tmp_max = t; dx = -1.0f; dy = 1.0f; }
    t = coeff3 - coeff4 - coeff5;
    if (t > tmp_max) { tmp_max = t; dx = 1.0f; dy = -1.0f; }
    t = -coeff3 - coeff4 + coeff5;
    if (t > tmp_max) { tmp_max = t; dx = -1.0f; dy = -1.0f; }
    dx_out = dx;
    dy_out = dy;
    return float(tmp_max + coeff1 + coeff2 + coeff6) / 18.0f;
  }
  float dx = float(2 * coeff2 * coeff3 - coeff4 * coeff5) / float(-H_det);
  float dy = float(2 * coeff1 * coeff4 - coeff3 * coeff5) / float(-H_det);
  bool tx = false, tx_ = false, ty = false, ty_ = false;
  if (dx > 1.0f) tx = true;
  else if (dx < -1.0f) tx_ = true;
  if (dy > 1.0f) ty = true;
  if (dy < -1.0f) ty_ = true;
  if (tx || tx_ || ty || ty_) {
    float dx1 = 0.0f, dx2 = 0.0f, dy1 = 0.0f, dy2 = 0.0f;
    if (tx) {
      dx1 = 1.0f;
      dy1 = -float(coeff4 + coeff5) / float(2 * coeff2);
    } else if (tx_) {
      dx1 = -1.0f;
      dy1 = -float(coeff4 - coeff5) / float(2 * coeff2);
    }
    dy1 = fminf(fmaxf(dy1, -1.0f), 1.0f);
    if (ty) {
      dy2 = 1.0f;
      dx2 = -float(coeff3 + coeff5) / float(2 * coeff1);
    } else if (ty_) {
      dy2 = -1.0f;
      dx2 = -float(coeff3 - coeff5) / float(2 * coeff1);
    }
    dx2 = fminf(fmaxf(dx2, -1.0f), 1.0f);
    const float m1 = quad(dx1, dy1), m2 = quad(dx2, dy2);
    if (m1 > m2) {
      dx_out = dx1;
      dy_out = dx1;
      return m1;
    }
    dx_out = dx2;
    dy_out = dx2;
    return m2;
  }
  dx_out = dx;
  dy_out = dy;
  return quad(dx, dy);
}

struct Cand {
  unsigned long long key;  // layer << 42 | y << 21 | x: BRISK's emission order
  float x, y, size, response;
  int layer, pad;
};

__global__ void k_detect_layer(Layers LS, int i, int thr, Cand* __restrict__ out, int cap, int* __restrict__ count) {
  const Layer& L = LS.l[i];
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= L.w || y >= L.h) return;
  const int c = s_at(L, x, y, thr);
  if (c == 0) return;
  // isMax2D
  int eq = 0;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) {
      if (!dx && !dy) continue;
      const int v = s_at(L, x + dx, y + dy, thr);
      if (v > c) return;
      if (v == c) eq |= 1 << ((dy + 1) * 3 + dx + 1);
    }
  if (eq) {
    auto smooth = [&](int cx, int cy) {
      return s_at(L, cx - 1, cy - 1, thr) + 2 * s_at(L, cx, cy - 1, thr) + s_at(L, cx + 1, cy - 1, thr) +
             2 * s_at(L, cx - 1, cy, thr) + 4 * s_at(L, cx, cy, thr) + 2 * s_at(L, cx + 1, cy, thr) +
             s_at(L, cx - 1, cy + 1, thr) + 2 * s_at(L, cx, cy + 1, thr) + s_at(L, cx + 1, cy + 1, thr);
    };
    const int sc = smooth(x, y);
    for (int b = 0; b < 9; ++b)
      if ((eq >> b) & 1)
        if (smooth(x + b % 3 - 1, y + b / 3 - 1) > sc) return;
  }
  // scale test against the adjacent layers (nearest sample, 3x3 max)
  for (int j = i - 1; j <= i + 1; j += 2) {
    if (j < 0 || j >= LS.n) continue;
    const Layer& M = LS.l[j];
    const float X = float(x) * L.scale + L.offset, Y = float(y) * L.scale + L.offset;
    const int xj = int((X - M.offset) / M.scale + 0.5f), yj = int((Y - M.offset) / M.scale + 0.5f);
    const int x0 = max(xj - 1, 0), x1 = min(xj + 1, M.w - 1), y0 = max(yj - 1, 0), y1 = min(yj + 1, M.h - 1);
    for (int yy = y0; yy <= y1; ++yy)
      for (int xx = x0; xx <= x1; ++xx)
        if (s_at(M, xx, yy, thr) > c) return;
  }
  int s3[3][3];  // s_i_j of subpixel2D: the score at (x + i - 1, y + j - 1)
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int q = 0; q < 3; ++q) s3[q][r] = L.R[size_t(y - 1 + r) * L.w + x - 1 + q];
  float ddx, ddy;
  const float mx = subpixel2d(s3, ddx, ddy);
  const int k = atomicAdd(count, 1);
  if (k >= cap) return;
  Cand cd;
  cd.key = (static_cast<unsigned long long>(i) << 42) | (static_cast<unsigned long long>(y) << 21) |
           static_cast<unsigned long long>(x);
  cd.x = (float(x) + ddx) * L.scale + L.offset;
  cd.y = (float(y) + ddy) * L.scale + L.offset;
  cd.size = kBasicSize * L.scale;
  cd.response = mx;
  cd.layer = i;
  cd.pad = 0;
  out[k] = cd;
}

__global__ void k_gather_cands(const Cand* __restrict__ c, const int32_t* __restrict__ order, int n,
                               float* __restrict__ kps3, float* __restrict__ resp, int32_t* __restrict__ layer) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const Cand& q = c[order[k]];
  kps3[3 * k] = q.x;
  kps3[3 * k + 1] = q.y;
  kps3[3 * k + 2] = q.size;
  resp[k] = q.response;
  layer[k] = q.layer;
}
__global__ void k_cand_keys(const Cand* __restrict__ c, int n, unsigned long long* __restrict__ key,
                            int32_t* __restrict__ idx) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  key[k] = c[k].key;
  idx[k] = k;
}

// grow-only per-device workspace of the detector (one frame per call)
struct BriskWork {
  std::vector<std::pair<void*, size_t>> buf;
  void* get(int slot, size_t bytes, int* rc) {
    if (int(buf.size()) <= slot) buf.resize(slot + 1, {nullptr, 0});
    auto& e = buf[slot];
    if (e.second < bytes) {
      if (e.first) (void)hipFree(e.first);
      e = {nullptr, 0};
      if (hipMalloc(&e.first, std::max<size_t>(bytes, 256)) != hipSuccess) {
        *rc = bfail(SFM_ENOMEM, "hipMalloc failed (detector workspace)");
        return nullptr;
      }
      e.second = std::max<size_t>(bytes, 256);
    }
    return e.first;
  }
};
BriskWork* work_for(int device) {
  static std::vector<BriskWork*> w(64, nullptr);
  if (!w[device]) w[device] = new BriskWork;
  return w[device];
}
std::mutex& work_mutex() {
  static std::mutex m;
  return m;
}

}  // namespace
}  // namespace sfm

using namespace sfm;

extern "C" int sfm_brisk_describe(int32_t device, const uint8_t* img, int32_t w, int32_t h, const float* kps,
                                  int32_t n, int32_t* kept, float* angle, uint8_t* desc, int32_t* n_kept) {
  if (!n_kept) return bfail(SFM_EINVAL, "n_kept is NULL");
  *n_kept = 0;
  if (w <= 0 || h <= 0 || n < 0) return bfail(SFM_EINVAL, "bad sizes");
  if (!img || (n && (!kps || !kept || !angle || !desc))) return bfail(SFM_EINVAL, "NULL argument");
  if (hipSetDevice(device) != hipSuccess) return bfail(SFM_ENODEV, "hipSetDevice failed");
  for (int32_t i = 0; i < n; ++i)
    if (!std::isfinite(kps[3 * i]) || !std::isfinite(kps[3 * i + 1]) || !(kps[3 * i + 2] > 0.0f))
      return bfail(SFM_EINVAL, "keypoint " + std::to_string(i) + ": non-finite position or size <= 0");
  if (n == 0) return 0;
  int rc = 0;
  DevPattern* P = device_pattern(device, &rc);
  if (!P) return rc;
  const size_t npx = size_t(w) * h, nii = size_t(w + 1) * (h + 1);
  uint8_t *d_img = nullptr, *d_desc = nullptr;
  int32_t *d_ii = nullptr, *d_keep = nullptr;
  float *d_kps = nullptr, *d_ang = nullptr;
  const int n_bytes = ((P->n_short + 127) / 128) * 16;
  bool ok = hipMalloc(&d_img, npx) == hipSuccess && hipMalloc(&d_ii, nii * 4) == hipSuccess &&
            hipMalloc(&d_kps, size_t(n) * 12) == hipSuccess && hipMalloc(&d_keep, size_t(n) * 4) == hipSuccess &&
            hipMalloc(&d_ang, size_t(n) * 4) == hipSuccess && hipMalloc(&d_desc, size_t(n) * n_bytes) == hipSuccess;
  if (ok) {
    ok = hipMemcpy(d_img, img, npx, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(d_kps, kps, size_t(n) * 12, hipMemcpyHostToDevice) == hipSuccess;
    k_integral_rows<<<(h + 1 + 255) / 256, 256>>>(d_img, w, h, d_ii);
    k_integral_cols<<<(w + 1 + 255) / 256, 256>>>(w, h, d_ii);
    k_brisk_describe<<<n, 64>>>(d_img, w, h, d_ii, *P, d_kps, n, d_keep, d_ang, d_desc);
    std::vector<int32_t> kp(n);
    std::vector<float> an(n);
    std::vector<uint8_t> de(size_t(n) * n_bytes);
    ok = ok && hipDeviceSynchronize() == hipSuccess &&
         hipMemcpy(kp.data(), d_keep, size_t(n) * 4, hipMemcpyDeviceToHost) == hipSuccess &&
         hipMemcpy(an.data(), d_ang, size_t(n) * 4, hipMemcpyDeviceToHost) == hipSuccess &&
         hipMemcpy(de.data(), d_desc, de.size(), hipMemcpyDeviceToHost) == hipSuccess;
    if (ok) {
      int m = 0;
      for (int32_t i = 0; i < n; ++i)
        if (kp[i]) {
          kept[m] = i;
          angle[m] = an[i];
          std::memcpy(desc + size_t(m) * n_bytes, de.data() + size_t(i) * n_bytes, n_bytes);
          ++m;
        }
      *n_kept = m;
    }
  }
  for (void* p : {(void*)d_img, (void*)d_ii, (void*)d_kps, (void*)d_keep, (void*)d_ang, (void*)d_desc})
    if (p) (void)hipFree(p);
  return ok ? 0 : bfail(SFM_EIO, "allocation, kernel or copy failed");
}

extern "C" int sfm_brisk_detect_describe(int32_t device, const uint8_t* img, int32_t w, int32_t h, int32_t threshold,
                                         int32_t octaves, int32_t capacity, float* kps, int32_t* octave,
                                         uint8_t* desc, int32_t* n_out) {
  if (!n_out) return bfail(SFM_EINVAL, "n_out is NULL");
  *n_out = 0;
  if (w < 8 || h < 8 || threshold < 1 || threshold > 255 || octaves < 0 || 2 * octaves > kMaxLayers || capacity < 0)
    return bfail(SFM_EINVAL, "bad sizes (w, h >= 8; threshold 1..255; octaves 0..8)");
  if (!img || (capacity && (!kps || !octave))) return bfail(SFM_EINVAL, "NULL argument");
  if (hipSetDevice(device) != hipSuccess) return bfail(SFM_ENODEV, "hipSetDevice failed");
  int rc = 0;
  DevPattern* P = nullptr;
  if (desc && !(P = device_pattern(device, &rc))) return rc;
  std::lock_guard<std::mutex> lock(work_mutex());
  BriskWork* W = work_for(device);
  // layer geometry (BriskScaleSpace::constructPyramid)
  const int nl = std::max(1, 2 * octaves);
  int lw[kMaxLayers], lh[kMaxLayers];
  float lsc[kMaxLayers], loff[kMaxLayers];
  size_t loff_px[kMaxLayers + 1];
  lw[0] = w; lh[0] = h; lsc[0] = 1.0f; loff[0] = 0.0f;
  int nuse = 1;
  for (int i = 1; i < nl; ++i) {
    if (i == 1) { lw[1] = 2 * (w / 3); lh[1] = 2 * (h / 3); lsc[1] = 1.5f; }
    else { lw[i] = lw[i - 2] / 2; lh[i] = lh[i - 2] / 2; lsc[i] = lsc[i - 2] * 2.0f; }
    loff[i] = 0.5f * lsc[i] - 0.5f;
    nuse = i + 1;
  }
  loff_px[0] = 0;
  for (int i = 0; i < nuse; ++i) loff_px[i + 1] = loff_px[i] + size_t(lw[i]) * lh[i];
  const size_t total = loff_px[nuse];
  auto* limg = static_cast<uint8_t*>(W->get(0, total, &rc));
  auto* lR = static_cast<uint8_t*>(W->get(1, total, &rc));
  const int cap_c = int(std::min<size_t>(size_t(w) * h / 4 + 1024, size_t(1) << 22));
  auto* cand = static_cast<Cand*>(W->get(2, sizeof(Cand) * size_t(cap_c), &rc));
  auto* cnt = static_cast<int32_t*>(W->get(3, sizeof(int32_t), &rc));
  if (rc) return rc;
  if (hipMemcpy(limg, img, size_t(w) * h, hipMemcpyHostToDevice) != hipSuccess) return bfail(SFM_EIO, "upload failed");
  for (int i = 1; i < nuse; ++i) {
    if (lw[i] < 1 || lh[i] < 1) continue;
    if (i == 1) {
      dim3 g(unsigned((lw[1] / 2 + 127) / 128), unsigned(lh[1] / 2));
      k_twothirdsample<<<g, 128>>>(limg, w, limg + loff_px[1], lw[1], lh[1]);
    } else {
      dim3 g(unsigned((lw[i] + 255) / 256), unsigned(lh[i]));
      k_halfsample<<<g, 256>>>(limg + loff_px[i - 2], lw[i - 2], limg + loff_px[i], lw[i], lh[i]);
    }
  }
  Layers LS;
  LS.n = nuse;
  for (int i = 0; i < nuse; ++i) {
    if (lw[i] >= 1 && lh[i] >= 1) {
      dim3 g(unsigned((lw[i] + 255) / 256), unsigned(lh[i]));
      k_fast_score<<<g, 256>>>(limg + loff_px[i], lw[i], lh[i], lR + loff_px[i]);
    }
    LS.l[i] = Layer{limg + loff_px[i], lR + loff_px[i], lw[i], lh[i], lsc[i], loff[i]};
  }
  (void)hipMemset(cnt, 0, sizeof(int32_t));
  for (int i = 0; i < nuse; ++i) {
    if (lw[i] < 1 || lh[i] < 1) continue;
    dim3 g(unsigned((lw[i] + 255) / 256), unsigned(lh[i]));
    k_detect_layer<<<g, 256>>>(LS, i, threshold, cand, cap_c, cnt);
  }
  int32_t n = 0;
  if (hipMemcpy(&n, cnt, sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess) return bfail(SFM_EIO, "kernel failed");
  if (n > cap_c) return bfail(SFM_EIO, "candidate buffer overflow");
  if (n == 0) return 0;
  // BRISK's order: layer, then row-major (stable radix sort on the key)
  auto* key = static_cast<unsigned long long*>(W->get(4, sizeof(unsigned long long) * 2 * size_t(n), &rc));
  auto* idx = static_cast<int32_t*>(W->get(5, sizeof(int32_t) * 2 * size_t(n), &rc));
  auto* kp3 = static_cast<float*>(W->get(6, sizeof(float) * 3 * size_t(n), &rc));
  auto* resp = static_cast<float*>(W->get(7, sizeof(float) * size_t(n), &rc));
  auto* lay = static_cast<int32_t*>(W->get(8, sizeof(int32_t) * size_t(n), &rc));
  if (rc) return rc;
  k_cand_keys<<<(n + 255) / 256, 256>>>(cand, n, key, idx);
  size_t tb = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key, key + n, idx, idx + n, n, 0, 46);
  void* tmp = W->get(9, tb, &rc);
  if (rc) return rc;
  if (hipcub::DeviceRadixSort::SortPairs(tmp, tb, key, key + n, idx, idx + n, n, 0, 46) != hipSuccess)
    return bfail(SFM_EIO, "sort failed");
  k_gather_cands<<<(n + 255) / 256, 256>>>(cand, idx + n, n, kp3, resp, lay);
  std::vector<float> hk(3 * size_t(n)), hr(n);
  std::vector<int32_t> hl(n), hkeep(n, 1);
  std::vector<float> hang(n, -1.0f);
  std::vector<uint8_t> hd;
  if (desc) {
    const int n_bytes = ((P->n_short + 127) / 128) * 16;
    auto* keep = static_cast<int32_t*>(W->get(10, sizeof(int32_t) * size_t(n), &rc));
    auto* ang = static_cast<float*>(W->get(11, sizeof(float) * size_t(n), &rc));
    auto* ii = static_cast<int32_t*>(W->get(12, sizeof(int32_t) * size_t(w + 1) * (h + 1), &rc));
    auto* dd = static_cast<uint8_t*>(W->get(13, size_t(n) * n_bytes, &rc));
    if (rc) return rc;
    k_integral_rows<<<(h + 1 + 255) / 256, 256>>>(limg, w, h, ii);
    k_integral_cols<<<(w + 1 + 255) / 256, 256>>>(w, h, ii);
    k_brisk_describe<<<n, 64>>>(limg, w, h, ii, *P, kp3, n, keep, ang, dd);
    hd.resize(size_t(n) * n_bytes);
    if (hipMemcpy(hkeep.data(), keep, sizeof(int32_t) * n, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(hang.data(), ang, sizeof(float) * n, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(hd.data(), dd, hd.size(), hipMemcpyDeviceToHost) != hipSuccess)
      return bfail(SFM_EIO, "download failed");
  }
  if (hipMemcpy(hk.data(), kp3, sizeof(float) * 3 * n, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(hr.data(), resp, sizeof(float) * n, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(hl.data(), lay, sizeof(int32_t) * n, hipMemcpyDeviceToHost) != hipSuccess)
    return bfail(SFM_EIO, "download failed");
  int m = 0;
  for (int k = 0; k < n; ++k) {
    if (!hkeep[k]) continue;
    if (m < capacity) {
      float* o = kps + 5 * size_t(m);
      o[0] = hk[3 * k]; o[1] = hk[3 * k + 1]; o[2] = hk[3 * k + 2]; o[3] = hang[k]; o[4] = hr[k];
      octave[m] = hl[k];
      if (desc) std::memcpy(desc + size_t(m) * 64, hd.data() + size_t(k) * 64, 64);
    }
    ++m;
  }
  *n_out = m;
  if (m > capacity) return bfail(SFM_EINVAL, "capacity " + std::to_string(capacity) + " < " + std::to_string(m));
  return 0;
}
