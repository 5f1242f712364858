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
#include "sfm_trace.h"
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

// integral image [h+1][w+1] (int32: 255 * 1280 * 720 < 2^31), exact
// integer sums in three passes: (1) one workgroup per row, the row's prefix
// sums (each thread a contiguous segment, a block scan of the segment
// totals); (2) per column, the sums of bands of kIIBand rows; (3) per
// (band, column), the previous bands' totals plus a running sum down the
// band, in place.
constexpr int kIIBand = 32;
__global__ __launch_bounds__(256) void k_integral_rows(const uint8_t* __restrict__ img, int w, int h,
                                                       int32_t* __restrict__ ii) {
  __shared__ int32_t sc[256];
  const int y = blockIdx.x, t = threadIdx.x;
  int32_t* row = ii + size_t(y) * (w + 1);
  const int per = (w + 255) / 256;
  const int x0 = min(w, t * per), x1 = min(w, x0 + per);
  if (y == 0) {
    for (int x = t; x <= w; x += 256) row[x] = 0;
    return;
  }
  const uint8_t* src = img + size_t(y - 1) * w;
  int32_t tot = 0;
  for (int x = x0; x < x1; ++x) tot += src[x];
  sc[t] = tot;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const int32_t v = t >= o ? sc[t - o] : 0;
    __syncthreads();
    sc[t] += v;
    __syncthreads();
  }
  int32_t s = sc[t] - tot;  // exclusive prefix of the segments before this one
  if (t == 0) row[0] = 0;
  for (int x = x0; x < x1; ++x) {
    s += src[x];
    row[x + 1] = s;
  }
}
__global__ __launch_bounds__(256) void k_integral_bandsum(int w, int h, const int32_t* __restrict__ ii,
                                                          int32_t* __restrict__ band) {
  const int x = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (x > w) return;
  const int y0 = 1 + b * kIIBand, y1 = min(h, y0 + kIIBand - 1);
  int32_t s = 0;
  for (int y = y0; y <= y1; ++y) s += ii[size_t(y) * (w + 1) + x];
  band[size_t(b) * (w + 1) + x] = s;
}
__global__ __launch_bounds__(256) void k_integral_cols(int w, int h, const int32_t* __restrict__ band,
                                                       int32_t* __restrict__ ii) {
  const int x = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (x > w) return;
  int32_t s = 0;
  for (int q = 0; q < b; ++q) s += band[size_t(q) * (w + 1) + x];
  const int y0 = 1 + b * kIIBand, y1 = min(h, y0 + kIIBand - 1);
  for (int y = y0; y <= y1; ++y) {
    s += ii[size_t(y) * (w + 1) + x];
    ii[size_t(y) * (w + 1) + x] = s;
  }
}
// the three passes; band: ceil(h / kIIBand) x (w + 1) int32 scratch
void integral_image(const uint8_t* img, int w, int h, int32_t* ii, int32_t* band, hipStream_t s = nullptr) {
  const int nb = (h + kIIBand - 1) / kIIBand;
  k_integral_rows<<<h + 1, 256, 0, s>>>(img, w, h, ii);
  if (nb > 0) {
    const dim3 g(unsigned((w + 1 + 255) / 256), unsigned(nb));
    k_integral_bandsum<<<g, 256, 0, s>>>(w, h, ii, band);
    k_integral_cols<<<g, 256, 0, s>>>(w, h, band, ii);
  }
}
size_t integral_band_ints(int w, int h) { return size_t((h + kIIBand - 1) / kIIBand + 1) * size_t(w + 1); }

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
// Detector (BriskScaleSpace, oracle/brisk_oracle.py): layers c_i / d_i
// resampled by OpenCV's resize(INTER_AREA), FAST 9-16 scores, FAST's 3x3
// non-maximum suppression, then per candidate (one thread) BRISK's 3-D
// refinement (refine3D): interpolated scores of the neighbouring layers
// over the candidate's footprint, subpixel2D in each layer, the parabola
// through the three layers' maxima for the scale, the interpolated position;
// layer 0's virtual lower layer from the 5-8 FAST score.
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
  const uint8_t* R58;  // layer 0's 5-8 scores
  int n;
};

__global__ void k_halfsample(const uint8_t* __restrict__ src, int sw, uint8_t* __restrict__ dst, int dw, int dh) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= dw || y >= dh) return;
  const uint8_t* a = src + size_t(2 * y) * sw + 2 * x;
  dst[size_t(y) * dw + x] = uint8_t((int(a[0]) + a[1] + a[sw] + a[sw + 1] + 2) >> 2);
}
// resize(INTER_AREA) for a ratio other than exactly 2 (OpenCV 3.0
// resizeArea_): per destination pixel, its computeResizeAreaTab entries per
// axis (double geometry, float weights), buf = sum_x S * alpha per source
// row and sum = sum_y beta * buf (float, table order), then cvRound.
struct AreaTab {
  int n;
  int si[6];
  float al[6];
};
__device__ AreaTab area_tab(int d, int ssize, double scale) {
  AreaTab t;
  t.n = 0;
  const double fs1 = d * scale, fs2 = fs1 + scale;
  const double cell = fmin(scale, ssize - fs1);
  int s1 = int(ceil(fs1)), s2 = int(floor(fs2));
  s2 = min(s2, ssize - 1);
  s1 = min(s1, s2);
  if (s1 - fs1 > 1e-3) { t.si[t.n] = s1 - 1; t.al[t.n++] = float((s1 - fs1) / cell); }
  for (int q = s1; q < s2 && t.n < 5; ++q) { t.si[t.n] = q; t.al[t.n++] = float(1.0 / cell); }
  if (fs2 - s2 > 1e-3) { t.si[t.n] = s2; t.al[t.n++] = float(fmin(fmin(fs2 - s2, 1.0), cell) / cell); }
  return t;
}
__global__ void k_area_resize(const uint8_t* __restrict__ src, int sw, int sh, uint8_t* __restrict__ dst, int dw,
                              int dh, double scale_x, double scale_y) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= dw || y >= dh) return;
  const AreaTab tx = area_tab(x, sw, scale_x), ty = area_tab(y, sh, scale_y);
  float acc = 0.0f;
  for (int j = 0; j < ty.n; ++j) {
    const uint8_t* row = src + size_t(ty.si[j]) * sw;
    float buf = 0.0f;
    for (int k = 0; k < tx.n; ++k) buf = buf + float(row[tx.si[k]]) * tx.al[k];
    acc = acc + ty.al[j] * buf;
  }
  dst[size_t(y) * dw + x] = uint8_t(fminf(fmaxf(rintf(acc), 0.0f), 255.0f));
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

// getAgastScore_5_8(x, y, 1): cornerScore<8> (5 contiguous of the 8
// radius-1 neighbours) with threshold 0, kept when >= 1; 0 within 2 pixels
// of the border (layer 0's virtual lower layer in refine3D)
__constant__ int2 kCircle8[8] = {{1, 0}, {1, 1}, {0, 1}, {-1, 1}, {-1, 0}, {-1, -1}, {0, -1}, {1, -1}};
__global__ void k_fast58_score(const uint8_t* __restrict__ img, int w, int h, uint8_t* __restrict__ R) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w || y >= h) return;
  int out = 0;
  if (x >= 2 && y >= 2 && x < w - 2 && y < h - 2) {
    const int v = img[size_t(y) * w + x];
    int d[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = v - int(img[size_t(y + kCircle8[k].y) * w + x + kCircle8[k].x]);
    int dark = -1000000, bright = -1000000;
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      int mn = 1000000, mx = -1000000;
#pragma unroll
      for (int m = 0; m < 5; ++m) {
        mn = min(mn, d[(st + m) & 7]);
        mx = max(mx, d[(st + m) & 7]);
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

// getAgastScore(x, y, 1) and getAgastScore(xf, yf, 1, 1) (bilinear in
// float, truncated like the C++ (uchar) cast of the restatement)
__device__ __forceinline__ int lsc(const Layer& L, int x, int y) {
  if (x < 3 || y < 3 || x >= L.w - 3 || y >= L.h - 3) return 0;
  return L.R[size_t(y) * L.w + x];
}
__device__ int lsc_f(const Layer& L, float xf, float yf) {
  const int x = int(xf), y = int(yf);
  const float rx1 = xf - float(x), rx = 1.0f - rx1;
  const float ry1 = yf - float(y), ry = 1.0f - ry1;
  float v = (rx * ry) * float(lsc(L, x, y));
  v = v + (rx1 * ry) * float(lsc(L, x + 1, y));
  v = v + (rx * ry1) * float(lsc(L, x, y + 1));
  v = v + (rx1 * ry1) * float(lsc(L, x + 1, y + 1));
  return int(v) & 0xFF;
}
__device__ __forceinline__ void patch3(const Layer& L, int cx, int cy, int s[3][3]) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) s[i][j] = lsc(L, cx + i - 1, cy + j - 1);
}

// getScoreMaxAbove / getScoreMaxBelow (oracle score_max_neighbour): false
// when a footprint sample exceeds thr; else the neighbour layer's refined
// maximum and the offset it implies in this layer
__device__ bool score_max_nb(const Layers& LS, int layer, int x, int y, int thr, bool above, float& out_max,
                             float& odx, float& ody) {
  const Layer& M = LS.l[above ? layer + 1 : layer - 1];
  int a, b, c, d;
  if (above) {
    if (layer % 2 == 0) { a = 4; b = -1; c = 2; d = 6; } else { a = 6; b = -1; c = 3; d = 8; }
  } else {
    if (layer % 2 == 0) { a = 8; b = 1; c = 4; d = 6; } else { a = 6; b = 1; c = 3; d = 4; }
  }
  const float x_1 = float(a * x + b - c) / float(d), x1 = float(a * x + b + c) / float(d);
  const float y_1 = float(a * y + b - c) / float(d), y1 = float(a * y + b + c) / float(d);
  const int ix_1 = int(x_1), ix1 = int(x1), iy_1 = int(y_1), iy1 = int(y1);
  int max_x = ix_1 + 1, max_y = iy_1 + 1;
  float best = float(lsc_f(M, x_1, y_1));
  if (best > float(thr)) return false;
  auto take = [&](float v, int mx, int my) {
    if (v > best) { best = v; max_x = mx; max_y = my; }
  };
  for (int xx = ix_1 + 1; xx <= ix1; ++xx) {
    const float v = float(lsc_f(M, float(xx), y_1));
    if (v > float(thr)) return false;
    take(v, xx, max_y);
  }
  {
    const float v = float(lsc_f(M, x1, y_1));
    if (v > float(thr)) return false;
    take(v, ix1, max_y);
  }
  for (int yy = iy_1 + 1; yy <= iy1 + 1; ++yy) {
    const bool last = yy == iy1 + 1;  // the bottom row at y1
    const float yv = last ? y1 : float(yy);
    const int yi = last ? iy1 : yy;
    float v = float(lsc_f(M, x_1, yv));
    if (v > float(thr)) return false;
    take(v, int(x_1 + 1.0f), yi);
    for (int xx = ix_1 + 1; xx <= ix1; ++xx) {
      v = last ? float(lsc_f(M, float(xx), yv)) : float(lsc(M, xx, yy));
      if (v > float(thr)) return false;
      take(v, xx, yi);
    }
    v = float(lsc_f(M, x1, yv));
    if (v > float(thr)) return false;
    take(v, ix1, yi);
  }
  int s3[3][3];
  patch3(M, max_x, max_y, s3);
  float dx1, dy1;
  const float refined = subpixel2d(s3, dx1, dy1);
  float real_x = float(max_x) + dx1, real_y = float(max_y) + dy1;
  bool ret_refined = true;
  if (real_x > x1) { ret_refined = false; real_x = x1; }
  if (real_x < x_1) { ret_refined = false; real_x = x_1; }
  if (real_y > y1) { ret_refined = false; real_y = y1; }
  if (real_y < y_1) { ret_refined = false; real_y = y_1; }
  int m, o, dv;
  if (above) {
    if (layer % 2 == 0) { m = 6; o = 1; dv = 4; } else { m = 8; o = 1; dv = 6; }
  } else {
    if (layer % 2 == 0) { m = 6; o = -1; dv = 8; } else { m = 4; o = -1; dv = 6; }
  }
  float ddx = (real_x * float(m) + float(o)) / float(dv) - float(x);
  float ddy = (real_y * float(m) + float(o)) / float(dv) - float(y);
  odx = fminf(fmaxf(ddx, -1.0f), 1.0f);
  ody = fminf(fmaxf(ddy, -1.0f), 1.0f);
  out_max = ret_refined ? fmaxf(refined, best) : best;
  return true;
}

// refine1D (kind 0: samples at 3/4, 1, 3/2), refine1D_1 (1: 2/3, 1, 4/3),
// refine1D_2 (2: 2/3, 1, 3/2)
__device__ float refine1d(float s_05, float s0, float s05, int kind, float& mx) {
  const int i_05 = int(1024.0 * double(s_05) + 0.5), i0 = int(1024.0 * double(s0) + 0.5),
            i05 = int(1024.0 * double(s05) + 0.5);
  int A0, A1, A2, B0, B1, B2, C0, C1, C2;
  float lo, hi, den;
  if (kind == 0) {
    A0 = 16; A1 = -24; A2 = 8; B0 = -40; B1 = 54; B2 = -14; C0 = 24; C1 = -27; C2 = 6;
    lo = 0.75f; hi = 1.5f; den = 3072.0f;
  } else if (kind == 1) {
    A0 = 9; A1 = -18; A2 = 9; B0 = -21; B1 = 36; B2 = -15; C0 = 12; C1 = -16; C2 = 6;
    lo = float(2.0 / 3.0); hi = float(4.0 / 3.0); den = 2048.0f;
  } else {
    A0 = 18; A1 = -30; A2 = 12; B0 = -45; B1 = 65; B2 = -20; C0 = 27; C1 = -30; C2 = 8;
    lo = float(2.0 / 3.0); hi = 1.5f; den = 5120.0f;
  }
  const int a = A0 * i_05 + A1 * i0 + A2 * i05;
  if (a >= 0) {
    if (s0 >= s_05 && s0 >= s05) { mx = s0; return 1.0f; }
    if (s_05 >= s0 && s_05 >= s05) { mx = s_05; return lo; }
    if (s05 >= s0 && s05 >= s_05) { mx = s05; return hi; }
  }
  const int b = B0 * i_05 + B1 * i0 + B2 * i05;
  float r = -float(b) / float(2 * a);
  if (r < lo) r = lo;
  else if (r > hi) r = hi;
  const int c = C0 * i_05 + C1 * i0 + C2 * i05;
  mx = ((float(c) + (float(a) * r) * r) + float(b) * r) / den;
  return r;
}

// One thread per pixel of layer i: FAST's 3x3 non-maximum suppression on the
// corner scores, then refine3D (or, on the last layer, the 2-D refinement
// against the layer below) -- oracle/brisk_oracle.py detect().
__global__ void k_detect_layer(Layers LS, int i, int thr, Cand* __restrict__ out, int cap, int* __restrict__ count) {
  const Layer& L = LS.l[i];
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= L.w || y >= L.h) return;
  const int c = s_at(L, x, y, thr);
  if (c == 0) return;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx)
      if ((dx || dy) && !(c > s_at(L, x + dx, y + dy, thr))) return;
  const int n = LS.n;
  float kx, ky, ksize, kresp;
  int s3[3][3];
  patch3(L, x, y, s3);
  if (n == 1 || i == n - 1) {
    float mb, bdx, bdy;
    if (n > 1 && !score_max_nb(LS, i, x, y, lsc(L, x, y), false, mb, bdx, bdy)) return;
    float ddx, ddy;
    kresp = subpixel2d(s3, ddx, ddy);
    kx = (float(x) + ddx) * L.scale + L.offset;
    ky = (float(y) + ddy) * L.scale + L.offset;
    ksize = kBasicSize * L.scale;
  } else {
    const int center = lsc(L, x, y);
    float max_above, dxa, dya;
    if (!score_max_nb(LS, i, x, y, center, true, max_above, dxa, dya)) return;
    float max_below, dxb, dyb;
    if (i == 0) {
      int p58[3][3], mb = 0;
#pragma unroll
      for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          const int px = x + a - 1, py = y + b - 1;
          p58[a][b] = (px >= 0 && py >= 0 && px < L.w && py < L.h) ? LS.R58[size_t(py) * L.w + px] : 0;
          mb = max(mb, p58[a][b]);
        }
      subpixel2d(p58, dxb, dyb);
      max_below = float(mb);
    } else if (!score_max_nb(LS, i, x, y, center, false, max_below, dxb, dyb)) {
      return;
    }
    float dxl, dyl;
    const float max_layer = subpixel2d(s3, dxl, dyl);
    const float mid = fmaxf(float(center), max_layer);
    const int kind = i == 0 ? 2 : (i % 2 == 0 ? 0 : 1);
    float mx;
    const float scale = refine1d(max_below, mid, max_above, kind, mx);
    float r0, ro, odx, ody;
    if (i % 2 == 0) {
      if (scale > 1.0f) {
        r0 = (1.5f - scale) / 0.5f;
        ro = 1.0f - r0; odx = dxa; ody = dya;
      } else {
        const float lo = i == 0 ? float(2.0 / 3.0) : 0.75f;
        r0 = (scale - lo) / (1.0f - lo);
        ro = 1.0f - r0; odx = dxb; ody = dyb;
      }
    } else {
      if (scale > 1.0f) {
        r0 = 4.0f - scale * 3.0f;
        ro = 1.0f - r0; odx = dxa; ody = dya;
      } else {
        r0 = scale * 3.0f - 2.0f;
        ro = 1.0f - r0; odx = dxb; ody = dyb;
      }
    }
    if (!(mx > float(thr))) return;
    kx = ((r0 * dxl + ro * odx) + float(x)) * L.scale + L.offset;
    ky = ((r0 * dyl + ro * ody) + float(y)) * L.scale + L.offset;
    ksize = kBasicSize * (scale * L.scale);
    kresp = mx;
  }
  const int k = atomicAdd(count, 1);
  if (k >= cap) return;
  Cand cd;
  cd.key = (static_cast<unsigned long long>(i) << 42) | (static_cast<unsigned long long>(y) << 21) |
           static_cast<unsigned long long>(x);
  cd.x = kx;
  cd.y = ky;
  cd.size = ksize;
  cd.response = kresp;
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
  // pinned host staging of the one packed download (six pageable copies of
  // the per-keypoint outputs before: BRISK 1.0 -> 0.74 ms per frame)
  void* host = nullptr;
  size_t host_cap = 0;
  void* pinned(size_t bytes, int* rc) {
    if (host_cap < bytes) {
      const size_t cap = std::max(bytes, 2 * host_cap);
      if (host) (void)hipHostFree(host);
      host = nullptr;
      host_cap = 0;
      if (hipHostMalloc(&host, cap) != hipSuccess) {
        host = nullptr;
        *rc = bfail(SFM_ENOMEM, "hipHostMalloc failed (detector staging)");
        return nullptr;
      }
      host_cap = cap;
    }
    return host;
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
    int32_t* d_band = nullptr;
    ok = hipMalloc(&d_band, sizeof(int32_t) * integral_band_ints(w, h)) == hipSuccess;
    if (ok) {
      integral_image(d_img, w, h, d_ii, d_band);
      k_brisk_describe<<<n, 64>>>(d_img, w, h, d_ii, *P, d_kps, n, d_keep, d_ang, d_desc);
    }
    if (d_band) (void)hipFree(d_band);
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

// BRISK on an 8-bit frame that is either in host memory (uploaded here) or
// already resident on the device (sfm_klt_brisk_detect_describe: the KLT
// handle's current frame, copied device to device).
namespace sfm {
int brisk_detect_describe_impl(int32_t device, const uint8_t* img, bool img_on_device, int32_t w, int32_t h,
                               int32_t threshold, int32_t octaves, int32_t capacity, float* kps, int32_t* octave,
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
  if (img_on_device) {
    if (hipMemcpy(limg, img, size_t(w) * h, hipMemcpyDeviceToDevice) != hipSuccess)
      return bfail(SFM_EIO, "frame copy failed");
  } else if (hipMemcpy(limg, img, size_t(w) * h, hipMemcpyHostToDevice) != hipSuccess) {
    return bfail(SFM_EIO, "frame copy failed");
  }
  for (int i = 1; i < nuse; ++i) {
    if (lw[i] < 1 || lh[i] < 1) continue;
    // resize(INTER_AREA): OpenCV's scales are 1 / (dsize / ssize); exactly 2
    // on both axes takes the 2x2 average, anything else the area filter
    const int src = i == 1 ? 0 : i - 2;
    const int sw = i == 1 ? w : lw[src], sh = i == 1 ? h : lh[src];
    const double scx = 1.0 / (double(lw[i]) / sw), scy = 1.0 / (double(lh[i]) / sh);
    if (scx == 2.0 && scy == 2.0) {
      dim3 g(unsigned((lw[i] + 255) / 256), unsigned(lh[i]));
      k_halfsample<<<g, 256>>>(limg + loff_px[src], sw, limg + loff_px[i], lw[i], lh[i]);
    } else {
      dim3 g(unsigned((lw[i] + 127) / 128), unsigned(lh[i]));
      k_area_resize<<<g, 128>>>(limg + loff_px[src], sw, sh, limg + loff_px[i], lw[i], lh[i], scx, scy);
    }
  }
  Layers LS;
  LS.n = nuse;
  auto* R58 = static_cast<uint8_t*>(W->get(14, size_t(w) * h, &rc));
  if (rc) return rc;
  {
    dim3 g(unsigned((w + 255) / 256), unsigned(h));
    k_fast58_score<<<g, 256>>>(limg, w, h, R58);
  }
  LS.R58 = R58;
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
  // every per-keypoint output in one buffer (descriptors first, 16-B
  // aligned), downloaded by one copy: desc | kp3 | resp | layer | keep | angle
  const int n_bytes = desc ? ((P->n_short + 127) / 128) * 16 : 0;
  const size_t o_kp = size_t(n) * n_bytes, o_resp = o_kp + 12 * size_t(n), o_lay = o_resp + 4 * size_t(n),
               o_keep = o_lay + 4 * size_t(n), o_ang = o_keep + 4 * size_t(n), out_bytes = o_ang + 4 * size_t(n);
  auto* ob = static_cast<uint8_t*>(W->get(6, out_bytes, &rc));
  if (rc) return rc;
  auto* kp3 = reinterpret_cast<float*>(ob + o_kp);
  auto* resp = reinterpret_cast<float*>(ob + o_resp);
  auto* lay = reinterpret_cast<int32_t*>(ob + o_lay);
  k_cand_keys<<<(n + 255) / 256, 256>>>(cand, n, key, idx);
  size_t tb = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key, key + n, idx, idx + n, n, 0, 46);
  void* tmp = W->get(9, tb, &rc);
  if (rc) return rc;
  if (hipcub::DeviceRadixSort::SortPairs(tmp, tb, key, key + n, idx, idx + n, n, 0, 46) != hipSuccess)
    return bfail(SFM_EIO, "sort failed");
  k_gather_cands<<<(n + 255) / 256, 256>>>(cand, idx + n, n, kp3, resp, lay);
  if (desc) {
    auto* keep = reinterpret_cast<int32_t*>(ob + o_keep);
    auto* ang = reinterpret_cast<float*>(ob + o_ang);
    auto* ii = static_cast<int32_t*>(W->get(12, sizeof(int32_t) * size_t(w + 1) * (h + 1), &rc));
    auto* band = static_cast<int32_t*>(W->get(15, sizeof(int32_t) * integral_band_ints(w, h), &rc));
    if (rc) return rc;
    integral_image(limg, w, h, ii, band);
    k_brisk_describe<<<n, 64>>>(limg, w, h, ii, *P, kp3, n, keep, ang, ob);
  }
  // one download of the packed outputs (without descriptors: kp3 | resp | layer)
  const size_t dl_off = desc ? 0 : o_kp, dl_bytes = desc ? out_bytes : o_keep - o_kp;
  auto* hb = static_cast<uint8_t*>(W->pinned(out_bytes, &rc));
  if (rc) return rc;
  if (hipMemcpy(hb + dl_off, ob + dl_off, dl_bytes, hipMemcpyDeviceToHost) != hipSuccess)
    return bfail(SFM_EIO, "download failed");
  const float* hk = reinterpret_cast<const float*>(hb + o_kp);
  const float* hr = reinterpret_cast<const float*>(hb + o_resp);
  const int32_t* hl = reinterpret_cast<const int32_t*>(hb + o_lay);
  const int32_t* hkeep = desc ? reinterpret_cast<const int32_t*>(hb + o_keep) : nullptr;
  const float* hang = desc ? reinterpret_cast<const float*>(hb + o_ang) : nullptr;
  const uint8_t* hd = hb;
  int m = 0;
  for (int k = 0; k < n; ++k) {
    if (hkeep && !hkeep[k]) continue;
    if (m < capacity) {
      float* o = kps + 5 * size_t(m);
      o[0] = hk[3 * k]; o[1] = hk[3 * k + 1]; o[2] = hk[3 * k + 2]; o[3] = hang ? hang[k] : -1.0f; o[4] = hr[k];
      octave[m] = hl[k];
      if (desc) std::memcpy(desc + size_t(m) * 64, hd + size_t(k) * n_bytes, 64);
    }
    ++m;
  }
  *n_out = m;
  if (m > capacity) return bfail(SFM_EINVAL, "capacity " + std::to_string(capacity) + " < " + std::to_string(m));
  return 0;
}
}  // namespace sfm

extern "C" int sfm_brisk_detect_describe(int32_t device, const uint8_t* img, int32_t w, int32_t h, int32_t threshold,
                                         int32_t octaves, int32_t capacity, float* kps, int32_t* octave,
                                         uint8_t* desc, int32_t* n_out) {
  SFM_TRACE("sfm_brisk_detect_describe");
  return brisk_detect_describe_impl(device, img, false, w, h, threshold, octaves, capacity, kps, octave, desc, n_out);
}
