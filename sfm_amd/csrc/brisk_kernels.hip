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
