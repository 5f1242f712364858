// Per-frame pyramidal Lucas-Kanade tracker for gfx950.
//
// Replaces the tracker seam CTracker::computeOpticalFlow
// (/root/reference/CTracker.cpp:480-562, decl. CTracker.h:60) and the
// external call it makes at CTracker.cpp:513,
//   cv::calcOpticalFlowPyrLK(prevGrey, currGrey, prevPts, currPts, status,
//                            err, Size(21,21), 3,
//                            TermCriteria(COUNT|EPS, 20, 0.03), 0, 0.001),
// plus the nearest-detected-point association of
// CFrame::findClosestPointIndexDistorted (CFrame.cpp:437-450) and the
// gate / better-or-equal replacement loop of CTracker.cpp:515-545.
// Arithmetic follows the oracle restatement (oracle/klt_oracle.cpp) op for
// op: integer pyramid and Scharr derivatives, 14-bit fixed-point bilinear
// patches, exact int64 sums of the integer products, float Newton steps
// with contraction disabled — so results are bit-exact against it.
//
// Layout (one handle = one frame size on one GPU): two frame slots
// (ping-pong: pushing a frame makes the old current frame the previous);
// each slot holds every pyramid level (u8, unpadded, row-major) and the
// Scharr derivatives of every level (int16 pairs).  Frames are 0.92 MB at
// 1280x720, so the pyramid build is L2-resident; the tracking kernel is
// latency bound (one wavefront per point, 4 levels x <= 20 dependent
// Newton steps), see DESIGN.md §5.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cfloat>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>
#include "sfm_trace.h"
#include "../../include/sfm_amd.h"
#include "ordered_compact.h"
#include "klt_internal.h"

void sfm_internal_set_error(const std::string& msg);  // ba_solver.hip

namespace {

constexpr int kMaxLv = 16;

struct Pyr {
  const uint8_t* img[kMaxLv];
  const short2* dxy[kMaxLv];
  int w[kMaxLv], h[kMaxLv];
};

int kfail(int code, const std::string& m) {
  sfm_internal_set_error(m);
  return code;
}

// BORDER_REFLECT_101 (cv::borderInterpolate), repeated for tiny levels.
__device__ __forceinline__ int r101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
  }
  return i;
}

__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }

// pyrDown: 5x5 [1 4 6 4 1]^2 / 256, reflect-101 borders, +128 rounding.
__global__ __launch_bounds__(256) void k_pyr_down(const uint8_t* __restrict__ s, int sw, int sh,
                                                  uint8_t* __restrict__ d, int dw, int dh) {
  const int x = blockIdx.x * 32 + (threadIdx.x & 31);
  const int y = blockIdx.y * 8 + (threadIdx.x >> 5);
  if (x >= dw || y >= dh) return;
  const int k[5] = {1, 4, 6, 4, 1};
  int cx[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) cx[j] = r101(2 * x + j - 2, sw);
  int acc = 0;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const uint8_t* row = s + size_t(r101(2 * y + i - 2, sh)) * sw;
    int hs = 0;
#pragma unroll
    for (int j = 0; j < 5; ++j) hs += k[j] * row[cx[j]];
    acc += k[i] * hs;
  }
  d[size_t(y) * dw + x] = uint8_t((acc + 128) >> 8);
}

// calcSharrDeriv: (Ix, Iy) per pixel, rows and columns reflect-101.
__global__ __launch_bounds__(256) void k_scharr(const uint8_t* __restrict__ s, int w, int h,
                                                short2* __restrict__ d) {
  const int x = blockIdx.x * 32 + (threadIdx.x & 31);
  const int y = blockIdx.y * 8 + (threadIdx.x >> 5);
  if (x >= w || y >= h) return;
  const uint8_t* s0 = s + size_t(y > 0 ? y - 1 : (h > 1 ? 1 : 0)) * w;
  const uint8_t* s1 = s + size_t(y) * w;
  const uint8_t* s2 = s + size_t(y < h - 1 ? y + 1 : (h > 1 ? h - 2 : 0)) * w;
  const int xl = x > 0 ? x - 1 : (w > 1 ? 1 : 0), xr = x < w - 1 ? x + 1 : (w > 1 ? w - 2 : 0);
  const int t0l = (s0[xl] + s2[xl]) * 3 + s1[xl] * 10, t0r = (s0[xr] + s2[xr]) * 3 + s1[xr] * 10;
  const int t1l = s2[xl] - s0[xl], t1c = s2[x] - s0[x], t1r = s2[xr] - s0[xr];
  d[size_t(y) * w + x] = make_short2(short(t0r - t0l), short((t1r + t1l) * 3 + t1c * 10));
}

__device__ __forceinline__ long long wave_sum(long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// LKTrackerInvoker for one point over every level: one wavefront per point,
// the window's pixels spread over the 64 lanes (SLOTS per lane), integer
// products summed per lane and across the wave in int64 (exact), the 2x2
// solve and the stopping rules evaluated uniformly by every lane.
template <int SLOTS>
__global__ __launch_bounds__(64) void k_lk(Pyr I, Pyr J, int n, const float2* __restrict__ prev,
                                           float2* __restrict__ next, uint8_t* __restrict__ status, int win,
                                           int maxLevel, int maxCount, double eps2, double minEigThr) {
#pragma clang fp contract(off)
  const int i = blockIdx.x;
  if (i >= n) return;
  const int lane = threadIdx.x;
  const int area = win * win;
  const float half = (win - 1) * 0.5f;
  const float FLT_SCALE = 1.f / (1 << 20);
  const float px = prev[i].x, py = prev[i].y;
  float nx = 0.f, ny = 0.f;
  bool st = true;
  int sx[SLOTS], sy[SLOTS];
  bool sv[SLOTS];
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const int k = lane + 64 * s;
    sv[s] = k < area;
    sy[s] = k / win;
    sx[s] = k - sy[s] * win;
  }
  int Ip[SLOTS], Dx[SLOTS], Dy[SLOTS];
  for (int level = maxLevel; level >= 0; --level) {
    const uint8_t* Ii = I.img[level];
    const short2* Di = I.dxy[level];
    const int w = I.w[level], h = I.h[level];
    const float sc = (float)(1. / (1 << level));
    float ppx = px * sc, ppy = py * sc;
    float npx, npy;
    if (level == maxLevel) { npx = ppx; npy = ppy; }
    else { npx = nx * 2.f; npy = ny * 2.f; }
    nx = npx;
    ny = npy;
    ppx -= half;
    ppy -= half;
    const int ipx = (int)floorf(ppx), ipy = (int)floorf(ppy);
    if (ipx < -win || ipx >= w || ipy < -win || ipy >= h) {
      if (level == 0) st = false;
      continue;
    }
    float a = ppx - ipx, b = ppy - ipy;
    int iw00 = __float2int_rn((1.f - a) * (1.f - b) * 16384.f);
    int iw01 = __float2int_rn(a * (1.f - b) * 16384.f);
    int iw10 = __float2int_rn((1.f - a) * b * 16384.f);
    int iw11 = 16384 - iw00 - iw01 - iw10;
    long long a11 = 0, a12 = 0, a22 = 0;
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) {
      Ip[s] = Dx[s] = Dy[s] = 0;
      if (!sv[s]) continue;
      const int X = ipx + sx[s], Y = ipy + sy[s];
      const int x0 = r101(X, w), x1 = r101(X + 1, w);
      const uint8_t* r0 = Ii + size_t(r101(Y, h)) * w;
      const uint8_t* r1 = Ii + size_t(r101(Y + 1, h)) * w;
      Ip[s] = descale(r0[x0] * iw00 + r0[x1] * iw01 + r1[x0] * iw10 + r1[x1] * iw11, 9);
      const bool cin0 = X >= 0 && X < w, cin1 = X + 1 >= 0 && X + 1 < w;
      const bool rin0 = Y >= 0 && Y < h, rin1 = Y + 1 >= 0 && Y + 1 < h;
      const short2 z = make_short2(0, 0);
      const short2 d00 = (rin0 && cin0) ? Di[size_t(Y) * w + X] : z;
      const short2 d01 = (rin0 && cin1) ? Di[size_t(Y) * w + X + 1] : z;
      const short2 d10 = (rin1 && cin0) ? Di[size_t(Y + 1) * w + X] : z;
      const short2 d11 = (rin1 && cin1) ? Di[size_t(Y + 1) * w + X + 1] : z;
      Dx[s] = descale(d00.x * iw00 + d01.x * iw01 + d10.x * iw10 + d11.x * iw11, 14);
      Dy[s] = descale(d00.y * iw00 + d01.y * iw01 + d10.y * iw10 + d11.y * iw11, 14);
      a11 += (long long)(Dx[s] * Dx[s]);
      a12 += (long long)(Dx[s] * Dy[s]);
      a22 += (long long)(Dy[s] * Dy[s]);
    }
    a11 = wave_sum(a11);
    a12 = wave_sum(a12);
    a22 = wave_sum(a22);
    const float A11 = (float)a11 * FLT_SCALE, A12 = (float)a12 * FLT_SCALE, A22 = (float)a22 * FLT_SCALE;
    float D = A11 * A22 - A12 * A12;
    const float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * area);
    if ((double)minEig < minEigThr || D < FLT_EPSILON) {
      if (level == 0) st = false;
      continue;
    }
    D = 1.f / D;
    npx -= half;
    npy -= half;
    float pdx = 0.f, pdy = 0.f;
    const uint8_t* Ij = J.img[level];
    const int wj = J.w[level], hj = J.h[level];
    for (int j = 0; j < maxCount; ++j) {
      const int inx = (int)floorf(npx), iny = (int)floorf(npy);
      if (inx < -win || inx >= wj || iny < -win || iny >= hj) {
        if (level == 0) st = false;
        break;
      }
      a = npx - inx;
      b = npy - iny;
      iw00 = __float2int_rn((1.f - a) * (1.f - b) * 16384.f);
      iw01 = __float2int_rn(a * (1.f - b) * 16384.f);
      iw10 = __float2int_rn((1.f - a) * b * 16384.f);
      iw11 = 16384 - iw00 - iw01 - iw10;
      long long b1 = 0, b2 = 0;
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        if (!sv[s]) continue;
        const int X = inx + sx[s], Y = iny + sy[s];
        const int x0 = r101(X, wj), x1 = r101(X + 1, wj);
        const uint8_t* r0 = Ij + size_t(r101(Y, hj)) * wj;
        const uint8_t* r1 = Ij + size_t(r101(Y + 1, hj)) * wj;
        const int diff = descale(r0[x0] * iw00 + r0[x1] * iw01 + r1[x0] * iw10 + r1[x1] * iw11, 9) - Ip[s];
        b1 += (long long)(diff * Dx[s]);
        b2 += (long long)(diff * Dy[s]);
      }
      b1 = wave_sum(b1);
      b2 = wave_sum(b2);
      const float fb1 = (float)b1 * FLT_SCALE, fb2 = (float)b2 * FLT_SCALE;
      const float dx = (A12 * fb2 - A22 * fb1) * D;
      const float dy = (A12 * fb1 - A11 * fb2) * D;
      npx += dx;
      npy += dy;
      nx = npx + half;
      ny = npy + half;
      if ((double)dx * dx + (double)dy * dy <= eps2) break;
      if (j > 0 && fabsf(dx + pdx) < 0.01 && fabsf(dy + pdy) < 0.01) {
        nx -= dx * 0.5f;
        ny -= dy * 0.5f;
        break;
      }
      pdx = dx;
      pdy = dy;
    }
  }
  if (lane == 0) {
    next[i] = make_float2(nx, ny);
    status[i] = st ? 1 : 0;
  }
}

// Association of every flowed point (status set) with the nearest detected
// point (double distances, first minimum: CFrame.cpp:437-450), the gates of
// CTracker.cpp:525 in float, and the order-free form of the replacement
// loop (CTracker.cpp:525-545): per detected point the surviving query is
// the LAST candidate with the minimum e (ties: `>=` replaces), the slot
// order is that of each detected point's first candidate.
constexpr int kAssocTile = 256;
__global__ __launch_bounds__(kAssocTile) void k_assoc(int n, const float2* __restrict__ prev,
                                                      const float2* __restrict__ flowed,
                                                      const uint8_t* __restrict__ status, int m,
                                                      const double2* __restrict__ curr, double maxDistSq,
                                                      double maxFeatDistSq, double minDistSq,
                                                      unsigned long long* __restrict__ key, int* __restrict__ first) {
#pragma clang fp contract(off)
  __shared__ double2 tile[kAssocTile];
  const int i = blockIdx.x * kAssocTile + threadIdx.x;
  const bool active = i < n && status[i];
  const float cx = active ? flowed[i].x : 0.f, cy = active ? flowed[i].y : 0.f;
  const double dcx = cx, dcy = cy;
  double best = DBL_MAX;
  int idx = -1;
  for (int t0 = 0; t0 < m; t0 += kAssocTile) {
    const int nt = min(kAssocTile, m - t0);
    __syncthreads();
    if (threadIdx.x < nt) tile[threadIdx.x] = curr[t0 + threadIdx.x];
    __syncthreads();
    if (active)
      for (int t = 0; t < nt; ++t) {
        const double ex = tile[t].x - dcx, ey = tile[t].y - dcy;
        const double d = ex * ex + ey * ey;
        if (d < best) { best = d; idx = t0 + t; }
      }
  }
  if (!active || idx < 0) return;
  const float qx = (float)curr[idx].x, qy = (float)curr[idx].y;
  const float e = (cx - qx) * (cx - qx) + (cy - qy) * (cy - qy);
  const float px = prev[i].x, py = prev[i].y;
  const float d = (px - cx) * (px - cx) + (py - cy) * (py - cy);
  if ((double)d < maxDistSq && (double)e < maxFeatDistSq && (double)d > minDistSq) {
    atomicMin(&key[idx], (static_cast<unsigned long long>(__float_as_uint(e)) << 32) |
                             static_cast<unsigned long long>(0xffffffffu - unsigned(i)));
    atomicMin(&first[idx], i);
  }
}

__global__ void k_assoc_init(int m, unsigned long long* __restrict__ key, int* __restrict__ first) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < m) {
    key[j] = ~0ull;
    first[j] = 0x7fffffff;
  }
}

int slots_for(int win) { return (win * win + 63) / 64; }

int launch_lk(const Pyr& I, const Pyr& J, int n, const float2* prev, float2* next, uint8_t* st, int win, int maxLevel,
              int maxCount, double eps2, double minEig, hipStream_t s) {
  if (n == 0) return 0;
  switch (slots_for(win)) {
#define CASE(k) case k: k_lk<k><<<n, 64, 0, s>>>(I, J, n, prev, next, st, win, maxLevel, maxCount, eps2, minEig); break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
    CASE(9) CASE(10) CASE(11) CASE(12) CASE(13) CASE(14) CASE(15) CASE(16)
#undef CASE
    default: return kfail(SFM_ENOTSUP, "window larger than 31x31 is not supported");
  }
  return hipGetLastError() == hipSuccess ? 0 : kfail(SFM_EIO, "k_lk launch failed");
}

// buildOpticalFlowPyramid's level count: stop once a level would not exceed
// the window (lkpyramid.cpp).
int pyramid_levels(int w, int h, int max_level, int win) {
  int l = 0;
  while (l < max_level && l + 1 < kMaxLv) {
    w = (w + 1) / 2;
    h = (h + 1) / 2;
    if (w <= win || h <= win) break;
    ++l;
  }
  return l;
}

}  // namespace

namespace sfm {
// brisk_kernels.hip
int brisk_detect_describe_impl(int32_t device, const uint8_t* img, bool img_on_device, int32_t w, int32_t h,
                               int32_t threshold, int32_t octaves, int32_t capacity, float* kps, int32_t* octave,
                               uint8_t* desc, int32_t* n_out);
}  // namespace sfm

struct sfm_klt_handle {
  int device = 0;
  hipStream_t stream = nullptr;
  int w = 0, h = 0, levels = 0;
  sfm_klt_params prm{};
  int lw[kMaxLv] = {}, lh[kMaxLv] = {};
  size_t img_off[kMaxLv + 1] = {}, pix_total = 0;
  uint8_t* img[2] = {nullptr, nullptr};
  short2* dxy[2] = {nullptr, nullptr};
  int n_frames = 0;  // frames pushed so far
  int cur = 0;       // slot of the current frame (prev = cur ^ 1)
  // point buffers
  int cap_n = 0, cap_m = 0;
  float2* d_prev = nullptr;
  float2* d_next = nullptr;
  uint8_t* d_status = nullptr;
  int* d_slot = nullptr;
  int* d_out = nullptr;  // [2n + 1]
  double2* d_curr = nullptr;
  unsigned long long* d_key = nullptr;
  int* d_first = nullptr;
  // phase timing: [0,1] pyramid, [2,3] lk, [4,5] association
  hipEvent_t ev[6] = {};
  bool timed_push = false, timed_flow = false, timed_assoc = false;
  void* gftt = nullptr;  // corner-detector state (gftt_kernels.hip)

  Pyr pyr(int slot) const {
    Pyr p{};
    for (int l = 0; l <= levels; ++l) {
      p.img[l] = img[slot] + img_off[l];
      p.dxy[l] = dxy[slot] + img_off[l];
      p.w[l] = lw[l];
      p.h[l] = lh[l];
    }
    return p;
  }
};

namespace {

// (Re)allocates a device buffer to hold `count` elements (contents dropped).
template <typename T>
bool realloc_dev(T** p, size_t count) {
  if (*p) hipFree(*p);
  *p = nullptr;
  return hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T)) == hipSuccess;
}

int ensure_points(sfm_klt_handle* h, int n, int m) {
  if (n > h->cap_n) {
    h->cap_n = 0;
    if (!realloc_dev(&h->d_prev, n) || !realloc_dev(&h->d_next, n) || !realloc_dev(&h->d_status, n) ||
        !realloc_dev(&h->d_slot, n) || !realloc_dev(&h->d_out, 2 * size_t(n) + 1))
      return kfail(SFM_ENOMEM, "hipMalloc failed (klt points)");
    h->cap_n = n;
  }
  if (m > h->cap_m) {
    h->cap_m = 0;
    if (!realloc_dev(&h->d_curr, m) || !realloc_dev(&h->d_key, m) || !realloc_dev(&h->d_first, m))
      return kfail(SFM_ENOMEM, "hipMalloc failed (klt detections)");
    h->cap_m = m;
  }
  return 0;
}

int check_params(const sfm_klt_params* p) {
  if (p->win_size < 3 || (p->win_size & 1) == 0) return kfail(SFM_EINVAL, "win_size must be odd and >= 3");
  if (p->win_size > 31) return kfail(SFM_ENOTSUP, "win_size > 31 is not supported");
  if (p->max_level < 0) return kfail(SFM_EINVAL, "max_level must be >= 0");
  return 0;
}

double eps2_of(const sfm_klt_params& p) {
  const double e = std::min(std::max(p.epsilon, 0.), 10.);
  return e * e;
}
int max_count_of(const sfm_klt_params& p) { return std::min(std::max(p.max_count, 0), 100); }

float ms_between(hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  return hipEventElapsedTime(&ms, a, b) == hipSuccess ? ms : 0.f;
}

}  // namespace

extern "C" {

void sfm_klt_default_params(sfm_klt_params* p) {
  // CTracker::computeOpticalFlow (CTracker.cpp:484-489) and the CTracker
  // constructor's match gates (CTracker.cpp:30-33).
  p->win_size = 21;
  p->max_level = 3;
  p->max_count = 20;
  p->reserved = 0;
  p->epsilon = 0.03;
  p->min_eig_threshold = 0.001;
  p->max_match_distance = 40.0;
  p->min_match_distance = 1.5;
  p->max_org_feat_dist = 1.0;
}

int sfm_klt_create(int32_t device, int32_t width, int32_t height, const sfm_klt_params* params,
                   sfm_klt_handle** out) {
  if (!out) return kfail(SFM_EINVAL, "out is NULL");
  *out = nullptr;
  if (width <= 0 || height <= 0) return kfail(SFM_EINVAL, "bad frame size");
  sfm_klt_params p;
  sfm_klt_default_params(&p);
  if (params) p = *params;
  if (int rc = check_params(&p)) return rc;
  if (hipSetDevice(device) != hipSuccess) return kfail(SFM_ENODEV, "hipSetDevice failed");
  auto* h = new sfm_klt_handle();
  h->device = device;
  h->w = width;
  h->h = height;
  h->prm = p;
  h->levels = pyramid_levels(width, height, p.max_level, p.win_size);
  int w = width, hh = height;
  size_t off = 0;
  for (int l = 0; l <= h->levels; ++l) {
    h->lw[l] = w;
    h->lh[l] = hh;
    h->img_off[l] = off;
    off += size_t(w) * hh;
    off = (off + 255) & ~size_t(255);
    w = (w + 1) / 2;
    hh = (hh + 1) / 2;
  }
  h->img_off[h->levels + 1] = off;
  h->pix_total = off;
  bool ok = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) == hipSuccess;
  for (int s = 0; s < 2 && ok; ++s) {
    ok = hipMalloc(reinterpret_cast<void**>(&h->img[s]), off) == hipSuccess &&
         hipMalloc(reinterpret_cast<void**>(&h->dxy[s]), off * sizeof(short2)) == hipSuccess;
  }
  for (int e = 0; e < 6 && ok; ++e) ok = hipEventCreate(&h->ev[e]) == hipSuccess;
  if (!ok) {
    sfm_klt_destroy(h);
    return kfail(SFM_ENOMEM, "device allocation failed (klt frames)");
  }
  *out = h;
  return 0;
}

int sfm_klt_destroy(sfm_klt_handle* h) {
  if (!h) return 0;
  hipSetDevice(h->device);
  if (h->stream) hipStreamSynchronize(h->stream);
  for (int s = 0; s < 2; ++s) {
    if (h->img[s]) hipFree(h->img[s]);
    if (h->dxy[s]) hipFree(h->dxy[s]);
  }
  void* bufs[] = {h->d_prev, h->d_next, h->d_status, h->d_slot, h->d_out, h->d_curr, h->d_key, h->d_first};
  for (void* b : bufs)
    if (b) hipFree(b);
  for (auto& e : h->ev)
    if (e) hipEventDestroy(e);
  if (h->gftt) sfm_internal_gftt_free(h->gftt);
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
  return 0;
}

int32_t sfm_klt_num_levels(const sfm_klt_handle* h) { return h ? h->levels + 1 : 0; }

int sfm_klt_push_frame(sfm_klt_handle* h, const uint8_t* grey, int32_t stride) {
  SFM_TRACE("sfm_klt_push_frame");
  if (!h || !grey) return kfail(SFM_EINVAL, "NULL argument");
  if (stride < h->w) return kfail(SFM_EINVAL, "stride < width");
  hipSetDevice(h->device);
  const int slot = h->n_frames == 0 ? 0 : (h->cur ^ 1);
  hipStream_t s = h->stream;
  // Synchronous with respect to the caller's buffer (pageable source; a
  // pinned stage measured no faster for the 0.9-MB frame: the runtime
  // pipelines its staging copies with the DMA).
  if (hipMemcpy2DAsync(h->img[slot], h->w, grey, stride, h->w, h->h, hipMemcpyHostToDevice, s) != hipSuccess)
    return kfail(SFM_EIO, "frame upload failed");
  hipEventRecord(h->ev[0], s);
  for (int l = 1; l <= h->levels; ++l) {
    dim3 g((h->lw[l] + 31) / 32, (h->lh[l] + 7) / 8);
    k_pyr_down<<<g, 256, 0, s>>>(h->img[slot] + h->img_off[l - 1], h->lw[l - 1], h->lh[l - 1],
                                 h->img[slot] + h->img_off[l], h->lw[l], h->lh[l]);
  }
  for (int l = 0; l <= h->levels; ++l) {
    dim3 g((h->lw[l] + 31) / 32, (h->lh[l] + 7) / 8);
    k_scharr<<<g, 256, 0, s>>>(h->img[slot] + h->img_off[l], h->lw[l], h->lh[l], h->dxy[slot] + h->img_off[l]);
  }
  hipEventRecord(h->ev[1], s);
  if (hipGetLastError() != hipSuccess) return kfail(SFM_EIO, "pyramid launch failed");
  if (hipStreamSynchronize(s) != hipSuccess) return kfail(SFM_EIO, "pyramid build failed");
  h->cur = slot;
  ++h->n_frames;
  h->timed_push = true;
  return 0;
}

int sfm_klt_brisk_detect_describe(sfm_klt_handle* h, int32_t threshold, int32_t octaves, int32_t capacity,
                                  float* kps, int32_t* octave, uint8_t* desc, int32_t* n_out) {
  if (!h || !n_out) return kfail(SFM_EINVAL, "NULL argument");
  if (h->n_frames == 0) return kfail(SFM_EINVAL, "no frame pushed");
  hipSetDevice(h->device);
  // (push_frame left its stream drained; this keeps any later use ordered)
  if (hipStreamSynchronize(h->stream) != hipSuccess) return kfail(SFM_EIO, "klt stream failed");
  return sfm::brisk_detect_describe_impl(h->device, h->img[h->cur], true, h->w, h->h, threshold, octaves, capacity,
                                         kps, octave, desc, n_out);
}

int sfm_klt_get_level(sfm_klt_handle* h, int32_t which, int32_t level, uint8_t* img, int16_t* dxy, int32_t* w,
                      int32_t* hh) {
  if (!h) return kfail(SFM_EINVAL, "NULL handle");
  if (level < 0 || level > h->levels) return kfail(SFM_EINVAL, "level out of range");
  if (which != 0 && which != 1) return kfail(SFM_EINVAL, "which must be 0 (previous) or 1 (current)");
  if (h->n_frames < (which == 0 ? 2 : 1)) return kfail(SFM_EINVAL, "frame not pushed yet");
  hipSetDevice(h->device);
  const int slot = which == 1 ? h->cur : (h->cur ^ 1);
  const size_t np = size_t(h->lw[level]) * h->lh[level];
  if (w) *w = h->lw[level];
  if (hh) *hh = h->lh[level];
  hipStreamSynchronize(h->stream);
  if (img && hipMemcpy(img, h->img[slot] + h->img_off[level], np, hipMemcpyDeviceToHost) != hipSuccess)
    return kfail(SFM_EIO, "copy failed");
  if (dxy && hipMemcpy(dxy, h->dxy[slot] + h->img_off[level], np * sizeof(short2), hipMemcpyDeviceToHost) !=
                 hipSuccess)
    return kfail(SFM_EIO, "copy failed");
  return 0;
}

int sfm_klt_calc_flow(sfm_klt_handle* h, const float* prev_pts, int32_t n, float* next_pts, uint8_t* status) {
  if (!h) return kfail(SFM_EINVAL, "NULL handle");
  if (n < 0 || (n > 0 && (!prev_pts || !next_pts || !status))) return kfail(SFM_EINVAL, "bad point arrays");
  if (h->n_frames < 2) return kfail(SFM_EINVAL, "calc_flow needs two pushed frames");
  if (n == 0) return 0;
  hipSetDevice(h->device);
  if (int rc = ensure_points(h, n, 0)) return rc;
  hipStream_t s = h->stream;
  hipMemcpyAsync(h->d_prev, prev_pts, sizeof(float2) * n, hipMemcpyHostToDevice, s);
  hipEventRecord(h->ev[2], s);
  const Pyr I = h->pyr(h->cur ^ 1), J = h->pyr(h->cur);
  if (int rc = launch_lk(I, J, n, h->d_prev, h->d_next, h->d_status, h->prm.win_size, h->levels,
                         max_count_of(h->prm), eps2_of(h->prm), h->prm.min_eig_threshold, s))
    return rc;
  hipEventRecord(h->ev[3], s);
  hipMemcpyAsync(next_pts, h->d_next, sizeof(float2) * n, hipMemcpyDeviceToHost, s);
  hipMemcpyAsync(status, h->d_status, n, hipMemcpyDeviceToHost, s);
  if (hipStreamSynchronize(s) != hipSuccess) return kfail(SFM_EIO, "k_lk failed");
  h->timed_flow = true;
  h->timed_assoc = false;
  return 0;
}

int sfm_klt_compute_optical_flow(sfm_klt_handle* h, const double* prev_pts_dist, int32_t n_prev,
                                 const double* curr_pts_dist, int32_t n_curr, int32_t* prev_idx, int32_t* curr_idx,
                                 int32_t* n_matches, float* flowed, uint8_t* status) {
  if (!h || !n_matches) return kfail(SFM_EINVAL, "NULL argument");
  *n_matches = 0;
  if (n_prev < 0 || n_curr < 0) return kfail(SFM_EINVAL, "negative point count");
  if (h->n_frames < 2) return kfail(SFM_EINVAL, "compute_optical_flow needs two pushed frames");
  if (n_prev == 0) return 0;
  if (!prev_pts_dist || (n_curr > 0 && (!curr_pts_dist || !prev_idx || !curr_idx)))
    return kfail(SFM_EINVAL, "bad point arrays");
  hipSetDevice(h->device);
  if (int rc = ensure_points(h, n_prev, n_curr)) return rc;
  hipStream_t s = h->stream;
  // Mat(vector<Point2d>).copyTo(vector<Point2f>) (CTracker.cpp:498): float cast.
  std::vector<float2> pf(n_prev);
  for (int i = 0; i < n_prev; ++i) pf[i] = make_float2((float)prev_pts_dist[2 * i], (float)prev_pts_dist[2 * i + 1]);
  hipMemcpyAsync(h->d_prev, pf.data(), sizeof(float2) * n_prev, hipMemcpyHostToDevice, s);
  if (n_curr > 0) hipMemcpyAsync(h->d_curr, curr_pts_dist, sizeof(double2) * n_curr, hipMemcpyHostToDevice, s);
  hipEventRecord(h->ev[2], s);
  const Pyr I = h->pyr(h->cur ^ 1), J = h->pyr(h->cur);
  if (int rc = launch_lk(I, J, n_prev, h->d_prev, h->d_next, h->d_status, h->prm.win_size, h->levels,
                         max_count_of(h->prm), eps2_of(h->prm), h->prm.min_eig_threshold, s))
    return rc;
  hipEventRecord(h->ev[3], s);
  int m = 0;
  if (n_curr > 0) {
    k_assoc_init<<<(n_curr + 255) / 256, 256, 0, s>>>(n_curr, h->d_key, h->d_first);
    hipMemsetAsync(h->d_slot, 0, sizeof(int) * n_prev, s);
    const double maxD = h->prm.max_match_distance, minD = h->prm.min_match_distance, mf = h->prm.max_org_feat_dist;
    k_assoc<<<(n_prev + kAssocTile - 1) / kAssocTile, kAssocTile, 0, s>>>(
        n_prev, h->d_prev, h->d_next, h->d_status, n_curr, h->d_curr, maxD * maxD, mf * mf, minD * minD, h->d_key,
        h->d_first);
    sfm::k_mark_first<<<(n_curr + 255) / 256, 256, 0, s>>>(n_curr, h->d_first, h->d_slot);
    sfm::k_compact_slots<true><<<1, 1024, 0, s>>>(n_prev, h->d_slot, h->d_key, h->d_out, h->d_out + n_prev,
                                                  h->d_out + 2 * n_prev);
    hipEventRecord(h->ev[5], s);
    if (hipGetLastError() != hipSuccess) return kfail(SFM_EIO, "association launch failed");
    hipMemcpyAsync(&m, h->d_out + 2 * n_prev, sizeof(int), hipMemcpyDeviceToHost, s);
  }
  if (flowed) hipMemcpyAsync(flowed, h->d_next, sizeof(float2) * n_prev, hipMemcpyDeviceToHost, s);
  if (status) hipMemcpyAsync(status, h->d_status, n_prev, hipMemcpyDeviceToHost, s);
  if (hipStreamSynchronize(s) != hipSuccess) return kfail(SFM_EIO, "optical flow kernels failed");
  if (m > 0) {
    if (hipMemcpy(prev_idx, h->d_out, sizeof(int) * m, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(curr_idx, h->d_out + n_prev, sizeof(int) * m, hipMemcpyDeviceToHost) != hipSuccess)
      return kfail(SFM_EIO, "copy failed");
  }
  *n_matches = m;
  h->timed_flow = true;
  h->timed_assoc = n_curr > 0;
  return 0;
}

int sfm_klt_phase_times(sfm_klt_handle* h, double* ms3) {
  if (!h || !ms3) return kfail(SFM_EINVAL, "NULL argument");
  hipSetDevice(h->device);
  hipStreamSynchronize(h->stream);
  ms3[0] = h->timed_push ? ms_between(h->ev[0], h->ev[1]) : 0.0;
  ms3[1] = h->timed_flow ? ms_between(h->ev[2], h->ev[3]) : 0.0;
  ms3[2] = h->timed_assoc ? ms_between(h->ev[3], h->ev[5]) : 0.0;
  return 0;
}

int sfm_calc_optical_flow_pyr_lk(int32_t device, const uint8_t* prev, const uint8_t* next, int32_t width,
                                 int32_t height, const float* prev_pts, int32_t n, float* next_pts, uint8_t* status,
                                 const sfm_klt_params* params) {
  sfm_klt_handle* h = nullptr;
  if (int rc = sfm_klt_create(device, width, height, params, &h)) return rc;
  int rc = sfm_klt_push_frame(h, prev, width);
  if (!rc) rc = sfm_klt_push_frame(h, next, width);
  if (!rc) rc = sfm_klt_calc_flow(h, prev_pts, n, next_pts, status);
  sfm_klt_destroy(h);
  return rc;
}

}  // extern "C"

int sfm_internal_klt_frame(sfm_klt_handle* h, KltFrame* out) {
  if (!h || !out) return kfail(SFM_EINVAL, "NULL argument");
  if (h->n_frames == 0) return kfail(SFM_EINVAL, "no frame pushed");
  hipSetDevice(h->device);
  out->img = h->img[h->cur] + h->img_off[0];
  out->w = h->lw[0];
  out->h = h->lh[0];
  out->stream = h->stream;
  out->gftt_slot = &h->gftt;
  return 0;
}
