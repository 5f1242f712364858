// Corner detector of the optical-flow tracker for gfx950.
//
// Replaces CTracker::detectFeaturesOpticalFlow (/root/reference/CTracker.cpp:
// 252-272): goodFeaturesToTrack(grey, pts, 500, 0.05, 10) followed by
// cornerSubPix(grey, pts, Size(5,5), Size(-1,-1), TermCriteria(COUNT|EPS,
// 20, 0.03)), on the current frame already resident in HBM in the KLT
// handle (sfm_klt_push_frame).  Arithmetic follows oracle/gftt_oracle.cpp op
// for op with contraction off, so results are bit-exact against it.
//
// Pipeline (one stream, one host sync for the candidate count):
//   k_min_eig   64x16 output tile per workgroup: frame patch staged in LDS
//               (interior tiles), Sobel products of the (66x18) halo,
//               direct 3x3 box sums, min eigenvalue;
//               frame maximum by an ordered-uint atomicMax.
//   k_cand      threshold TOZERO + 3x3 dilate + local-max test per interior
//               pixel; candidates append (value bits << 32 | raster index)
//               keys (append order is irrelevant: the keys are unique).
//   radix sort  hipcub, keys descending = response descending, ties ->
//               larger raster index (OpenCV greaterThanPtr).
//   k_select    one 1024-thread workgroup: the greedy min-distance pass in
//               batches of 1024 sorted candidates: each is first tested
//               against the corners already accepted, then the batch's own
//               conflicts are settled in rounds (a candidate is accepted
//               once every higher-priority conflicting candidate is
//               rejected, rejected once one is accepted -- decisions are
//               final, so the result is exactly the sequential greedy one);
//               stops at max_corners.
//   k_subpix    one wavefront per corner: 13x13 bilinear resample (3 taps
//               per lane), per-pixel normal-equation terms, the fixed
//               lane order + xor-butterfly double sums of the oracle; every
//               lane then holds the same sums and steps identically.
// The frame is 0.92 MB at 1280x720 (L2-resident); the work is latency and
// launch bound, not HBM bound.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <string>
#include <vector>
#include "../../include/sfm_amd.h"
#include "klt_internal.h"

void sfm_internal_set_error(const std::string& msg);  // ba_solver.hip

namespace {

constexpr int kTX = 64, kTY = 16;      // k_min_eig output tile (256 threads, 4 pixels each)
constexpr int kEigThreads = 256;
constexpr int kBatch = 1024;           // k_select batch (= workgroup size)
constexpr int kMaxCorners = 4096;      // LDS list of accepted corners
constexpr int kMaxCells = 4096;        // k_select cell grids (LDS)
constexpr int kMaxWin = 7;             // cornerSubPix half window
constexpr int kMaxSub = (2 * kMaxWin + 3) * (2 * kMaxWin + 3);

int gfail(int code, const std::string& m) {
  sfm_internal_set_error(m);
  return code;
}

__device__ __forceinline__ int r101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
  }
  return i;
}

// float <-> order-preserving uint (for atomicMax over signed floats)
__device__ __forceinline__ unsigned int ord_of(float f) {
  const unsigned int b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float float_of_ord(unsigned int o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

__global__ __launch_bounds__(kEigThreads) void k_min_eig(const uint8_t* __restrict__ img, int w, int h,
                                                        float* __restrict__ eig, unsigned int* __restrict__ max_ord) {
  constexpr int HX = kTX + 2, HY = kTY + 2, IX = kTX + 4, IY = kTY + 4;
  __shared__ int pix[IY][IX];
  __shared__ float cxx[HY][HX], cxy[HY][HX], cyy[HY][HX];
  __shared__ float rxx[HY][kTX], rxy[HY][kTX], ryy[HY][kTX];
  __shared__ unsigned int red[kEigThreads / 64];
  const int x0 = blockIdx.x * kTX, y0 = blockIdx.y * kTY, t = threadIdx.x;
  const double scale = 1.0 / (4.0 * 3.0 * 255.0);
  // interior tiles: the (kTX+4) x (kTY+4) frame patch staged in LDS, no
  // reflection anywhere; border tiles read the frame through reflect-101
  const bool inner = x0 >= 2 && y0 >= 2 && x0 + kTX + 2 <= w && y0 + kTY + 2 <= h;
  if (inner) {
    for (int q = t; q < IX * IY; q += kEigThreads) {
      const int iy = q / IX, ix = q % IX;
      pix[iy][ix] = img[size_t(y0 - 2 + iy) * w + (x0 - 2 + ix)];
    }
    __syncthreads();
  }
  // Sobel products at the halo positions, each taken at its reflect-101
  // position (the box filter's border is in the products' coordinates)
  for (int q = t; q < HX * HY; q += kEigThreads) {
    const int hy = q / HX, hx = q % HX;
    int dx, dy;
    if (inner) {
      const int* rm = pix[hy];
      const int* rc = pix[hy + 1];
      const int* rp = pix[hy + 2];
      const int xm = hx, xc = hx + 1, xp = hx + 2;
      dx = (rm[xp] - rm[xm]) + 2 * (rc[xp] - rc[xm]) + (rp[xp] - rp[xm]);
      dy = (rp[xm] - rm[xm]) + 2 * (rp[xc] - rm[xc]) + (rp[xp] - rm[xp]);
    } else {
      const int x = r101(x0 + hx - 1, w), y = r101(y0 + hy - 1, h);
      const int xm = r101(x - 1, w), xp = r101(x + 1, w), ym = r101(y - 1, h), yp = r101(y + 1, h);
      const uint8_t* rm = img + size_t(ym) * w;
      const uint8_t* rc = img + size_t(y) * w;
      const uint8_t* rp = img + size_t(yp) * w;
      dx = (int(rm[xp]) - int(rm[xm])) + 2 * (int(rc[xp]) - int(rc[xm])) + (int(rp[xp]) - int(rp[xm]));
      dy = (int(rp[xm]) - int(rm[xm])) + 2 * (int(rp[x]) - int(rm[x])) + (int(rp[xp]) - int(rm[xp]));
    }
    const float ix = float(double(dx) * scale), iy = float(double(dy) * scale);
    cxx[hy][hx] = ix * ix;
    cxy[hy][hx] = ix * iy;
    cyy[hy][hx] = iy * iy;
  }
  __syncthreads();
  for (int q = t; q < HY * kTX; q += kEigThreads) {
    const int hy = q / kTX, ox = q % kTX;
    rxx[hy][ox] = (cxx[hy][ox] + cxx[hy][ox + 1]) + cxx[hy][ox + 2];
    rxy[hy][ox] = (cxy[hy][ox] + cxy[hy][ox + 1]) + cxy[hy][ox + 2];
    ryy[hy][ox] = (cyy[hy][ox] + cyy[hy][ox + 1]) + cyy[hy][ox + 2];
  }
  __syncthreads();
  unsigned int mo = 0u;
  for (int q = t; q < kTX * kTY; q += kEigThreads) {
    const int ox = q % kTX, oy = q / kTX, x = x0 + ox, y = y0 + oy;
    if (x < w && y < h) {
      const float sxx = (rxx[oy][ox] + rxx[oy + 1][ox]) + rxx[oy + 2][ox];
      const float sxy = (rxy[oy][ox] + rxy[oy + 1][ox]) + rxy[oy + 2][ox];
      const float syy = (ryy[oy][ox] + ryy[oy + 1][ox]) + ryy[oy + 2][ox];
      const float A = sxx * 0.5f, B = sxy, C = syy * 0.5f;
      const float e = (A + C) - __fsqrt_rn((A - C) * (A - C) + B * B);
      eig[size_t(y) * w + x] = e;
      mo = max(mo, ord_of(e));
    }
  }
  for (int off = 32; off >= 1; off >>= 1) mo = max(mo, __shfl_xor(mo, off));
  if ((t & 63) == 0) red[t >> 6] = mo;
  __syncthreads();
  if (t == 0) {
    unsigned int m = red[0];
    for (int i = 1; i < kEigThreads / 64; ++i) m = max(m, red[i]);
    atomicMax(max_ord, m);
  }
}

// 64x64 pixels per 256-thread workgroup (16 per thread), one atomic per
// workgroup: one counter hit once per wavefront still serialised ~14k
// atomics (~12 ns each) on textured frames.
constexpr int kCandT = 64;
__global__ __launch_bounds__(256) void k_cand(const float* __restrict__ eig, int w, int h,
                                              const unsigned int* __restrict__ max_ord, double quality,
                                              unsigned long long* __restrict__ keys, int* __restrict__ count) {
  __shared__ int wcnt[4];
  __shared__ int s_base;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int x = blockIdx.x * kCandT + lane, yb = blockIdx.y * kCandT + wv;
  const float thr = float(double(float_of_ord(*max_ord)) * quality);
  auto T = [&](int xx, int yy) {
    const float v = eig[size_t(yy) * w + xx];
    return v > thr ? v : 0.0f;
  };
  unsigned int mine = 0u;  // bit k: row yb + 4k holds a candidate
  float val[kCandT / 4];
#pragma unroll
  for (int k = 0; k < kCandT / 4; ++k) {
    const int y = yb + 4 * k;
    val[k] = 0.0f;
    if (x >= 1 && y >= 1 && x < w - 1 && y < h - 1) {
      const float v = T(x, y);
      if (v != 0.0f) {
        float d = v;
        for (int yy = y - 1; yy <= y + 1; ++yy)
          for (int xx = x - 1; xx <= x + 1; ++xx) d = fmaxf(d, T(xx, yy));
        if (v == d) {
          mine |= 1u << k;
          val[k] = v;
        }
      }
    }
  }
  const int c = __popc(mine);
  int incl = c;
  for (int off = 1; off < 64; off <<= 1) {
    const int v = __shfl_up(incl, off);
    if (lane >= off) incl += v;
  }
  if (lane == 63) wcnt[wv] = incl;
  __syncthreads();
  if (t == 0) {
    const int tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    s_base = tot ? atomicAdd(count, tot) : 0;
  }
  __syncthreads();
  int slot = s_base + incl - c;
  for (int k = 0; k < wv; ++k) slot += wcnt[k];
#pragma unroll
  for (int k = 0; k < kCandT / 4; ++k)
    if (mine & (1u << k))
      keys[slot++] = (static_cast<unsigned long long>(__float_as_uint(val[k])) << 32) |
                     unsigned((yb + 4 * k) * w + x);
}

// Greedy min-distance selection over the sorted keys (see file header).
// Conflicts are found through two cell grids in LDS (accepted corners and
// the current batch): cells are at least min_distance wide, so every pair
// closer than min_distance lies in the same or an adjacent cell.
__global__ __launch_bounds__(kBatch) void k_select(const unsigned long long* __restrict__ keys, int n, int w,
                                                  int max_corners, double md2, int use_dist, int cs, int gw,
                                                  int gh, float2* __restrict__ out, int* __restrict__ n_out) {
  __shared__ short ax[kMaxCorners], ay[kMaxCorners], anext[kMaxCorners];
  __shared__ short bx[kBatch], by[kBatch], bnext[kBatch];
  __shared__ int ahead[kMaxCells], bhead[kMaxCells];
  __shared__ unsigned char st[kBatch];   // 0 undecided, 1 accepted, 2 rejected / absent
  __shared__ int wsum[kBatch / 64];
  __shared__ int s_flag, s_nacc;
  const int i = threadIdx.x, lane = i & 63, wv = i >> 6;
  const int ncell = gw * gh;
  for (int c = i; c < ncell; c += kBatch) ahead[c] = -1;
  if (i == 0) s_nacc = 0;
  __syncthreads();
  for (int base = 0; base < n; base += kBatch) {
    const int nacc = s_nacc;
    if (nacc >= max_corners) break;
    for (int c = i; c < ncell; c += kBatch) bhead[c] = -1;
    const bool valid = base + i < n;
    int x = 0, y = 0;
    if (valid) {
      const int lin = int(unsigned(keys[base + i]));
      y = lin / w;
      x = lin - y * w;
    }
    const int gx = x / cs, gy = y / cs;
    bx[i] = short(x);
    by[i] = short(y);
    auto conflict = [&](int xx, int yy) {
      const int dx = x - xx, dy = y - yy;
      return double(dx * dx + dy * dy) < md2;
    };
    unsigned char sv = valid ? 0 : 2;
    if (valid && use_dist)
      for (int cy = max(gy - 1, 0); cy <= min(gy + 1, gh - 1) && sv == 0; ++cy)
        for (int cx = max(gx - 1, 0); cx <= min(gx + 1, gw - 1) && sv == 0; ++cx)
          for (int j = ahead[cy * gw + cx]; j >= 0; j = anext[j])
            if (conflict(ax[j], ay[j])) { sv = 2; break; }
    st[i] = sv;
    __syncthreads();  // bhead cleared, st / bx / by written
    if (sv == 0 && use_dist) bnext[i] = short(atomicExch(&bhead[gy * gw + gx], i));
    __syncthreads();
    for (;;) {
      if (i == 0) s_flag = 0;
      __syncthreads();
      if (st[i] == 0) {
        bool any_acc = false, all_rej = true;
        if (use_dist)
          for (int cy = max(gy - 1, 0); cy <= min(gy + 1, gh - 1); ++cy)
            for (int cx = max(gx - 1, 0); cx <= min(gx + 1, gw - 1); ++cx)
              for (int j = bhead[cy * gw + cx]; j >= 0; j = bnext[j])
                if (j < i && conflict(bx[j], by[j])) {
                  const unsigned char sj = st[j];
                  any_acc |= sj == 1;
                  all_rej &= sj == 2;
                }
        if (any_acc) st[i] = 2;
        else if (all_rej) st[i] = 1;
        else s_flag = 1;  // still undecided
      }
      __syncthreads();
      if (!s_flag) break;
    }
    // accepted corners of the batch in priority order, up to max_corners
    const int acc = st[i] == 1 ? 1 : 0;
    int incl = acc;
    for (int off = 1; off < 64; off <<= 1) {
      const int v = __shfl_up(incl, off);
      if (lane >= off) incl += v;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int before = 0, tot = 0;
    for (int k = 0; k < kBatch / 64; ++k) {
      if (k < wv) before += wsum[k];
      tot += wsum[k];
    }
    const int rank = nacc + before + incl - acc;
    if (acc && rank < max_corners) {
      ax[rank] = short(x);
      ay[rank] = short(y);
      out[rank] = make_float2(float(x), float(y));
      if (use_dist) anext[rank] = short(atomicExch(&ahead[gy * gw + gx], rank));
    }
    __syncthreads();
    if (i == 0) s_nacc = min(max_corners, nacc + tot);
    __syncthreads();
  }
  if (i == 0) *n_out = s_nacc;
}

// cornerSubPix, one wavefront per corner (see file header).
__global__ __launch_bounds__(64) void k_subpix(const uint8_t* __restrict__ img, int w, int h,
                                               const float* __restrict__ mask, int win, int max_iter, double eps2,
                                               const int* __restrict__ n_pts, float2* __restrict__ pts) {
  __shared__ float sub[kMaxSub];
  const int p = blockIdx.x, L = threadIdx.x;
  if (p >= *n_pts) return;
  const int ww = 2 * win + 1, sw = ww + 2, nk = ww * ww, ns = sw * sw;
  const float2 t0 = pts[p];
  float cx = t0.x, cy = t0.y;
  auto px = [&](int x, int y) {
    x = min(max(x, 0), w - 1);
    y = min(max(y, 0), h - 1);
    return float(img[size_t(y) * w + x]);
  };
  int iter = 0;
  for (;;) {
    const float ox = cx - float(sw - 1) * 0.5f, oy = cy - float(sw - 1) * 0.5f;
    const int ix = int(floorf(ox)), iy = int(floorf(oy));
    const float a = ox - float(ix), b = oy - float(iy);
    const float a11 = (1.f - a) * (1.f - b), a12 = a * (1.f - b), a21 = (1.f - a) * b, a22 = a * b;
    for (int k = L; k < ns; k += 64) {
      const int i = k / sw, j = k - i * sw, X = ix + j, Y = iy + i;
      sub[k] = ((px(X, Y) * a11 + px(X + 1, Y) * a12) + px(X, Y + 1) * a21) + px(X + 1, Y + 1) * a22;
    }
    __syncthreads();
    double v[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    for (int k = L; k < nk; k += 64) {
      const int i = k / ww, j = k - i * ww;
      const float* s = sub + (i + 1) * sw + 1;
      const double m = mask[k];
      const double tgx = double(s[j + 1] - s[j - 1]);
      const double tgy = double(s[j + sw] - s[j - sw]);
      const double gxx = tgx * tgx * m, gxy = tgx * tgy * m, gyy = tgy * tgy * m;
      const double pxx = double(j - win), py = double(i - win);
      const double tt[5] = {gxx, gxy, gyy, gxx * pxx + gxy * py, gxy * pxx + gyy * py};
      if (k == L) {
        for (int e = 0; e < 5; ++e) v[e] = tt[e];
      } else {
        for (int e = 0; e < 5; ++e) v[e] = v[e] + tt[e];
      }
    }
    for (int off = 32; off >= 1; off >>= 1)
      for (int e = 0; e < 5; ++e) v[e] = v[e] + __shfl_xor(v[e], off);
    __syncthreads();  // sub is rewritten next iteration
    const double A = v[0], B = v[1], C = v[2], bb1 = v[3], bb2 = v[4];
    const double det = A * C - B * B;
    if (fabs(det) <= DBL_EPSILON * DBL_EPSILON) break;
    const double sc = 1.0 / det;
    const float nx = float(double(cx) + C * sc * bb1 - B * sc * bb2);
    const float ny = float(double(cy) - B * sc * bb1 + A * sc * bb2);
    const double err = double((nx - cx) * (nx - cx) + (ny - cy) * (ny - cy));
    cx = nx;
    cy = ny;
    if (cx < 0 || cx >= float(w) || cy < 0 || cy >= float(h)) break;
    if (!(++iter < max_iter && err > eps2)) break;
  }
  if (fabsf(cx - t0.x) > float(win) || fabsf(cy - t0.y) > float(win)) {
    cx = t0.x;
    cy = t0.y;
  }
  if (L == 0) pts[p] = make_float2(cx, cy);
}

// Per-handle device state (lives in the KLT handle, freed with it).
struct GfttState {
  int w = 0, h = 0;
  float* eig = nullptr;
  unsigned long long* keys = nullptr;
  unsigned long long* keys_sorted = nullptr;
  int* ints = nullptr;              // [0] max_ord, [1] candidate count, [2] corner count
  float2* corners = nullptr;        // [kMaxCorners]
  float* mask = nullptr;            // [(2 kMaxWin + 1)^2]
  void* sort_tmp = nullptr;
  size_t sort_tmp_bytes = 0;
  hipEvent_t ev[2] = {};
};

void free_state(GfttState* g) {
  if (!g) return;
  void* bufs[] = {g->eig, g->keys, g->keys_sorted, g->ints, g->corners, g->mask, g->sort_tmp};
  for (void* b : bufs)
    if (b) hipFree(b);
  for (auto& e : g->ev)
    if (e) hipEventDestroy(e);
  delete g;
}

int ensure_state(void** slot, int w, int h) {
  auto* g = static_cast<GfttState*>(*slot);
  if (g && g->w == w && g->h == h) return 0;
  free_state(g);
  *slot = nullptr;
  g = new GfttState();
  g->w = w;
  g->h = h;
  const size_t npx = size_t(w) * h;
  bool ok = hipMalloc(&g->eig, npx * sizeof(float)) == hipSuccess &&
            hipMalloc(&g->keys, npx * sizeof(unsigned long long)) == hipSuccess &&
            hipMalloc(&g->keys_sorted, npx * sizeof(unsigned long long)) == hipSuccess &&
            hipMalloc(&g->ints, 4 * sizeof(int)) == hipSuccess &&
            hipMalloc(&g->corners, kMaxCorners * sizeof(float2)) == hipSuccess &&
            hipMalloc(&g->mask, (2 * kMaxWin + 1) * (2 * kMaxWin + 1) * sizeof(float)) == hipSuccess;
  if (ok) {
    hipcub::DeviceRadixSort::SortKeysDescending(nullptr, g->sort_tmp_bytes, g->keys, g->keys_sorted, int(npx));
    ok = hipMalloc(&g->sort_tmp, std::max<size_t>(g->sort_tmp_bytes, 16)) == hipSuccess &&
         hipEventCreate(&g->ev[0]) == hipSuccess && hipEventCreate(&g->ev[1]) == hipSuccess;
  }
  if (!ok) {
    free_state(g);
    return gfail(SFM_ENOMEM, "hipMalloc failed (gftt state)");
  }
  *slot = g;
  return 0;
}

// cornerSubPix's Gaussian window, on the host with the C library's expf
// (the oracle's too), so the device weights are the oracle's bit for bit.
std::vector<float> subpix_mask(int win) {
  const int ww = 2 * win + 1;
  std::vector<float> m(size_t(ww) * ww);
  for (int i = 0; i < ww; ++i) {
    volatile float y = float(i - win) / float(win);
    const float vy = std::exp(-y * y);
    for (int j = 0; j < ww; ++j) {
      volatile float x = float(j - win) / float(win);
      m[size_t(i) * ww + j] = vy * std::exp(-x * x);
    }
  }
  return m;
}

}  // namespace

void sfm_internal_gftt_free(void* state) { free_state(static_cast<GfttState*>(state)); }

extern "C" {

void sfm_gftt_default_params(sfm_gftt_params* p) {
  p->max_corners = 500;
  p->subpix_win = 5;
  p->subpix_max_iter = 20;
  p->min_features = 5;
  p->quality_level = 0.05;
  p->min_distance = 10.0;
  p->subpix_epsilon = 0.03;
}

int sfm_klt_detect_features(sfm_klt_handle* kh, const sfm_gftt_params* params, float* pts, int32_t capacity,
                            int32_t* n_pts) {
  if (!kh || !pts || !n_pts) return gfail(SFM_EINVAL, "NULL argument");
  sfm_gftt_params prm;
  if (params) prm = *params;
  else sfm_gftt_default_params(&prm);
  if (prm.max_corners < 1 || prm.max_corners > kMaxCorners)
    return gfail(SFM_ENOTSUP, "max_corners must be in [1, 4096]");
  if (capacity < prm.max_corners) return gfail(SFM_EINVAL, "capacity < max_corners");
  if (prm.subpix_win < 0 || prm.subpix_win > kMaxWin) return gfail(SFM_ENOTSUP, "subpix_win must be in [0, 7]");
  if (!(prm.quality_level > 0.0) || !(prm.min_distance >= 0.0)) return gfail(SFM_EINVAL, "bad quality / distance");
  KltFrame f{};
  int rc = sfm_internal_klt_frame(kh, &f);
  if (rc) return rc;
  if (f.w < 3 || f.h < 3) return gfail(SFM_EINVAL, "frame smaller than 3x3");
  if ((rc = ensure_state(f.gftt_slot, f.w, f.h))) return rc;
  auto* g = static_cast<GfttState*>(*f.gftt_slot);
  hipStream_t s = f.stream;
  const std::vector<float> mask = subpix_mask(std::max(prm.subpix_win, 1));
  hipEventRecord(g->ev[0], s);
  hipMemsetAsync(g->ints, 0, 4 * sizeof(int), s);
  hipMemcpyAsync(g->mask, mask.data(), mask.size() * sizeof(float), hipMemcpyHostToDevice, s);
  dim3 ge((f.w + kTX - 1) / kTX, (f.h + kTY - 1) / kTY);
  k_min_eig<<<ge, kEigThreads, 0, s>>>(f.img, f.w, f.h, g->eig, reinterpret_cast<unsigned int*>(g->ints));
  dim3 gc((f.w + kCandT - 1) / kCandT, (f.h + kCandT - 1) / kCandT);
  k_cand<<<gc, 256, 0, s>>>(g->eig, f.w, f.h, reinterpret_cast<unsigned int*>(g->ints), prm.quality_level, g->keys,
                            g->ints + 1);
  int n_cand = 0;
  if (hipMemcpyAsync(&n_cand, g->ints + 1, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return gfail(SFM_EIO, "corner response failed");
  if (n_cand > 0) {
    size_t tmp = g->sort_tmp_bytes;
    if (hipcub::DeviceRadixSort::SortKeysDescending(g->sort_tmp, tmp, g->keys, g->keys_sorted, n_cand, 0, 64, s) !=
        hipSuccess)
      return gfail(SFM_EIO, "candidate sort failed");
    // cells at least min_distance wide and few enough for LDS
    int cs = std::max(1, int(std::ceil(prm.min_distance)));
    while (size_t((f.w + cs - 1) / cs) * size_t((f.h + cs - 1) / cs) > size_t(kMaxCells)) ++cs;
    const int gw = (f.w + cs - 1) / cs, gh = (f.h + cs - 1) / cs;
    k_select<<<1, kBatch, 0, s>>>(g->keys_sorted, n_cand, f.w, prm.max_corners,
                                  prm.min_distance * prm.min_distance, prm.min_distance >= 1.0 ? 1 : 0, cs, gw, gh,
                                  g->corners, g->ints + 2);
    const int max_iter = std::min(std::max(prm.subpix_max_iter, 1), 100);
    const double e = std::max(prm.subpix_epsilon, 0.0);
    if (prm.subpix_win > 0)
      k_subpix<<<prm.max_corners, 64, 0, s>>>(f.img, f.w, f.h, g->mask, prm.subpix_win, max_iter, e * e, g->ints + 2,
                                            g->corners);
  }
  hipEventRecord(g->ev[1], s);
  int n = 0;
  if (hipGetLastError() != hipSuccess) return gfail(SFM_EIO, "corner detector launch failed");
  if (hipMemcpyAsync(&n, g->ints + 2, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return gfail(SFM_EIO, "corner detector failed");
  if (n > 0 && hipMemcpy(pts, g->corners, size_t(n) * sizeof(float2), hipMemcpyDeviceToHost) != hipSuccess)
    return gfail(SFM_EIO, "corner download failed");
  *n_pts = n;
  return 0;
}

int sfm_klt_detect_time(sfm_klt_handle* kh, double* ms) {
  if (!kh || !ms) return gfail(SFM_EINVAL, "NULL argument");
  KltFrame f{};
  int rc = sfm_internal_klt_frame(kh, &f);
  if (rc) return rc;
  auto* g = static_cast<GfttState*>(*f.gftt_slot);
  float v = 0.f;
  *ms = (g && hipEventElapsedTime(&v, g->ev[0], g->ev[1]) == hipSuccess) ? double(v) : 0.0;
  return 0;
}

int sfm_good_features_to_track(int32_t device, const uint8_t* grey, int32_t width, int32_t height, int32_t stride,
                               const sfm_gftt_params* params, float* pts, int32_t capacity, int32_t* n_pts) {
  sfm_klt_params kp;
  sfm_klt_default_params(&kp);
  kp.max_level = 0;
  sfm_klt_handle* kh = nullptr;
  int rc = sfm_klt_create(device, width, height, &kp, &kh);
  if (rc) return rc;
  rc = sfm_klt_push_frame(kh, grey, stride);
  if (!rc) rc = sfm_klt_detect_features(kh, params, pts, capacity, n_pts);
  sfm_klt_destroy(kh);
  return rc;
}

}  // extern "C"
