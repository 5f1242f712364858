// CMap's observation store on the device: the map
// points, their (frame, keypoint) observations and their descriptor rows,
// resident in HBM, with the queries the live tracking path makes of CMap:
//
//   addNewPoints       CMap.cpp:36-78   points + one observation per frame,
//                                       emplaced point-major (i, then j)
//   addPointMatches    CMap.cpp:118-132 one observation per point
//   addDescriptors     CMap.cpp:308-315 one descriptor row per point
//   getPointsAtIdx     CMap.cpp:134-143 (and the BA write-back)
//   getPointsInFrames  CMap.cpp:277-295 sorted unique points seen in any of
//                                       the frames (CSfM.cpp:648)
//   getPointsInFrame   CMap.cpp:145-240 multimap equal_range order; for
//                                       every entry, EVERY 2D index the point
//                                       has in that frame (a point matched
//                                       twice in a frame yields 2 x 2)
//   getRepresentativeDescriptors  CMap.cpp:345-381 (CSfM.cpp:669)
//
// Layout: observations are kept in global emplace order, which is taken as
// the multimap's order within one key (the reference's container is an
// unordered_multimap, CMap.h:96-97, whose equal_range order is
// implementation-defined; libc++, the reference's toolchain, keeps insertion
// order) and is the order of each point's _frameNo/_pts2DIdx lists.  Descriptor rows are kept in append order with their point.  The
// per-point CSRs (observations, descriptor rows) are rebuilt lazily by a
// stable radix sort after appends.  Queries are flag + stable compaction
// (hipcub DeviceSelect), so every result keeps the reference's order.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <climits>
#include <cstring>
#include <map>
#include <string>
#include <vector>
#include "sfm_trace.h"
#include "../../include/sfm_amd.h"

void sfm_internal_set_error(const std::string& msg);  // ba_solver.hip

namespace sfm {
namespace {

int mapfail(int code, const std::string& m) {
  sfm_internal_set_error("sfm_map: " + m);
  return code;
}

__global__ void k_mark_frames(int64_t n, const int32_t* __restrict__ ob_pt, const int32_t* __restrict__ ob_frame,
                              const int32_t* __restrict__ fset, int nf, uint8_t* __restrict__ mark) {
  const int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int f = ob_frame[e];
  int lo = 0, hi = nf;  // fset ascending
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (fset[mid] < f) lo = mid + 1; else hi = mid;
  }
  if (lo < nf && fset[lo] == f) mark[ob_pt[e]] = 1;  // idempotent plain store
}

__global__ void k_flag_frame(int64_t n, const int32_t* __restrict__ ob_frame, int f, uint8_t* __restrict__ flag) {
  const int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e < n) flag[e] = ob_frame[e] == f;
}

// rank of each observation's frame in the query list (fr sorted by frame,
// with the query position alongside), nf when the frame is not queried
__global__ void k_frame_rank(int64_t n, const int32_t* __restrict__ ob_frame, const int2* __restrict__ fr, int nf,
                             uint32_t* __restrict__ key, int32_t* __restrict__ iota) {
  const int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int f = ob_frame[e];
  int lo = 0, hi = nf;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (fr[mid].x < f) lo = mid + 1; else hi = mid;
  }
  key[e] = uint32_t(lo < nf && fr[lo].x == f ? fr[lo].y : nf);
  iota[e] = int32_t(e);
}

__global__ void k_count_keys(int64_t n, const int32_t* __restrict__ key, int32_t* __restrict__ cnt) {
  const int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e < n) atomicAdd(cnt + key[e], 1);
}

__global__ void k_iota(int64_t n, int32_t* __restrict__ v) {
  const int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e < n) v[e] = int32_t(e);
}

// entry e of the frame's equal range (observation sel[e] of point p): how
// many of p's observations are in frame f
__global__ void k_dup_count(int n_sel, const int32_t* __restrict__ sel, const int32_t* __restrict__ ob_pt,
                            const int32_t* __restrict__ ob_frame, const int32_t* __restrict__ orow,
                            const int32_t* __restrict__ ooff, int f, int32_t* __restrict__ cnt) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_sel) return;
  const int p = ob_pt[sel[e]];
  const int fe = f == INT32_MIN ? ob_frame[sel[e]] : f;  // INT32_MIN: the entry's own frame (multi-frame query)
  int c = 0;
  for (int q = ooff[p]; q < ooff[p + 1]; ++q) c += ob_frame[orow[q]] == fe;
  cnt[e] = c;
}

__global__ void k_dup_fill(int n_sel, const int32_t* __restrict__ sel, const int32_t* __restrict__ ob_pt,
                           const int32_t* __restrict__ ob_frame, const int32_t* __restrict__ ob_idx,
                           const int32_t* __restrict__ orow, const int32_t* __restrict__ ooff, int f,
                           const int32_t* __restrict__ off2, int32_t* __restrict__ out3, int32_t* __restrict__ out2) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_sel) return;
  const int p = ob_pt[sel[e]];
  const int fe = f == INT32_MIN ? ob_frame[sel[e]] : f;
  out3[e] = p;
  int w = off2[e];
  for (int q = ooff[p]; q < ooff[p + 1]; ++q) {
    const int o = orow[q];
    if (ob_frame[o] == fe) out2[w++] = ob_idx[o];
  }
}

// k_dup_count over the rank-sorted observations of a multi-frame query:
// entries of the queried frames (rank < nf) count their point's
// observations in their own frame, the rest 0
__global__ void k_dup_count_ranked(int64_t n, const int32_t* __restrict__ sel, const uint32_t* __restrict__ rank,
                                   int nf, const int32_t* __restrict__ ob_pt, const int32_t* __restrict__ ob_frame,
                                   const int32_t* __restrict__ orow, const int32_t* __restrict__ ooff,
                                   int32_t* __restrict__ cnt) {
  const int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= n) return;
  int c = 0;
  if (int(rank[e]) < nf) {
    const int o = sel[e], p = ob_pt[o], f = ob_frame[o];
    for (int q = ooff[p]; q < ooff[p + 1]; ++q) c += ob_frame[orow[q]] == f;
  }
  cnt[e] = c;
}

// the frames' entry offsets (exclusive scan of the per-rank counts) and 2D
// offsets (the entry scan at each frame's first entry): offs[0..nf] and
// offs[nf+1 .. 2nf+1]
__global__ void k_frame_offsets(int nf, const int32_t* __restrict__ fcnt, int64_t n, const int32_t* __restrict__ cnt,
                                const int32_t* __restrict__ eoff, int32_t* __restrict__ offs) {
  const int32_t total2 = n ? eoff[n - 1] + cnt[n - 1] : 0;
  int32_t o = 0;
  for (int i = 0; i <= nf; ++i) {
    offs[i] = o;
    offs[nf + 1 + i] = o < n ? eoff[o] : total2;
    if (i < nf) o += fcnt[i];
  }
}

// one wave per queried point: the point's row (in append order) with the
// smallest sum of Hamming distances to its other rows, the first on ties
// (CMap.cpp:345-381)
template <int W>
__global__ __launch_bounds__(64) void k_map_repr(const uint64_t* __restrict__ desc, const int32_t* __restrict__ drow,
                                                 const int32_t* __restrict__ doff, const int32_t* __restrict__ qpt,
                                                 int n, const int32_t* __restrict__ n_dev,
                                                 int32_t* __restrict__ best_local, uint64_t* __restrict__ out) {
  const int i = blockIdx.x, l = threadIdx.x;
  if (i >= (n_dev ? *n_dev : n)) return;  // (n_dev: the count on the device, n its bound)
  const int p = qpt[i];
  const int r0 = doff[p], k = doff[p + 1] - r0;
  if (k == 0) {  // no descriptor row (the callers check; reported as -1)
    if (l == 0) best_local[i] = -1;
    if (l < W) out[size_t(i) * W + l] = 0;
    return;
  }
  unsigned long long key = ~0ull;  // (sum << 32 | local row)
  for (int r = l; r - l < k; r += 64) {
    uint64_t x[W];
    const uint64_t* xr = desc + size_t(drow[r0 + (r < k ? r : 0)]) * W;
#pragma unroll
    for (int w = 0; w < W; ++w) x[w] = xr[w];
    unsigned int sum = 0;
    for (int q = 0; q < k; ++q) {
      const uint64_t* y = desc + size_t(drow[r0 + q]) * W;
#pragma unroll
      for (int w = 0; w < W; ++w) sum += __popcll(x[w] ^ y[w]);
    }
    if (r < k) key = min(key, (static_cast<unsigned long long>(sum) << 32) | unsigned(r));
  }
  for (int o = 32; o >= 1; o >>= 1) key = min(key, static_cast<unsigned long long>(__shfl_xor(key, o)));
  const int b = int(key & 0xffffffffu);
  if (l == 0) best_local[i] = b;
  if (l < W) out[size_t(i) * W + l] = desc[size_t(drow[r0 + b]) * W + l];
}

__global__ void k_scatter_points(int n, const int32_t* __restrict__ idx, const double* __restrict__ v,
                                 double* __restrict__ X) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const size_t p = size_t(idx[i]) * 3;
  X[p] = v[3 * size_t(i)];
  X[p + 1] = v[3 * size_t(i) + 1];
  X[p + 2] = v[3 * size_t(i) + 2];
}

inline unsigned grid(int64_t n, int b = 256) { return unsigned((n + b - 1) / b); }

__global__ void k_gather_points(int n, const int32_t* __restrict__ idx, const double* __restrict__ X,
                                double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const size_t p = size_t(idx[i]) * 3;
  out[3 * size_t(i)] = X[p];
  out[3 * size_t(i) + 1] = X[p + 1];
  out[3 * size_t(i) + 2] = X[p + 2];
}

__global__ void k_unmark(int n, const int32_t* __restrict__ pts, uint8_t* __restrict__ mark) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) mark[pts[i]] = 0;
}

// The queried points projected with the frame's pose (CSfM.cpp:664-668, the
// reference's GeometryUtils::projectPoints with zero distortion, as
// sfm_amd/live.py's _project): uv = (x / z) f + c.
__global__ void k_project(int n, const int32_t* __restrict__ n_dev, const int32_t* __restrict__ qpt,
                          const double* __restrict__ X, double r0, double r1,
                          double r2, double r3, double r4, double r5, double r6, double r7, double r8, double t0,
                          double t1, double t2, double fx, double fy, double cx, double cy, double* __restrict__ uv) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (n_dev ? *n_dev : n)) return;
  const double* x = X + 3 * size_t(qpt[i]);
  const double x0 = x[0], x1 = x[1], x2 = x[2];
  const double c0 = r0 * x0 + r1 * x1 + r2 * x2 + t0;
  const double c1 = r3 * x0 + r4 * x1 + r5 * x2 + t1;
  const double c2 = r6 * x0 + r7 * x1 + r8 * x2 + t2;
  uv[2 * size_t(i)] = c0 / c2 * fx + cx;
  uv[2 * size_t(i) + 1] = c1 / c2 * fy + cy;
}

template <class T>
struct DVec {
  T* p = nullptr;
  int64_t n = 0, cap = 0;
};

}  // namespace
// match_kernels.hip
int matcher_match_current_dev(sfm_matcher* h, hipEvent_t after, const uint64_t* q, const double* p0, int n0,
                              const int32_t* d_n0, const int32_t* d_train_idx, int n1, double ratio, double mn,
                              double mx, int** res);
int matcher_current_n(const sfm_matcher* h);
int matcher_words(const sfm_matcher* h);
int matcher_device(const sfm_matcher* h);
}  // namespace sfm

using namespace sfm;

struct sfm_map {
  int device = 0, desc_bytes = 0, W = 0;
  hipStream_t s = nullptr;
  DVec<int32_t> ob_pt, ob_frame, ob_idx;  // observations, emplace order
  DVec<double> X;                          // [n_pts][3]
  int32_t n_pts = 0;
  DVec<uint64_t> desc;                     // [rows][W]
  DVec<int32_t> desc_pt;                   // point of each row
  bool ocsr = false, dcsr = false;         // per-point CSRs current?
  int32_t *orow = nullptr, *ooff = nullptr, *drow = nullptr, *doff = nullptr;
  std::map<std::string, std::pair<void*, size_t>> scratch;
  hipEvent_t ev = nullptr;                 // sfm_map_match_frame: its queries are ready
  int32_t* pin = nullptr;                  // sfm_map_match_frame's pinned readback
  size_t pin_cap = 0;
};

namespace {

void* scratch(sfm_map* h, const char* name, size_t bytes, int* rc) {
  auto& e = h->scratch[name];
  if (e.second >= bytes && e.first) return e.first;
  // grow by half again at least: the map grows every keyframe, and a
  // reallocation costs a stream synchronisation plus hipFree / hipMalloc
  const size_t want = std::max<size_t>({bytes, e.second + e.second / 2, 256});
  if (e.first) { (void)hipStreamSynchronize(h->s); (void)hipFree(e.first); e.first = nullptr; e.second = 0; }
  void* p = nullptr;
  if (hipMalloc(&p, want) != hipSuccess) {
    *rc = mapfail(SFM_ENOMEM, std::string("hipMalloc failed (") + name + ")");
    return nullptr;
  }
  e = {p, want};
  return p;
}

template <class T>
int grow(sfm_map* h, DVec<T>& v, int64_t need) {
  if (need <= v.cap) return 0;
  const int64_t cap = std::max<int64_t>({need, 2 * v.cap, 1024});
  T* p = nullptr;
  if (hipMalloc(&p, size_t(cap) * sizeof(T)) != hipSuccess) return mapfail(SFM_ENOMEM, "hipMalloc failed (growth)");
  if (v.n) (void)hipMemcpyAsync(p, v.p, size_t(v.n) * sizeof(T), hipMemcpyDeviceToDevice, h->s);
  (void)hipStreamSynchronize(h->s);
  if (v.p) (void)hipFree(v.p);
  v.p = p;
  v.cap = cap;
  return 0;
}

template <class T>
int append(sfm_map* h, DVec<T>& v, const T* src, int64_t n) {
  if (int rc = grow(h, v, v.n + n)) return rc;
  if (n && hipMemcpyAsync(v.p + v.n, src, size_t(n) * sizeof(T), hipMemcpyHostToDevice, h->s) != hipSuccess)
    return mapfail(SFM_EIO, "upload failed");
  v.n += n;
  return 0;
}

// The handle's pinned block, at least n ints (grown while the stream is idle).
int32_t* pin_reserve(sfm_map* h, size_t n, int* rc) {
  if (h->pin_cap < n) {
    if (h->pin) { (void)hipStreamSynchronize(h->s); (void)hipHostFree(h->pin); }
    h->pin = nullptr;
    h->pin_cap = 0;
    const size_t cap = std::max<size_t>(n, 8192) * 3 / 2;
    if (hipHostMalloc(reinterpret_cast<void**>(&h->pin), sizeof(int32_t) * cap) != hipSuccess) {
      *rc = mapfail(SFM_ENOMEM, "hipHostMalloc failed");
      return nullptr;
    }
    h->pin_cap = cap;
  }
  return h->pin;
}
int sync(sfm_map* h) {
  return hipStreamSynchronize(h->s) == hipSuccess ? 0 : mapfail(SFM_EIO, "kernel or copy failed");
}

// CSR by point of `key` (n entries, keys < P): rows (entry ids grouped by
// key, ascending within a key = append order) and offsets [P+1]
int build_csr(sfm_map* h, const char* tag, const int32_t* key, int64_t n, int32_t** rows_out, int32_t** off_out) {
  int rc = 0;
  const int P = h->n_pts;
  std::string t(tag);
  auto* kk = static_cast<uint32_t*>(scratch(h, (t + "k").c_str(), sizeof(uint32_t) * std::max<int64_t>(n, 1), &rc));
  auto* iv = static_cast<int32_t*>(scratch(h, (t + "i").c_str(), sizeof(int32_t) * std::max<int64_t>(n, 1), &rc));
  auto* rows = static_cast<int32_t*>(scratch(h, (t + "r").c_str(), sizeof(int32_t) * std::max<int64_t>(n, 1), &rc));
  auto* cnt = static_cast<int32_t*>(scratch(h, (t + "c").c_str(), sizeof(int32_t) * (size_t(P) + 1), &rc));
  auto* off = static_cast<int32_t*>(scratch(h, (t + "o").c_str(), sizeof(int32_t) * (size_t(P) + 1), &rc));
  if (rc) return rc;
  (void)hipMemsetAsync(cnt, 0, sizeof(int32_t) * (size_t(P) + 1), h->s);
  if (n) {
    k_count_keys<<<grid(n), 256, 0, h->s>>>(n, key, cnt);
    k_iota<<<grid(n), 256, 0, h->s>>>(n, iv);
    int bits = 1;
    while (bits < 32 && (1ll << bits) < P) ++bits;
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, reinterpret_cast<const uint32_t*>(key), kk, iv, rows,
                                             int(n), 0, bits, h->s);
    void* tmp = scratch(h, (t + "t").c_str(), bytes, &rc);
    if (rc) return rc;
    if (hipcub::DeviceRadixSort::SortPairs(tmp, bytes, reinterpret_cast<const uint32_t*>(key), kk, iv, rows, int(n),
                                           0, bits, h->s) != hipSuccess)
      return mapfail(SFM_EIO, "radix sort failed");
  }
  size_t bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, cnt, off, P + 1, h->s);
  void* tmp = scratch(h, (t + "s").c_str(), bytes, &rc);
  if (rc) return rc;
  if (hipcub::DeviceScan::ExclusiveSum(tmp, bytes, cnt, off, P + 1, h->s) != hipSuccess)
    return mapfail(SFM_EIO, "scan failed");
  *rows_out = rows;
  *off_out = off;
  return 0;
}

int check_pts(const sfm_map* h, int32_t n, const int32_t* idx) {
  for (int32_t i = 0; i < n; ++i)
    if (idx[i] < 0 || idx[i] >= h->n_pts)
      return mapfail(SFM_EINVAL, "point index " + std::to_string(idx[i]) + " out of range at " + std::to_string(i));
  return 0;
}

}  // namespace

extern "C" {

int sfm_map_create(int32_t device, int32_t desc_bytes, sfm_map** out) {
  if (!out) return mapfail(SFM_EINVAL, "out is NULL");
  *out = nullptr;
  if (desc_bytes <= 0 || desc_bytes > 512 || desc_bytes % 8 || ((desc_bytes / 8) & (desc_bytes / 8 - 1)))
    return mapfail(SFM_EINVAL, "desc_bytes must be 8 x a power of two, <= 512 (BRISK: 64, ORB: 32)");
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || device < 0 || device >= nd) return mapfail(SFM_ENODEV, "no such device");
  if (hipSetDevice(device) != hipSuccess) return mapfail(SFM_ENODEV, "hipSetDevice failed");
  auto* h = new sfm_map;
  h->device = device;
  h->desc_bytes = desc_bytes;
  h->W = desc_bytes / 8;
  if (hipStreamCreateWithFlags(&h->s, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return mapfail(SFM_EIO, "hipStreamCreate failed");
  }
  *out = h;
  return 0;
}

int sfm_map_destroy(sfm_map* h) {
  if (!h) return 0;
  (void)hipSetDevice(h->device);
  (void)hipStreamSynchronize(h->s);
  for (void* p : {(void*)h->ob_pt.p, (void*)h->ob_frame.p, (void*)h->ob_idx.p, (void*)h->X.p, (void*)h->desc.p,
                  (void*)h->desc_pt.p})
    if (p) (void)hipFree(p);
  for (auto& e : h->scratch)
    if (e.second.first) (void)hipFree(e.second.first);
  if (h->ev) (void)hipEventDestroy(h->ev);
  if (h->pin) (void)hipHostFree(h->pin);
  (void)hipStreamDestroy(h->s);
  delete h;
  return 0;
}

int sfm_map_size(sfm_map* h, int32_t* n_pts, int64_t* n_obs, int64_t* n_desc_rows) {
  if (!h) return mapfail(SFM_EINVAL, "NULL handle");
  if (n_pts) *n_pts = h->n_pts;
  if (n_obs) *n_obs = h->ob_pt.n;
  if (n_desc_rows) *n_desc_rows = h->desc.n / h->W;
  return 0;
}

int sfm_map_add_new_points(sfm_map* h, int32_t n_pts, const double* pts3d, int32_t n_frames, const int32_t* frame_no,
                           const int32_t* pts2d_idx, int32_t* pts3d_idx) {
  SFM_TRACE("sfm_map_add_new_points");
  if (!h) return mapfail(SFM_EINVAL, "NULL handle");
  if (n_pts < 0 || n_frames < 0) return mapfail(SFM_EINVAL, "negative size");
  if (n_pts == 0) return 0;
  if (!pts3d || (n_frames && (!frame_no || !pts2d_idx))) return mapfail(SFM_EINVAL, "NULL argument");
  if (hipSetDevice(h->device) != hipSuccess) return mapfail(SFM_ENODEV, "hipSetDevice failed");
  // emplace order of CMap.cpp:50-68: point i, then its frames j
  const int64_t m = int64_t(n_pts) * n_frames;
  std::vector<int32_t> pt(m), fr(m), ix(m);
  for (int32_t i = 0; i < n_pts; ++i)
    for (int32_t j = 0; j < n_frames; ++j) {
      const int64_t e = int64_t(i) * n_frames + j;
      pt[e] = h->n_pts + i;
      fr[e] = frame_no[j];
      ix[e] = pts2d_idx[int64_t(j) * n_pts + i];
    }
  if (int rc = append(h, h->X, pts3d, int64_t(n_pts) * 3)) return rc;
  if (int rc = append(h, h->ob_pt, pt.data(), m)) return rc;
  if (int rc = append(h, h->ob_frame, fr.data(), m)) return rc;
  if (int rc = append(h, h->ob_idx, ix.data(), m)) return rc;
  if (pts3d_idx)
    for (int32_t i = 0; i < n_pts; ++i) pts3d_idx[i] = h->n_pts + i;
  h->n_pts += n_pts;
  h->ocsr = h->dcsr = false;
  return sync(h);
}

int sfm_map_add_point_matches(sfm_map* h, int32_t n, const int32_t* pts3d_idx, const int32_t* pts2d_idx,
                              int32_t frame_no) {
  if (!h) return mapfail(SFM_EINVAL, "NULL handle");
  if (n < 0) return mapfail(SFM_EINVAL, "negative size");
  if (n == 0) return 0;
  if (!pts3d_idx || !pts2d_idx) return mapfail(SFM_EINVAL, "NULL argument");
  if (int rc = check_pts(h, n, pts3d_idx)) return rc;
  if (hipSetDevice(h->device) != hipSuccess) return mapfail(SFM_ENODEV, "hipSetDevice failed");
  std::vector<int32_t> fr(size_t(n), frame_no);
  if (int rc = append(h, h->ob_pt, pts3d_idx, n)) return rc;
  if (int rc = append(h, h->ob_frame, fr.data(), n)) return rc;
  if (int rc = append(h, h->ob_idx, pts2d_idx, n)) return rc;
  h->ocsr = false;
  return sync(h);
}

int sfm_map_add_descriptors(sfm_map* h, int32_t n, const int32_t* pts3d_idx, const uint8_t* desc) {
  if (!h) return mapfail(SFM_EINVAL, "NULL handle");
  if (n < 0) return mapfail(SFM_EINVAL, "negative size");
  if (n == 0) return 0;
  if (!pts3d_idx || !desc) return mapfail(SFM_EINVAL, "NULL argument");
  if (int rc = check_pts(h, n, pts3d_idx)) return rc;
  if (hipSetDevice(h->device) != hipSuccess) return mapfail(SFM_ENODEV, "hipSetDevice failed");
  // rows are desc_bytes = 8 W bytes: copy as words (unaligned host bytes)
  std::vector<uint64_t> words(size_t(n) * h->W);
  std::memcpy(words.data(), desc, size_t(n) * h->desc_bytes);
  if (int rc = append(h, h->desc, words.data(), int64_t(n) * h->W)) return rc;
  if (int rc = append(h, h->desc_pt, pts3d_idx, n)) return rc;
  h->dcsr = false;
  return sync(h);
}

int sfm_map_get_points(sfm_map* h, int32_t n, const int32_t* pts3d_idx, double* pts3d) {
  SFM_TRACE("sfm_map_get_points");
  if (!h) return mapfail(SFM_EINVAL, "NULL handle");
  if (n <= 0) return n < 0 ? mapfail(SFM_EINVAL, "negative size") : 0;
  if (!pts3d_idx || !pts3d) return mapfail(SFM_EINVAL, "NULL argument");
  if (int rc = check_pts(h, n, pts3d_idx)) return rc;
  if (hipSetDevice(h->device) != hipSuccess) return mapfail(SFM_ENODEV, "hipSetDevice failed");
  // gathered on the device: the indices up, n points down (the whole X
  // array went down before: 140 KB per tracked frame at 6k points)
  int rc = 0;
  auto* di = static_cast<int32_t*>(scratch(h, "gi", sizeof(int32_t) * size_t(n), &rc));
  auto* dv = static_cast<double*>(scratch(h, "gv", sizeof(double) * 3 * size_t(n), &rc));
  if (rc) return rc;
  if (h->pin_cap < 8 * size_t(n) + 8) {
    if (h->pin) { (void)hipStreamSynchronize(h->s); (void)hipHostFree(h->pin); }
    h->pin = nullptr;
    h->pin_cap = 0;
    const size_t cap = std::max<size_t>(8 * size_t(n) + 8, 8192) * 3 / 2;
    if (hipHostMalloc(reinterpret_cast<void**>(&h->pin), sizeof(int32_t) * cap) != hipSuccess)
      return mapfail(SFM_ENOMEM, "hipHostMalloc failed");
    h->pin_cap = cap;
  }
  (void)hipStreamSynchronize(h->s);  // (the pinned block may feed an earlier copy)
  std::memcpy(h->pin, pts3d_idx, sizeof(int32_t) * size_t(n));
  double* pv = reinterpret_cast<double*>(h->pin + ((size_t(n) + 1) & ~size_t(1)));
  (void)hipMemcpyAsync(di, h->pin, sizeof(int32_t) * size_t(n), hipMemcpyHostToDevice, h->s);
  k_gather_points<<<grid(n), 256, 0, h->s>>>(n, di, h->X.p, dv);
  if (hipMemcpyAsync(pv, dv, sizeof(double) * 3 * size_t(n), hipMemcpyDeviceToHost, h->s) != hipSuccess)
    return mapfail(SFM_EIO, "download failed");
  if (int r = sync(h)) return r;
  std::memcpy(pts3d, pv, sizeof(double) * 3 * size_t(n));
  return 0;
}

int sfm_map_set_points(sfm_map* h, int32_t n, const int32_t* pts3d_idx, const double* pts3d) {
  if (!h) return mapfail(SFM_EINVAL, "NULL handle");
  if (n <= 0) return n < 0 ? mapfail(SFM_EINVAL, "negative size") : 0;
  if (!pts3d_idx || !pts3d) return mapfail(SFM_EINVAL, "NULL argument");
  if (int rc = check_pts(h, n, pts3d_idx)) return rc;
  if (hipSetDevice(h->device) != hipSuccess) return mapfail(SFM_ENODEV, "hipSetDevice failed");
  int rc = 0;
  auto* di = static_cast<int32_t*>(scratch(h, "si", sizeof(int32_t) * size_t(n), &rc));
  auto* dv = static_cast<double*>(scratch(h, "sv", sizeof(double) * 3 * size_t(n), &rc));
  if (rc) return rc;
  if (hipMemcpyAsync(di, pts3d_idx, sizeof(int32_t) * size_t(n), hipMemcpyHostToDevice, h->s) != hipSuccess ||
      hipMemcpyAsync(dv, pts3d, sizeof(double) * 3 * size_t(n), hipMemcpyHostToDevice, h->s) != hipSuccess)
    return mapfail(SFM_EIO, "upload failed");
  k_scatter_points<<<grid(n), 256, 0, h->s>>>(n, di, dv, h->X.p);  // (indices expected unique)
  return sync(h);
}

int sfm_map_points_in_frames(sfm_map* h, int32_t n_frames, const int32_t* frame_no, int32_t capacity,
                             int32_t* pts3d_idx, int32_t* n_out) {
  if (!h || !n_out) return mapfail(SFM_EINVAL, "NULL argument");
  *n_out = 0;
  if (n_frames < 0) return mapfail(SFM_EINVAL, "negative size");
  if (n_frames == 0 || h->n_pts == 0 || h->ob_pt.n == 0) return 0;
  if (!frame_no) return mapfail(SFM_EINVAL, "NULL frame list");
  if (hipSetDevice(h->device) != hipSuccess) return mapfail(SFM_ENODEV, "hipSetDevice failed");
  int rc = 0;
  const int P = h->n_pts;
  std::vector<int32_t> fs(frame_no, frame_no + n_frames);
  std::sort(fs.begin(), fs.end());
  fs.erase(std::unique(fs.begin(), fs.end()), fs.end());
  auto* fset = static_cast<int32_t*>(scratch(h, "fset", sizeof(int32_t) * fs.size(), &rc));
  auto* mark = static_cast<uint8_t*>(scratch(h, "mark", size_t(P), &rc));
  auto* out = static_cast<int32_t*>(scratch(h, "pout", sizeof(int32_t) * size_t(P), &rc));
  auto* dn = static_cast<int32_t*>(scratch(h, "pn", sizeof(int32_t), &rc));
  if (rc) return rc;
  (void)hipMemcpyAsync(fset, fs.data(), sizeof(int32_t) * fs.size(), hipMemcpyHostToDevice, h->s);
  (void)hipMemsetAsync(mark, 0, size_t(P), h->s);
  k_mark_frames<<<grid(h->ob_pt.n), 256, 0, h->s>>>(h->ob_pt.n, h->ob_pt.p, h->ob_frame.p, fset, int(fs.size()),
                                                    mark);
  hipcub::CountingInputIterator<int32_t> it(0);
  size_t bytes = 0;
  (void)hipcub::DeviceSelect::Flagged(nullptr, bytes, it, mark, out, dn, P, h->s);
  void* tmp = scratch(h, "psel", bytes, &rc);
  if (rc) return rc;
  if (hipcub::DeviceSelect::Flagged(tmp, bytes, it, mark, out, dn, P, h->s) != hipSuccess)
    return mapfail(SFM_EIO, "select failed");
  int32_t n = 0;
  (void)hipMemcpyAsync(&n, dn, sizeof(int32_t), hipMemcpyDeviceToHost, h->s);
  if (int r = sync(h)) return r;
  *n_out = n;
  if (n > capacity) return mapfail(SFM_EINVAL, "capacity " + std::to_string(capacity) + " < " + std::to_string(n));
  if (n && (!pts3d_idx || hipMemcpy(pts3d_idx, out, sizeof(int32_t) * size_t(n), hipMemcpyDeviceToHost) != hipSuccess))
    return mapfail(SFM_EIO, "download failed");
  return 0;
}

int sfm_map_points_in_frame(sfm_map* h, int32_t frame_no, int32_t capacity, int32_t* pts3d_idx, int32_t* n3_out,
                            int32_t* pts2d_idx, int32_t* n2_out) {
  if (!h || !n3_out || !n2_out) return mapfail(SFM_EINVAL, "NULL argument");
  *n3_out = *n2_out = 0;
  const int64_t N = h->ob_pt.n;
  if (N == 0) return 0;
  if (hipSetDevice(h->device) != hipSuccess) return mapfail(SFM_ENODEV, "hipSetDevice failed");
  int rc = 0;
  if (!h->ocsr) {
    if (int r = build_csr(h, "ob", h->ob_pt.p, N, &h->orow, &h->ooff)) return r;
    h->ocsr = true;
  }
  const int32_t *orow = h->orow, *ooff = h->ooff;
  auto* flag = static_cast<uint8_t*>(scratch(h, "fflag", size_t(N), &rc));
  auto* sel = static_cast<int32_t*>(scratch(h, "fsel", sizeof(int32_t) * size_t(N), &rc));
  auto* dn = static_cast<int32_t*>(scratch(h, "fn", sizeof(int32_t), &rc));
  if (rc) return rc;
  k_flag_frame<<<grid(N), 256, 0, h->s>>>(N, h->ob_frame.p, frame_no, flag);
  hipcub::CountingInputIterator<int32_t> it(0);
  size_t bytes = 0;
  (void)hipcub::DeviceSelect::Flagged(nullptr, bytes, it, flag, sel, dn, int(N), h->s);
  void* tmp = scratch(h, "fselt", bytes, &rc);
  if (rc) return rc;
  if (hipcub::DeviceSelect::Flagged(tmp, bytes, it, flag, sel, dn, int(N), h->s) != hipSuccess)
    return mapfail(SFM_EIO, "select failed");
  int32_t n = 0;
  (void)hipMemcpyAsync(&n, dn, sizeof(int32_t), hipMemcpyDeviceToHost, h->s);
  if (int r = sync(h)) return r;
  if (n == 0) return 0;
  auto* cnt = static_cast<int32_t*>(scratch(h, "fcnt", sizeof(int32_t) * size_t(n), &rc));
  auto* off2 = static_cast<int32_t*>(scratch(h, "foff", sizeof(int32_t) * size_t(n), &rc));
  auto* out3 = static_cast<int32_t*>(scratch(h, "fo3", sizeof(int32_t) * size_t(n), &rc));
  if (rc) return rc;
  k_dup_count<<<grid(n), 256, 0, h->s>>>(n, sel, h->ob_pt.p, h->ob_frame.p, orow, ooff, frame_no, cnt);
  bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, cnt, off2, n, h->s);
  tmp = scratch(h, "fscan", bytes, &rc);
  if (rc) return rc;
  if (hipcub::DeviceScan::ExclusiveSum(tmp, bytes, cnt, off2, n, h->s) != hipSuccess)
    return mapfail(SFM_EIO, "scan failed");
  int32_t last[2] = {0, 0};
  (void)hipMemcpyAsync(last, off2 + n - 1, sizeof(int32_t), hipMemcpyDeviceToHost, h->s);
  (void)hipMemcpyAsync(last + 1, cnt + n - 1, sizeof(int32_t), hipMemcpyDeviceToHost, h->s);
  if (int r = sync(h)) return r;
  const int32_t n2 = last[0] + last[1];
  auto* out2 = static_cast<int32_t*>(scratch(h, "fo2", sizeof(int32_t) * size_t(std::max(n2, 1)), &rc));
  if (rc) return rc;
  k_dup_fill<<<grid(n), 256, 0, h->s>>>(n, sel, h->ob_pt.p, h->ob_frame.p, h->ob_idx.p, orow, ooff, frame_no, off2,
                                        out3, out2);
  if (int r = sync(h)) return r;
  *n3_out = n;
  *n2_out = n2;
  if (n > capacity || n2 > capacity)
    return mapfail(SFM_EINVAL, "capacity " + std::to_string(capacity) + " < " + std::to_string(std::max(n, n2)));
  if (!pts3d_idx || !pts2d_idx) return mapfail(SFM_EINVAL, "NULL output");
  if (hipMemcpy(pts3d_idx, out3, sizeof(int32_t) * size_t(n), hipMemcpyDeviceToHost) != hipSuccess ||
      (n2 && hipMemcpy(pts2d_idx, out2, sizeof(int32_t) * size_t(n2), hipMemcpyDeviceToHost) != hipSuccess))
    return mapfail(SFM_EIO, "download failed");
  return 0;
}

int sfm_map_points_in_frame_multi(sfm_map* h, int32_t n_frames, const int32_t* frame_no, int64_t capacity,
                                  int32_t* pts3d_idx, int32_t* off3, int32_t* pts2d_idx, int32_t* off2) {
  SFM_TRACE("sfm_map_points_in_frame_multi");
  if (!h || !off3 || !off2 || (n_frames > 0 && !frame_no)) return mapfail(SFM_EINVAL, "NULL argument");
  if (n_frames < 0) return mapfail(SFM_EINVAL, "negative size");
  for (int i = 0; i <= n_frames; ++i) off3[i] = off2[i] = 0;
  const int64_t N = h->ob_pt.n;
  if (N == 0 || n_frames == 0) return 0;
  std::vector<int2> fr(static_cast<size_t>(n_frames));
  for (int i = 0; i < n_frames; ++i) fr[i] = make_int2(frame_no[i], i);
  std::sort(fr.begin(), fr.end(), [](int2 a, int2 b) { return a.x < b.x || (a.x == b.x && a.y < b.y); });
  for (int i = 1; i < n_frames; ++i)
    if (fr[i].x == fr[i - 1].x) return mapfail(SFM_EINVAL, "frame " + std::to_string(fr[i].x) + " queried twice");
  if (hipSetDevice(h->device) != hipSuccess) return mapfail(SFM_ENODEV, "hipSetDevice failed");
  int rc = 0;
  if (!h->ocsr) {
    if (int r = build_csr(h, "ob", h->ob_pt.p, N, &h->orow, &h->ooff)) return r;
    h->ocsr = true;
  }
  // every observation keyed by its frame's position in the query list; a
  // stable sort groups them frame by frame, each frame's in emplace order
  // (its equal_range)
  auto* dfr = static_cast<int2*>(scratch(h, "mfr", sizeof(int2) * size_t(n_frames), &rc));
  auto* key = static_cast<uint32_t*>(scratch(h, "mk", sizeof(uint32_t) * size_t(N), &rc));
  auto* key2 = static_cast<uint32_t*>(scratch(h, "mk2", sizeof(uint32_t) * size_t(N), &rc));
  auto* iv = static_cast<int32_t*>(scratch(h, "mi", sizeof(int32_t) * size_t(N), &rc));
  auto* sel = static_cast<int32_t*>(scratch(h, "msel", sizeof(int32_t) * size_t(N), &rc));
  auto* fcnt = static_cast<int32_t*>(scratch(h, "mfc", sizeof(int32_t) * (size_t(n_frames) + 1), &rc));
  if (rc) return rc;
  (void)hipMemcpyAsync(dfr, fr.data(), sizeof(int2) * fr.size(), hipMemcpyHostToDevice, h->s);
  (void)hipMemsetAsync(fcnt, 0, sizeof(int32_t) * (size_t(n_frames) + 1), h->s);
  k_frame_rank<<<grid(N), 256, 0, h->s>>>(N, h->ob_frame.p, dfr, n_frames, key, iv);
  k_count_keys<<<grid(N), 256, 0, h->s>>>(N, reinterpret_cast<const int32_t*>(key), fcnt);
  int bits = 1;
  while ((1 << bits) <= n_frames) ++bits;
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, key, key2, iv, sel, int(N), 0, bits, h->s);
  void* tmp = scratch(h, "msort", bytes, &rc);
  if (rc) return rc;
  if (hipcub::DeviceRadixSort::SortPairs(tmp, bytes, key, key2, iv, sel, int(N), 0, bits, h->s) != hipSuccess)
    return mapfail(SFM_EIO, "sort failed");
  // per sorted entry: how many 2D indices its point has in the entry's frame
  // (0 past the queried frames), their exclusive scan, then the frames'
  // offsets on the device: one readback of 2 (nf + 1) ints
  auto* cnt = static_cast<int32_t*>(scratch(h, "mcnt", sizeof(int32_t) * size_t(N), &rc));
  auto* eoff = static_cast<int32_t*>(scratch(h, "moff", sizeof(int32_t) * size_t(N), &rc));
  auto* offs = static_cast<int32_t*>(scratch(h, "moffs", sizeof(int32_t) * 2 * (size_t(n_frames) + 1), &rc));
  if (rc) return rc;
  k_dup_count_ranked<<<grid(N), 256, 0, h->s>>>(N, sel, key2, n_frames, h->ob_pt.p, h->ob_frame.p, h->orow, h->ooff,
                                                 cnt);
  bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, cnt, eoff, int(N), h->s);
  tmp = scratch(h, "mscan", bytes, &rc);
  if (rc) return rc;
  if (hipcub::DeviceScan::ExclusiveSum(tmp, bytes, cnt, eoff, int(N), h->s) != hipSuccess)
    return mapfail(SFM_EIO, "scan failed");
  k_frame_offsets<<<1, 1, 0, h->s>>>(n_frames, fcnt, N, cnt, eoff, offs);
  // (readbacks through the pinned block: a pageable copy is staged by the
  // runtime, ~2x the time at these sizes)
  int32_t* offs_h = pin_reserve(h, 2 * (size_t(n_frames) + 1), &rc);
  if (rc) return rc;
  (void)hipMemcpyAsync(offs_h, offs, sizeof(int32_t) * 2 * (size_t(n_frames) + 1), hipMemcpyDeviceToHost, h->s);
  if (int r = sync(h)) return r;
  for (int i = 0; i <= n_frames; ++i) {
    off3[i] = offs_h[i];
    off2[i] = offs_h[n_frames + 1 + i];
  }
  const int32_t n = off3[n_frames], n2 = off2[n_frames];
  if (n == 0) return 0;
  if (int64_t(n) > capacity || int64_t(n2) > capacity)
    return mapfail(SFM_EINVAL, "capacity " + std::to_string(capacity) + " < " + std::to_string(std::max(n, n2)));
  if (!pts3d_idx || !pts2d_idx) return mapfail(SFM_EINVAL, "NULL output");
  auto* out3 = static_cast<int32_t*>(scratch(h, "mo3", sizeof(int32_t) * size_t(n), &rc));
  auto* out2 = static_cast<int32_t*>(scratch(h, "mo2", sizeof(int32_t) * size_t(std::max(n2, 1)), &rc));
  if (rc) return rc;
  k_dup_fill<<<grid(n), 256, 0, h->s>>>(n, sel, h->ob_pt.p, h->ob_frame.p, h->ob_idx.p, h->orow, h->ooff, INT32_MIN,
                                        eoff, out3, out2);
  int32_t* ph = pin_reserve(h, size_t(n) + size_t(n2), &rc);
  if (rc) return rc;
  (void)hipMemcpyAsync(ph, out3, sizeof(int32_t) * size_t(n), hipMemcpyDeviceToHost, h->s);
  if (n2) (void)hipMemcpyAsync(ph + n, out2, sizeof(int32_t) * size_t(n2), hipMemcpyDeviceToHost, h->s);
  if (int r = sync(h)) return r;
  std::memcpy(pts3d_idx, ph, sizeof(int32_t) * size_t(n));
  if (n2) std::memcpy(pts2d_idx, ph + n, sizeof(int32_t) * size_t(n2));
  return 0;
}

int sfm_map_representative_descriptors(sfm_map* h, int32_t n, const int32_t* pts3d_idx, uint8_t* desc_out,
                                       int32_t* best_row) {
  if (!h) return mapfail(SFM_EINVAL, "NULL handle");
  if (n <= 0) return n < 0 ? mapfail(SFM_EINVAL, "negative size") : 0;
  if (!pts3d_idx || !desc_out) return mapfail(SFM_EINVAL, "NULL argument");
  if (int rc = check_pts(h, n, pts3d_idx)) return rc;
  if (hipSetDevice(h->device) != hipSuccess) return mapfail(SFM_ENODEV, "hipSetDevice failed");
  int rc = 0;
  const int64_t rows = h->desc.n / h->W;
  if (!h->dcsr) {
    if (int r = build_csr(h, "de", h->desc_pt.p, rows, &h->drow, &h->doff)) return r;
    h->dcsr = true;
  }
  const int32_t *drow = h->drow, *doff = h->doff;
  // every queried point needs a row (the reference reads row -1 otherwise)
  std::vector<int32_t> off(size_t(h->n_pts) + 1);
  (void)hipMemcpyAsync(off.data(), doff, sizeof(int32_t) * off.size(), hipMemcpyDeviceToHost, h->s);
  if (int r = sync(h)) return r;
  for (int32_t i = 0; i < n; ++i)
    if (off[size_t(pts3d_idx[i]) + 1] == off[size_t(pts3d_idx[i])])
      return mapfail(SFM_EINVAL, "point " + std::to_string(pts3d_idx[i]) + " has no descriptor row");
  auto* q = static_cast<int32_t*>(scratch(h, "rq", sizeof(int32_t) * size_t(n), &rc));
  auto* best = static_cast<int32_t*>(scratch(h, "rb", sizeof(int32_t) * size_t(n), &rc));
  auto* out = static_cast<uint64_t*>(scratch(h, "ro", sizeof(uint64_t) * size_t(n) * h->W, &rc));
  if (rc) return rc;
  (void)hipMemcpyAsync(q, pts3d_idx, sizeof(int32_t) * size_t(n), hipMemcpyHostToDevice, h->s);
  switch (h->W) {
#define CASE(w) case w: k_map_repr<w><<<n, 64, 0, h->s>>>(h->desc.p, drow, doff, q, n, nullptr, best, out); break;
    CASE(1) CASE(2) CASE(4) CASE(8) CASE(16) CASE(32) CASE(64)
#undef CASE
    default: return mapfail(SFM_EINVAL, "descriptor width");  // excluded by sfm_map_create
  }
  (void)hipMemcpyAsync(desc_out, out, size_t(n) * h->desc_bytes, hipMemcpyDeviceToHost, h->s);
  std::vector<int32_t> b(static_cast<size_t>(n));
  (void)hipMemcpyAsync(b.data(), best, sizeof(int32_t) * size_t(n), hipMemcpyDeviceToHost, h->s);
  if (int r = sync(h)) return r;
  if (best_row) std::memcpy(best_row, b.data(), sizeof(int32_t) * size_t(n));
  return 0;
}

// CSfM::findMapPointsInCurrentFrame (CSfM.cpp:634-692) in one call: the
// points of the keyframes (getPointsInFrames), minus the frame's matched
// points, projected with the frame's pose, their representative descriptors,
// matched in the (min, max) window against the current frame's unmatched
// keypoints, which the matcher holds (sfm_matcher_push_frame).  Everything
// stays on the device: one readback of the query count, one of the results
// (the composed calls downloaded every map point and the descriptors, and
// uploaded them again for the match: ~10 synchronisations per frame).
int sfm_map_match_frame(sfm_map* h, sfm_matcher* mt, int32_t n_frames, const int32_t* frame_no, int32_t n_existing,
                        const int32_t* existing_pts, const double* R9, const double* t3, const double* K9,
                        int32_t n_train, const int32_t* train_idx, double ratio_test, double min_distance,
                        double max_distance, int32_t capacity, int32_t* pts3d_match, int32_t* train_match,
                        int32_t* n_matches) {
  SFM_TRACE("sfm_map_match_frame");
  if (!h || !mt || !n_matches) return mapfail(SFM_EINVAL, "NULL handle");
  *n_matches = 0;
  if (n_frames < 0 || n_existing < 0 || n_train < 0) return mapfail(SFM_EINVAL, "negative size");
  if ((n_frames && !frame_no) || (n_existing && !existing_pts) || (n_train && !train_idx) || !R9 || !t3 || !K9)
    return mapfail(SFM_EINVAL, "NULL argument");
  if (matcher_words(mt) != h->W || matcher_device(mt) != h->device)
    return mapfail(SFM_EINVAL, "the map and the matcher differ in descriptor width or device");
  if (int rc = check_pts(h, n_existing, existing_pts)) return rc;
  const int n_cur = matcher_current_n(mt);
  if (n_cur < 0) return mapfail(SFM_EINVAL, "push the current frame to the matcher first");
  for (int i = 0; i < n_train; ++i)
    if (train_idx[i] < 0 || train_idx[i] >= n_cur) return mapfail(SFM_EINVAL, "train index out of range");
  if (n_frames == 0 || h->n_pts == 0 || h->ob_pt.n == 0 || n_train < 2) return 0;
  if (hipSetDevice(h->device) != hipSuccess) return mapfail(SFM_ENODEV, "hipSetDevice failed");
  int rc = 0;
  const int P = h->n_pts;
  std::vector<int32_t> fs(frame_no, frame_no + n_frames);
  std::sort(fs.begin(), fs.end());
  fs.erase(std::unique(fs.begin(), fs.end()), fs.end());
  if (!h->dcsr) {
    if (int r = build_csr(h, "de", h->desc_pt.p, h->desc.n / h->W, &h->drow, &h->doff)) return r;
    h->dcsr = true;
  }
  const size_t n_up = fs.size() + size_t(n_existing) + size_t(n_train);
  auto* fset = static_cast<int32_t*>(scratch(h, "fset", sizeof(int32_t) * n_up, &rc));
  auto* mark = static_cast<uint8_t*>(scratch(h, "mark", size_t(P), &rc));
  // the selected points, then (after k_map_repr) their representative rows:
  // one download for both
  auto* out = static_cast<int32_t*>(scratch(h, "pout", sizeof(int32_t) * 2 * size_t(P), &rc));
  auto* dn = static_cast<int32_t*>(scratch(h, "pn", sizeof(int32_t), &rc));
  if (rc) return rc;
  if (h->pin_cap < std::max(2 * size_t(P) + 1, n_up)) {
    if (h->pin) { (void)hipStreamSynchronize(h->s); (void)hipHostFree(h->pin); }
    h->pin = nullptr;
    h->pin_cap = 0;
    const size_t cap = std::max<size_t>(std::max(2 * size_t(P) + 1, n_up), 8192) * 3 / 2;
    if (hipHostMalloc(reinterpret_cast<void**>(&h->pin), sizeof(int32_t) * cap) != hipSuccess)
      return mapfail(SFM_ENOMEM, "hipHostMalloc failed");
    h->pin_cap = cap;
  }
  if (!h->ev && hipEventCreateWithFlags(&h->ev, hipEventDisableTiming) != hipSuccess)
    return mapfail(SFM_EIO, "hipEventCreate failed");
  // frames, the frame's matched points and the train subset in one upload
  (void)hipStreamSynchronize(h->s);  // (the pinned block may feed an earlier copy)
  std::memcpy(h->pin, fs.data(), sizeof(int32_t) * fs.size());
  if (n_existing) std::memcpy(h->pin + fs.size(), existing_pts, sizeof(int32_t) * size_t(n_existing));
  std::memcpy(h->pin + fs.size() + n_existing, train_idx, sizeof(int32_t) * size_t(n_train));
  (void)hipMemcpyAsync(fset, h->pin, sizeof(int32_t) * n_up, hipMemcpyHostToDevice, h->s);
  (void)hipMemsetAsync(mark, 0, size_t(P), h->s);
  k_mark_frames<<<grid(h->ob_pt.n), 256, 0, h->s>>>(h->ob_pt.n, h->ob_pt.p, h->ob_frame.p, fset, int(fs.size()), mark);
  if (n_existing) k_unmark<<<grid(n_existing), 256, 0, h->s>>>(n_existing, fset + fs.size(), mark);
  hipcub::CountingInputIterator<int32_t> it(0);
  size_t bytes = 0;
  (void)hipcub::DeviceSelect::Flagged(nullptr, bytes, it, mark, out, dn, P, h->s);
  void* tmp = scratch(h, "psel", bytes, &rc);
  if (rc) return rc;
  if (hipcub::DeviceSelect::Flagged(tmp, bytes, it, mark, out, dn, P, h->s) != hipSuccess)
    return mapfail(SFM_EIO, "select failed");
  // no readback of the count here: the kernels below run on its bound P and
  // read the count itself (k_map_repr, k_project, the matcher's acceptance)
  int32_t* best = out + P;
  auto* qd = static_cast<uint64_t*>(scratch(h, "mq", sizeof(uint64_t) * size_t(P) * h->W, &rc));
  auto* uv = static_cast<double*>(scratch(h, "muv", sizeof(double) * 2 * size_t(P), &rc));
  if (rc) return rc;
  switch (h->W) {
#define CASE(w) case w: k_map_repr<w><<<P, 64, 0, h->s>>>(h->desc.p, h->drow, h->doff, out, P, dn, best, qd); break;
    CASE(1) CASE(2) CASE(4) CASE(8) CASE(16) CASE(32) CASE(64)
#undef CASE
    default: return mapfail(SFM_EINVAL, "descriptor width");
  }
  k_project<<<grid(P), 256, 0, h->s>>>(P, dn, out, h->X.p, R9[0], R9[1], R9[2], R9[3], R9[4], R9[5], R9[6], R9[7],
                                       R9[8], t3[0], t3[1], t3[2], K9[0], K9[4], K9[2], K9[5], uv);
  // points, representative rows and the count in one download
  (void)hipMemcpyAsync(h->pin, out, sizeof(int32_t) * 2 * size_t(P), hipMemcpyDeviceToHost, h->s);
  (void)hipMemcpyAsync(h->pin + 2 * size_t(P), dn, sizeof(int32_t), hipMemcpyDeviceToHost, h->s);
  if (hipEventRecord(h->ev, h->s) != hipSuccess) return mapfail(SFM_EIO, "hipEventRecord failed");
  int* res = nullptr;
  if ((rc = matcher_match_current_dev(mt, h->ev, qd, uv, P, dn, fset + fs.size() + n_existing, n_train, ratio_test,
                                      min_distance, max_distance, &res)))
    return rc;
  if (int r = sync(h)) return r;
  const int n_new = h->pin[2 * size_t(P)];
  for (int i = 0; i < n_new; ++i)
    if (h->pin[P + i] < 0)
      return mapfail(SFM_EINVAL, "point " + std::to_string(h->pin[i]) + " has no descriptor row");
  const int m = res[2 * P];
  if (m > capacity) return mapfail(SFM_EINVAL, "capacity " + std::to_string(capacity) + " < " + std::to_string(m));
  for (int k = 0; k < m; ++k) {
    pts3d_match[k] = h->pin[res[k]];
    train_match[k] = train_idx[res[P + k]];
  }
  *n_matches = m;
  return 0;
}

}  // extern "C"

namespace sfm {
// The device copy of the map's points for sfm_track_pnp, which reads it on
// the matcher's stream: the map stream is drained first (its calls already
// synchronise before returning; this keeps the rule local).
const double* map_points_dev(sfm_map* h, int32_t* n_pts, int* device) {
  (void)hipStreamSynchronize(h->s);
  *n_pts = h->n_pts;
  *device = h->device;
  return h->X.p;
}
}  // namespace sfm
