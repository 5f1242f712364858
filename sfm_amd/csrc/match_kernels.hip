// Per-frame descriptor matcher for gfx950.
//
// Replaces brisk::BruteForceMatcher::knnMatch(k = 2) (called at
// /root/reference/CTracker.cpp:117, 214, 381, 433) and the reference's
// sequential acceptance loop, identical in all four matchFeatures overloads
// (CTracker.cpp:122-148, 221-249, 390-416, 441-467):
//
//   for i in queries (in order):
//     accept if d^2 > min^2 && d^2 < max^2 && float(d0)/float(d1) < ratio
//            && (train j0 unmatched || d0 < bestDist[j0])
//     new j0 -> append (i, j0); better -> overwrite the query at j0's slot
//
// Order-free form: for each train j the surviving query is the
// FIRST accepted query with the minimum distance, and the output slots are
// ordered by the first accepted query of each j -- integer min-reductions
// (atomicMin on packed keys), bit-exact and independent of scheduling.  2-NN
// ties go to the lower train index (the restated knnMatch convention): the
// search keeps the two smallest (distance << 32 | train) keys, so the scan
// order of the train rows does not matter and the rows can be split across
// workgroups and waves.
//
// Hot-path layout: an sfm_matcher handle keeps the last two frames'
// keypoints and descriptors resident in HBM (one upload per frame, the
// _prevFrame = _currFrame swap of CSfM.cpp:626-629), pools every device and
// pinned buffer (no allocation per call) and runs a call as one stream of
// launches with one host sync.  The 2-NN search is a 2-D grid (64 queries x
// a train slice per workgroup, four waves each scanning a quarter of the
// slice), so a 2k x 2k frame pair fills the chip; train rows are
// wave-uniform 64-B scalar loads, the query lives in VGPRs.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <cmath>
#include <map>
#include <string>
#include <vector>
#include "sfm_trace.h"
#include "../../include/sfm_amd.h"
#include "ordered_compact.h"

void sfm_internal_set_error(const std::string& msg);  // ba_solver.hip

namespace {

int mfail(int code, const std::string& m) {
  sfm_internal_set_error(m);
  return code;
}

constexpr int kQ = 64;       // queries per workgroup (one per lane)
constexpr int kWaves = 4;    // waves per workgroup, each a quarter of the train slice
constexpr unsigned long long kNoKey = ~0ull;

// branch-free: two compares and three selects per candidate
__device__ __forceinline__ void top2_insert(unsigned long long k, unsigned long long& k0, unsigned long long& k1) {
  const bool lt0 = k < k0, lt1 = k < k1;
  k1 = lt0 ? k0 : (lt1 ? k : k1);
  k0 = lt0 ? k : k0;
}

// Partial 2-NN of query block blockIdx.x against train slice blockIdx.y.
// Query i is row qidx[i] of q (qidx == nullptr: row i), train t is row
// tidx[t] of tr; part[(y * n0 + i) * 2 + {0,1}] = the two smallest keys.
template <int W, bool kIdx>
__global__ __launch_bounds__(kQ * kWaves) void k_knn2_part(const uint64_t* __restrict__ q, const int* __restrict__ qidx,
                                                           int n0, const uint64_t* __restrict__ tr,
                                                           const int* __restrict__ tidx, int n1, int slice,
                                                           unsigned long long* __restrict__ part) {
  __shared__ unsigned long long red[kWaves][kQ][2];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: the train loop is scalar
  const int i = blockIdx.x * kQ + lane;
  uint64_t x[W];
  if (i < n0) {
    const size_t row = qidx ? size_t(qidx[i]) : size_t(i);
#pragma unroll
    for (int k = 0; k < W; ++k) x[k] = q[row * W + k];
  } else {
#pragma unroll
    for (int k = 0; k < W; ++k) x[k] = 0ull;
  }
  unsigned long long k0 = kNoKey, k1 = kNoKey;
  const int t0 = blockIdx.y * slice, t1 = min(n1, t0 + slice);
  const int per = (t1 - t0 + kWaves - 1) / kWaves;
  const int a = t0 + w * per, b = min(t1, a + per);
  // four rows in flight per step (four 64-B scalar loads, then the
  // popcounts), then the remainder
  int t = a;
  for (; t + 4 <= b; t += 4) {
    const uint64_t* r[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) r[u] = tr + (kIdx ? size_t(tidx[t + u]) : size_t(t + u)) * W;
    uint64_t y[4][W];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < W; ++k) y[u][k] = r[u][k];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      unsigned d = 0;
#pragma unroll
      for (int k = 0; k < W; ++k) d += unsigned(__popcll(x[k] ^ y[u][k]));
      top2_insert((static_cast<unsigned long long>(d) << 32) | unsigned(t + u), k0, k1);
    }
  }
  for (; t < b; ++t) {
    const uint64_t* r = tr + (kIdx ? size_t(tidx[t]) : size_t(t)) * W;   // wave-uniform: scalar loads
    unsigned d = 0;
#pragma unroll
    for (int k = 0; k < W; ++k) d += unsigned(__popcll(x[k] ^ r[k]));
    top2_insert((static_cast<unsigned long long>(d) << 32) | unsigned(t), k0, k1);
  }
  red[w][lane][0] = k0;
  red[w][lane][1] = k1;
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int v = 1; v < kWaves; ++v) {
      top2_insert(red[v][lane][0], k0, k1);
      top2_insert(red[v][lane][1], k0, k1);
    }
    if (i < n0) {
      part[(size_t(blockIdx.y) * n0 + i) * 2] = k0;
      part[(size_t(blockIdx.y) * n0 + i) * 2 + 1] = k1;
    }
  }
}

__device__ __forceinline__ void merge_parts(const unsigned long long* __restrict__ part, int n0, int nslice, int i,
                                            unsigned long long& k0, unsigned long long& k1) {
  k0 = kNoKey;
  k1 = kNoKey;
  for (int s = 0; s < nslice; ++s) {
    top2_insert(part[(size_t(s) * n0 + i) * 2], k0, k1);
    top2_insert(part[(size_t(s) * n0 + i) * 2 + 1], k0, k1);
  }
}

// The 2-NN result alone (sfm_knn2_hamming): best / second train + distance.
__global__ void k_knn2_merge(const unsigned long long* __restrict__ part, int n0, int nslice, int* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n0) return;
  unsigned long long k0, k1;
  merge_parts(part, n0, nslice, i, k0, k1);
  out[i] = k0 == kNoKey ? -1 : int(k0 & 0xffffffffu);
  out[n0 + i] = k0 == kNoKey ? (1 << 30) : int(k0 >> 32);
  out[2 * n0 + i] = k1 == kNoKey ? -1 : int(k1 & 0xffffffffu);
  out[3 * n0 + i] = k1 == kNoKey ? (1 << 30) : int(k1 >> 32);
}

// Merge + the acceptance test of query i + the per-train min-reductions:
//   key[j]   = min over accepted queries of (d0 << 32 | i)  -> surviving query
//   first[j] = min over accepted queries of i               -> slot order
// Positions are those of rows qidx[i] / tidx[j] (nullptr: i / j).
// (n0_dev: the query count on the device, n0 its bound -- sfm_map_match_frame)
__global__ void k_accept(const unsigned long long* __restrict__ part, int n0, const int* __restrict__ n0_dev, int nslice,
                         const double* __restrict__ p0, const int* __restrict__ qidx, const double* __restrict__ p1,
                         const int* __restrict__ tidx, double ratio_test, double minSq, double maxSq,
                         unsigned long long* __restrict__ key, int* __restrict__ first) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (n0_dev ? *n0_dev : n0)) return;
  unsigned long long k0, k1;
  merge_parts(part, n0, nslice, i, k0, k1);
  if (k0 == kNoKey || k1 == kNoKey) return;  // < 2 train rows: the reference reads past matches[i] (UB)
  const int j = int(k0 & 0xffffffffu);
  const unsigned d0 = unsigned(k0 >> 32), d1 = unsigned(k1 >> 32);
  // DMatch::distance is a float; the ratio is a float division stored in a double
  const float f0 = float(d0), f1 = float(d1);
  const double ratio = double(f0 / f1);
  const size_t a = qidx ? size_t(qidx[i]) : size_t(i), b = tidx ? size_t(tidx[j]) : size_t(j);
  const double dx = p0[2 * a] - p1[2 * b], dy = p0[2 * a + 1] - p1[2 * b + 1];
  const double d = dx * dx + dy * dy;
  if (d > minSq && d < maxSq && ratio < ratio_test) {
    atomicMin(&key[j], (static_cast<unsigned long long>(d0) << 32) | unsigned(i));
    atomicMin(&first[j], i);
  }
}

__global__ void k_reset(int n1, unsigned long long* __restrict__ key, int* __restrict__ first, int n0,
                        int* __restrict__ slot) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n1) { key[t] = kNoKey; first[t] = 0x7fffffff; }
  if (t < n0) slot[t] = 0;
}

// Pads descriptors to whole 64-bit words (W a power of two).
int words_for(int nbytes) {
  int W = (nbytes + 7) / 8;
  int p = 1;
  while (p < W) p <<= 1;
  return p;
}

void pack_words(const uint8_t* d, int n, int nbytes, int W, uint64_t* out) {
  if (nbytes == 8 * W) {
    std::memcpy(out, d, size_t(n) * nbytes);
    return;
  }
  std::memset(out, 0, size_t(n) * W * 8);
  for (int i = 0; i < n; ++i) std::memcpy(out + size_t(i) * W, d + size_t(i) * nbytes, nbytes);
}

// CMap::getRepresentativeDescriptors (CMap.cpp:345-381): one wavefront per
// map point; lane r owns rows r, r+64, ... of the point's descriptor matrix
// and sums its Hamming distances to every row (the reference's column sums
// of the symmetric distance matrix: integers, exact in its float), then a
// wave argmin keeps the lowest row on ties (the reference's strict `<` scan).
// Row k's words are wave-uniform loads (one line per instruction).
template <int W>
__global__ __launch_bounds__(64) void k_repr(const uint64_t* __restrict__ d, const int* __restrict__ off, int n_pts,
                                             int* __restrict__ best) {
  const int p = blockIdx.x, l = threadIdx.x;
  if (p >= n_pts) return;
  const int r0 = off[p], k = off[p + 1] - r0;
  const uint64_t* dp = d + size_t(r0) * W;
  unsigned long long key = ~0ull;  // (sum << 32 | row): the min is the first minimal row
  for (int r = l; r - l < k; r += 64) {
    uint64_t x[W];
#pragma unroll
    for (int w = 0; w < W; ++w) x[w] = r < k ? dp[size_t(r) * W + w] : 0ull;
    unsigned int sum = 0;
    for (int q = 0; q < k; ++q) {
#pragma unroll
      for (int w = 0; w < W; ++w) sum += __popcll(x[w] ^ dp[size_t(q) * W + w]);
    }
    if (r < k) key = min(key, (static_cast<unsigned long long>(sum) << 32) | unsigned(r));
  }
  for (int o = 32; o >= 1; o >>= 1) key = min(key, static_cast<unsigned long long>(__shfl_xor(key, o)));
  if (l == 0) best[p] = int(key & 0xffffffffu);
}

}  // namespace

// ---------------------------------------------------------------------------
// the handle

struct MatchFrame {
  int n = 0;
  uint64_t* desc = nullptr;   // [n][W]; one allocation with the two below
  double* pts = nullptr;      // [n][2] undistorted (CFrame::getPointsAt), right after desc
  double* ptsd = nullptr;     // [n][2] distorted (CFrame::getPointsDistorted), right after pts
  size_t cap = 0;
};

struct sfm_matcher {
  std::vector<MatchFrame> kf;  // keyframe store (sfm_matcher_store_keyframe)
  int device = 0;
  int desc_bytes = 64, W = 8;
  int n_cu = 256;
  hipStream_t stream = nullptr;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  MatchFrame frame[2];        // [prev, curr] after the swap
  int cur = 1;                // index of the current frame in frame[]
  int frames_pushed = 0;
  // pooled scratch (grow-only)
  std::map<std::string, std::pair<void*, size_t>> dev;
  std::map<std::string, std::pair<void*, size_t>> pin;
  float last_knn_ms = 0.f, last_total_ms = 0.f;
};

namespace {

template <typename T>
T* dbuf(sfm_matcher* h, const char* name, size_t count, int* rc) {
  auto& e = h->dev[name];
  const size_t bytes = std::max<size_t>(1, count) * sizeof(T);
  if (e.second < bytes) {
    if (e.first) hipFree(e.first);
    e.first = nullptr;
    e.second = 0;
    const size_t cap = std::max(bytes, size_t(4096)) * 3 / 2;
    if (hipMalloc(&e.first, cap) != hipSuccess) {
      *rc = mfail(SFM_ENOMEM, "hipMalloc failed (matcher scratch)");
      return nullptr;
    }
    e.second = cap;
  }
  return static_cast<T*>(e.first);
}

template <typename T>
T* pbuf(sfm_matcher* h, const char* name, size_t count, int* rc) {
  auto& e = h->pin[name];
  const size_t bytes = std::max<size_t>(1, count) * sizeof(T);
  if (e.second < bytes) {
    if (e.first) hipHostFree(e.first);
    e.first = nullptr;
    e.second = 0;
    const size_t cap = std::max(bytes, size_t(4096)) * 3 / 2;
    if (hipHostMalloc(&e.first, cap) != hipSuccess) {
      *rc = mfail(SFM_ENOMEM, "hipHostMalloc failed (matcher staging)");
      return nullptr;
    }
    e.second = cap;
  }
  return static_cast<T*>(e.first);
}

// Train slices: enough workgroups to put ~8 waves on every CU, each slice
// at least 64 rows (one row per lane-step of every wave is not worth less).
int slices_for(const sfm_matcher* h, int n0, int n1) {
  const int qb = (n0 + kQ - 1) / kQ;
  const int want = std::max(1, (2 * h->n_cu + qb - 1) / qb);
  const int most = std::max(1, n1 / 64);
  return std::min(want, most);
}

int launch_knn(sfm_matcher* h, const uint64_t* q, const int* qidx, int n0, const uint64_t* tr, const int* tidx,
               int n1, unsigned long long* part, int nslice) {
  const int slice = (n1 + nslice - 1) / nslice;
  dim3 grid((n0 + kQ - 1) / kQ, nslice);
  switch (h->W) {
#define CASE(w)                                                                                       \
  case w:                                                                                             \
    if (tidx) k_knn2_part<w, true><<<grid, kQ * kWaves, 0, h->stream>>>(q, qidx, n0, tr, tidx, n1, slice, part); \
    else k_knn2_part<w, false><<<grid, kQ * kWaves, 0, h->stream>>>(q, qidx, n0, tr, tidx, n1, slice, part);     \
    break;
    CASE(1) CASE(2) CASE(4) CASE(8) CASE(16) CASE(32) CASE(64)
#undef CASE
    default: return mfail(SFM_EINVAL, "descriptor width must be <= 512 bytes");
  }
  return 0;
}

// One match: queries (q, qidx, p0) against trains (tr, tidx, p1) already on
// the device; results (query, train) in subset-local indices into the pinned
// buffer `res` ([2 * n0 + 1]: idx0 | idx1 | count) after the stream sync.
// The kernels alone (no download, no synchronisation): the (query, train)
// pairs and their count land in the device buffer *out_dev ([2 n0 + 1]).
int run_match_async(sfm_matcher* h, const uint64_t* q, const int* qidx, const double* p0, int n0, const uint64_t* tr,
                    const int* tidx, const double* p1, int n1, double ratio, double mn, double mx, int** out_dev,
                    const int* n0_dev = nullptr) {
  int rc = 0;
  const int nslice = slices_for(h, n0, n1);
  auto* part = dbuf<unsigned long long>(h, "part", 2 * size_t(n0) * nslice, &rc);
  auto* key = dbuf<unsigned long long>(h, "key", size_t(n1), &rc);
  int* first = dbuf<int>(h, "first", size_t(n1), &rc);
  int* slot = dbuf<int>(h, "slot", size_t(n0), &rc);
  int* out = dbuf<int>(h, "out", 2 * size_t(n0) + 1, &rc);
  if (rc) return rc;
  hipStream_t s = h->stream;
  hipEventRecord(h->ev[0], s);
  k_reset<<<(std::max(n0, n1) + 255) / 256, 256, 0, s>>>(n1, key, first, n0, slot);
  if ((rc = launch_knn(h, q, qidx, n0, tr, tidx, n1, part, nslice))) return rc;
  hipEventRecord(h->ev[1], s);
  k_accept<<<(n0 + 255) / 256, 256, 0, s>>>(part, n0, n0_dev, nslice, p0, qidx, p1, tidx, ratio, mn * mn, mx * mx, key,
                                             first);
  sfm::k_mark_first<<<(n1 + 255) / 256, 256, 0, s>>>(n1, first, slot);
  sfm::k_compact_slots<false><<<1, 1024, 0, s>>>(n0, slot, key, out, out + n0, out + 2 * n0);
  hipEventRecord(h->ev[2], s);
  *out_dev = out;
  return 0;
}

int run_match(sfm_matcher* h, const uint64_t* q, const int* qidx, const double* p0, int n0, const uint64_t* tr,
              const int* tidx, const double* p1, int n1, double ratio, double mn, double mx, int** res_out,
              const int* n0_dev = nullptr) {
  int rc = 0;
  int* res = pbuf<int>(h, "res", 2 * size_t(n0) + 1, &rc);
  if (rc) return rc;
  int* out = nullptr;
  if ((rc = run_match_async(h, q, qidx, p0, n0, tr, tidx, p1, n1, ratio, mn, mx, &out, n0_dev))) return rc;
  hipStream_t s = h->stream;
  hipMemcpyAsync(res, out, (2 * size_t(n0) + 1) * sizeof(int), hipMemcpyDeviceToHost, s);
  if (hipStreamSynchronize(s) != hipSuccess) return mfail(SFM_EIO, "matcher kernels failed");
  hipEventElapsedTime(&h->last_knn_ms, h->ev[0], h->ev[1]);
  hipEventElapsedTime(&h->last_total_ms, h->ev[0], h->ev[2]);
  *res_out = res;
  return 0;
}

// sfm_track_pnp: the matches (query k -> prev keypoint pidx[out[k]], its map
// point pt3d[.]; train -> current keypoint out[n0 + k]) into PnP's object
// (the map point) and image (the current keypoint) arrays, with the match's
// map point and keypoint kept for the inlier lists; thread 0 copies the count
// into the result block's head.
__global__ void k_track_gather(const int* __restrict__ out, int n0, const int* __restrict__ pidx,
                               const int* __restrict__ pt3d, const double* __restrict__ X,
                               const double* __restrict__ pts, double* __restrict__ obj, double* __restrict__ img,
                               int* __restrict__ m3, int* __restrict__ kp, int* __restrict__ head) {
  const int m = out[2 * n0];
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k == 0) head[0] = m;
  if (k >= m) return;
  const int p = pt3d[pidx[out[k]]], c = out[n0 + k];
  obj[3 * k] = X[3 * size_t(p)];
  obj[3 * k + 1] = X[3 * size_t(p) + 1];
  obj[3 * k + 2] = X[3 * size_t(p) + 2];
  img[2 * k] = pts[2 * c];
  img[2 * k + 1] = pts[2 * c + 1];
  m3[k] = p;
  kp[k] = c;
}

bool ok_ratio_window(double ratio, double mn, double mx) {
  return std::isfinite(ratio) && std::isfinite(mn) && std::isfinite(mx);
}

}  // namespace

extern "C" {

}  // extern "C"

namespace sfm {
// pnp_kernels.hip / map_store.hip (sfm_track_pnp)
int pnp_ransac_dev(hipStream_t s, const int* d_n, int gate, const double* d_obj, const double* d_img, const double* K9,
                   int iterations, double reproj_err, double confidence, int* d_sub, double* d_model, int* d_cnt,
                   int* d_res, int* d_inl);
int pnp_max_iters();
int pnp_model_size();
const double* map_points_dev(sfm_map* h, int32_t* n_pts, int* device);
// For sfm_map_match_frame (map_store.hip): queries already on the device
// (descriptor words q, positions p0; produced on another stream, ordered
// after the event `after`) against a subset of the CURRENT frame's keypoints
// (d_train_idx, frame-local, on the device, checked by the caller against
// matcher_current_n); the (query, train) pairs in subset-local indices, as
// sfm_matcher_match returns them, in *res (pinned, valid after this call).
// No upload and no synchronisation before the kernels.
int matcher_match_current_dev(sfm_matcher* h, hipEvent_t after, const uint64_t* q, const double* p0, int n0,
                              const int32_t* d_n0, const int32_t* d_train_idx, int n1, double ratio, double mn,
                              double mx, int** res) {
  if (h->frames_pushed < 1) return mfail(SFM_EINVAL, "push the current frame first");
  if (!ok_ratio_window(ratio, mn, mx)) return mfail(SFM_EINVAL, "non-finite threshold");
  const MatchFrame& fc = h->frame[h->cur];
  if (after && hipStreamWaitEvent(h->stream, after, 0) != hipSuccess) return mfail(SFM_EIO, "stream wait failed");
  return run_match(h, q, nullptr, p0, n0, fc.desc, d_train_idx, fc.pts, n1, ratio, mn, mx, res, d_n0);
}
int matcher_current_n(const sfm_matcher* h) { return h->frames_pushed < 1 ? -1 : h->frame[h->cur].n; }
int matcher_words(const sfm_matcher* h) { return h->W; }
int matcher_device(const sfm_matcher* h) { return h->device; }
}  // namespace sfm

extern "C" {

int sfm_matcher_create(int32_t device, int32_t desc_bytes, sfm_matcher** out) {
  if (!out) return mfail(SFM_EINVAL, "out is NULL");
  *out = nullptr;
  if (desc_bytes <= 0 || desc_bytes > 512) return mfail(SFM_EINVAL, "desc_bytes must be in 1..512");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return mfail(SFM_ENODEV, "no HIP device visible");
  if (device < 0 || device >= n) return mfail(SFM_EINVAL, "device ordinal out of range");
  if (hipSetDevice(device) != hipSuccess) return mfail(SFM_EIO, "hipSetDevice failed");
  auto* h = new sfm_matcher();
  h->device = device;
  h->desc_bytes = desc_bytes;
  h->W = words_for(desc_bytes);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    h->n_cu = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return mfail(SFM_EIO, "hipStreamCreate failed");
  }
  for (auto& e : h->ev) hipEventCreate(&e);
  *out = h;
  return 0;
}

int sfm_matcher_destroy(sfm_matcher* h) {
  if (!h) return 0;
  hipSetDevice(h->device);
  hipStreamSynchronize(h->stream);
  for (auto& f : h->kf) hipFree(f.desc);
  for (auto& f : h->frame) {
    hipFree(f.desc);
  }
  for (auto& kv : h->dev) hipFree(kv.second.first);
  for (auto& kv : h->pin) hipHostFree(kv.second.first);
  for (auto e : h->ev) hipEventDestroy(e);
  hipStreamDestroy(h->stream);
  delete h;
  return 0;
}

int sfm_matcher_push_frame(sfm_matcher* h, const double* pts, const double* pts_distorted, const uint8_t* desc,
                           int32_t n) {
  SFM_TRACE("sfm_matcher_push_frame");
  if (!h) return mfail(SFM_EINVAL, "handle is NULL");
  if (n < 0 || (n > 0 && (!pts || !desc))) return mfail(SFM_EINVAL, "bad frame arguments");
  if (hipSetDevice(h->device) != hipSuccess) return mfail(SFM_EIO, "hipSetDevice failed");
  // the current frame becomes the previous one (CSfM.cpp:626-629)
  h->cur ^= 1;
  MatchFrame& f = h->frame[h->cur];
  int rc = 0;
  if (f.cap < size_t(std::max(n, 1))) {
    hipStreamSynchronize(h->stream);
    hipFree(f.desc);
    f.desc = nullptr; f.pts = f.ptsd = nullptr;
    f.cap = size_t(std::max(n, 1024)) * 3 / 2;
    if (hipMalloc(&f.desc, f.cap * (h->W * 8 + 32)) != hipSuccess) {
      f.cap = 0;
      return mfail(SFM_ENOMEM, "hipMalloc failed (matcher frame)");
    }
  }
  f.n = n;
  // [desc n W | pts 2n | ptsd 2n] as laid out in the stage: one copy
  f.pts = reinterpret_cast<double*>(f.desc + size_t(n) * h->W);
  f.ptsd = f.pts + 2 * size_t(n);
  if (n) {
    // staging: one pinned block per frame slot (the previous upload from it
    // may still be in flight only for the other slot)
    const char* nm = h->cur ? "stage1" : "stage0";
    const size_t words = size_t(n) * h->W;
    auto* st = pbuf<uint64_t>(h, nm, words + 4 * size_t(n), &rc);
    if (rc) return rc;
    hipStreamSynchronize(h->stream);   // the stage may feed an earlier copy
    pack_words(desc, n, h->desc_bytes, h->W, st);
    double* sp = reinterpret_cast<double*>(st + words);
    std::memcpy(sp, pts, 16 * size_t(n));
    std::memcpy(sp + 2 * size_t(n), pts_distorted ? pts_distorted : pts, 16 * size_t(n));
    hipMemcpyAsync(f.desc, st, words * 8 + 32 * size_t(n), hipMemcpyHostToDevice, h->stream);
  }
  ++h->frames_pushed;
  return 0;
}

int sfm_matcher_match_subset(sfm_matcher* h, const int32_t* prev_idx, int32_t n_prev, const int32_t* curr_idx,
                             int32_t n_curr, double ratio_test, double min_distance, double max_distance,
                             int32_t* prev_match, int32_t* curr_match, int32_t* n_matches) {
  SFM_TRACE("sfm_matcher_match_subset");
  if (!h || !n_matches) return mfail(SFM_EINVAL, "NULL argument");
  *n_matches = 0;
  if (h->frames_pushed < 2) return mfail(SFM_EINVAL, "push the previous and the current frame first");
  if (n_prev < 0 || n_curr < 0 || (n_prev && !prev_idx) || (n_curr && !curr_idx))
    return mfail(SFM_EINVAL, "bad index lists");
  if (!ok_ratio_window(ratio_test, min_distance, max_distance)) return mfail(SFM_EINVAL, "non-finite threshold");
  const MatchFrame& fp = h->frame[h->cur ^ 1];
  const MatchFrame& fc = h->frame[h->cur];
  for (int32_t i = 0; i < n_prev; ++i)
    if (prev_idx[i] < 0 || prev_idx[i] >= fp.n) return mfail(SFM_EINVAL, "prev index out of range");
  for (int32_t i = 0; i < n_curr; ++i)
    if (curr_idx[i] < 0 || curr_idx[i] >= fc.n) return mfail(SFM_EINVAL, "curr index out of range");
  if (n_prev == 0 || n_curr < 2) return 0;  // reference UB with < 2 train rows: no matches
  if (hipSetDevice(h->device) != hipSuccess) return mfail(SFM_EIO, "hipSetDevice failed");
  int rc = 0;
  int* ix = pbuf<int>(h, "idx", size_t(n_prev) + n_curr, &rc);
  int* dix = dbuf<int>(h, "didx", size_t(n_prev) + n_curr, &rc);
  if (rc) return rc;
  hipStreamSynchronize(h->stream);
  std::memcpy(ix, prev_idx, sizeof(int) * size_t(n_prev));
  std::memcpy(ix + n_prev, curr_idx, sizeof(int) * size_t(n_curr));
  hipMemcpyAsync(dix, ix, sizeof(int) * (size_t(n_prev) + n_curr), hipMemcpyHostToDevice, h->stream);
  int* res = nullptr;
  // undistorted positions (CFrame::getPointsAt, CTracker.cpp:375-376)
  if ((rc = run_match(h, fp.desc, dix, fp.pts, n_prev, fc.desc, dix + n_prev, fc.pts, n_curr, ratio_test,
                      min_distance, max_distance, &res)))
    return rc;
  const int m = res[2 * n_prev];
  // frame-global indices (CTracker.cpp:406-407, 412)
  for (int k = 0; k < m; ++k) {
    prev_match[k] = prev_idx[res[k]];
    curr_match[k] = curr_idx[res[n_prev + k]];
  }
  *n_matches = m;
  return 0;
}

int sfm_matcher_match_frames(sfm_matcher* h, int32_t distorted, double ratio_test, double min_distance,
                             double max_distance, int32_t* prev_idx, int32_t* curr_idx, int32_t* n_matches) {
  if (!h || !n_matches) return mfail(SFM_EINVAL, "NULL argument");
  *n_matches = 0;
  if (h->frames_pushed < 2) return mfail(SFM_EINVAL, "push the previous and the current frame first");
  if (!ok_ratio_window(ratio_test, min_distance, max_distance)) return mfail(SFM_EINVAL, "non-finite threshold");
  const MatchFrame& fp = h->frame[h->cur ^ 1];
  const MatchFrame& fc = h->frame[h->cur];
  if (fp.n == 0 || fc.n < 2) return 0;
  if (hipSetDevice(h->device) != hipSuccess) return mfail(SFM_EIO, "hipSetDevice failed");
  int* res = nullptr;
  int rc = run_match(h, fp.desc, nullptr, distorted ? fp.ptsd : fp.pts, fp.n, fc.desc, nullptr,
                     distorted ? fc.ptsd : fc.pts, fc.n, ratio_test, min_distance, max_distance, &res);
  if (rc) return rc;
  const int m = res[2 * fp.n];
  std::memcpy(prev_idx, res, sizeof(int) * size_t(m));
  std::memcpy(curr_idx, res + fp.n, sizeof(int) * size_t(m));
  *n_matches = m;
  return 0;
}

int sfm_matcher_match(sfm_matcher* h, const double* pts0, const uint8_t* desc0, int32_t n0, const double* pts1,
                      const uint8_t* desc1, int32_t n1, double ratio_test, double min_distance, double max_distance,
                      int32_t* idx0, int32_t* idx1, int32_t* n_matches) {
  SFM_TRACE("sfm_matcher_match");
  if (!h || !n_matches) return mfail(SFM_EINVAL, "NULL argument");
  *n_matches = 0;
  if (n0 < 0 || n1 < 0) return mfail(SFM_EINVAL, "negative size");
  if ((n0 && (!pts0 || !desc0)) || (n1 && (!pts1 || !desc1))) return mfail(SFM_EINVAL, "NULL array");
  if (!ok_ratio_window(ratio_test, min_distance, max_distance)) return mfail(SFM_EINVAL, "non-finite threshold");
  if (n0 == 0 || n1 < 2) return 0;  // reference UB with < 2 train rows: no matches
  if (hipSetDevice(h->device) != hipSuccess) return mfail(SFM_EIO, "hipSetDevice failed");
  int rc = 0;
  const size_t w0 = size_t(n0) * h->W, w1 = size_t(n1) * h->W;
  auto* st = pbuf<uint64_t>(h, "in", w0 + w1 + 2 * (size_t(n0) + n1), &rc);
  auto* d = dbuf<uint64_t>(h, "din", w0 + w1 + 2 * (size_t(n0) + n1), &rc);
  if (rc) return rc;
  hipStreamSynchronize(h->stream);
  pack_words(desc0, n0, h->desc_bytes, h->W, st);
  pack_words(desc1, n1, h->desc_bytes, h->W, st + w0);
  double* sp = reinterpret_cast<double*>(st + w0 + w1);
  std::memcpy(sp, pts0, 16 * size_t(n0));
  std::memcpy(sp + 2 * size_t(n0), pts1, 16 * size_t(n1));
  hipMemcpyAsync(d, st, (w0 + w1 + 2 * (size_t(n0) + n1)) * 8, hipMemcpyHostToDevice, h->stream);
  const double* dp = reinterpret_cast<const double*>(d + w0 + w1);
  int* res = nullptr;
  if ((rc = run_match(h, d, nullptr, dp, n0, d + w0, nullptr, dp + 2 * size_t(n0), n1, ratio_test, min_distance,
                      max_distance, &res)))
    return rc;
  const int m = res[2 * n0];
  std::memcpy(idx0, res, sizeof(int) * size_t(m));
  std::memcpy(idx1, res + n0, sizeof(int) * size_t(m));
  *n_matches = m;
  return 0;
}

// Keyframe store (CSfM::mapping's keyframe-pair matching, CSfM.cpp:141-221):
// slot `slot` takes pts [n][2] and desc [n][desc_bytes] once, resident.
int sfm_matcher_store_keyframe(sfm_matcher* h, int32_t slot, const double* pts, const uint8_t* desc, int32_t n) {
  SFM_TRACE("sfm_matcher_store_keyframe");
  if (!h) return mfail(SFM_EINVAL, "handle is NULL");
  if (slot < 0 || slot > (1 << 20) || n < 0 || (n > 0 && (!pts || !desc))) return mfail(SFM_EINVAL, "bad keyframe arguments");
  if (hipSetDevice(h->device) != hipSuccess) return mfail(SFM_EIO, "hipSetDevice failed");
  if (size_t(slot) >= h->kf.size()) h->kf.resize(size_t(slot) + 1);
  MatchFrame& f = h->kf[size_t(slot)];
  int rc = 0;
  if (f.cap < size_t(std::max(n, 1))) {
    hipStreamSynchronize(h->stream);
    hipFree(f.desc);
    f.desc = nullptr;
    f.cap = size_t(std::max(n, 1));
    if (hipMalloc(&f.desc, f.cap * (h->W * 8 + 16)) != hipSuccess) {
      f.cap = 0;
      return mfail(SFM_ENOMEM, "hipMalloc failed (matcher keyframe)");
    }
  }
  f.n = n;
  f.pts = reinterpret_cast<double*>(f.desc + size_t(n) * h->W);
  f.ptsd = f.pts;
  if (n) {
    const size_t words = size_t(n) * h->W;
    auto* st = pbuf<uint64_t>(h, "kfstage", words + 2 * size_t(n), &rc);
    if (rc) return rc;
    hipStreamSynchronize(h->stream);
    pack_words(desc, n, h->desc_bytes, h->W, st);
    std::memcpy(st + words, pts, 16 * size_t(n));
    hipMemcpyAsync(f.desc, st, words * 8 + 16 * size_t(n), hipMemcpyHostToDevice, h->stream);
  }
  return 0;
}

// sfm_matcher_match on keyframe rows: query rows q_idx of keyframe q_slot
// (positions q_pts [n_q][2] when given -- then q_idx must not repeat --,
// else the keyframe's own), train rows t_idx of keyframe t_slot; indices out
// are subset-local (into q_idx / t_idx), as sfm_matcher_match returns them.
int sfm_matcher_match_keyframes(sfm_matcher* h, int32_t q_slot, const int32_t* q_idx, int32_t n_q, const double* q_pts,
                                int32_t t_slot, const int32_t* t_idx, int32_t n_t, double ratio_test,
                                double min_distance, double max_distance, int32_t* idx0, int32_t* idx1,
                                int32_t* n_matches) {
  SFM_TRACE("sfm_matcher_match_keyframes");
  if (!h || !n_matches) return mfail(SFM_EINVAL, "NULL argument");
  *n_matches = 0;
  if (q_slot < 0 || t_slot < 0 || size_t(q_slot) >= h->kf.size() || size_t(t_slot) >= h->kf.size())
    return mfail(SFM_EINVAL, "keyframe slot not stored");
  if (n_q < 0 || n_t < 0 || (n_q && !q_idx) || (n_t && !t_idx)) return mfail(SFM_EINVAL, "bad index lists");
  if (!ok_ratio_window(ratio_test, min_distance, max_distance)) return mfail(SFM_EINVAL, "non-finite threshold");
  const MatchFrame& fq = h->kf[size_t(q_slot)];
  const MatchFrame& ft = h->kf[size_t(t_slot)];
  std::vector<char> seen(q_pts ? size_t(fq.n) : 0, 0);
  for (int32_t i = 0; i < n_q; ++i) {
    if (q_idx[i] < 0 || q_idx[i] >= fq.n) return mfail(SFM_EINVAL, "query index out of range");
    if (q_pts) {
      if (seen[size_t(q_idx[i])]) return mfail(SFM_EINVAL, "query index repeated with given positions");
      seen[size_t(q_idx[i])] = 1;
    }
  }
  for (int32_t i = 0; i < n_t; ++i)
    if (t_idx[i] < 0 || t_idx[i] >= ft.n) return mfail(SFM_EINVAL, "train index out of range");
  if (n_q == 0 || n_t < 2) return 0;  // reference UB with < 2 train rows: no matches
  if (hipSetDevice(h->device) != hipSuccess) return mfail(SFM_EIO, "hipSetDevice failed");
  int rc = 0;
  // stage: q_idx | t_idx | (8-B aligned) query positions at their rows
  const size_t ni = (size_t(n_q) + n_t + 1) & ~size_t(1);
  const size_t np = q_pts ? 2 * size_t(fq.n) : 0;
  auto* st = pbuf<int>(h, "kfidx", ni + 2 * np, &rc);
  auto* d = dbuf<int>(h, "dkfidx", ni + 2 * np, &rc);
  if (rc) return rc;
  hipStreamSynchronize(h->stream);
  std::memcpy(st, q_idx, sizeof(int) * size_t(n_q));
  std::memcpy(st + n_q, t_idx, sizeof(int) * size_t(n_t));
  double* sp = reinterpret_cast<double*>(st + ni);
  if (q_pts)
    for (int32_t i = 0; i < n_q; ++i) {
      sp[2 * size_t(q_idx[i])] = q_pts[2 * size_t(i)];
      sp[2 * size_t(q_idx[i]) + 1] = q_pts[2 * size_t(i) + 1];
    }
  hipMemcpyAsync(d, st, sizeof(int) * (ni + 2 * np), hipMemcpyHostToDevice, h->stream);
  const double* p0 = q_pts ? reinterpret_cast<const double*>(d + ni) : fq.pts;
  int* res = nullptr;
  if ((rc = run_match(h, fq.desc, d, p0, n_q, ft.desc, d + n_q, ft.pts, n_t, ratio_test, min_distance, max_distance,
                      &res)))
    return rc;
  const int m = res[2 * n_q];
  std::memcpy(idx0, res, sizeof(int) * size_t(m));
  std::memcpy(idx1, res + n_q, sizeof(int) * size_t(m));
  *n_matches = m;
  return 0;
}

int sfm_matcher_knn2(sfm_matcher* h, const uint8_t* desc0, int32_t n0, const uint8_t* desc1, int32_t n1,
                     int32_t* best_idx, int32_t* best_dist, int32_t* second_idx, int32_t* second_dist) {
  if (!h) return mfail(SFM_EINVAL, "handle is NULL");
  if (n0 < 0 || n1 < 0 || (n0 && !desc0) || (n1 && !desc1)) return mfail(SFM_EINVAL, "bad arguments");
  if (n0 == 0) return 0;
  if (hipSetDevice(h->device) != hipSuccess) return mfail(SFM_EIO, "hipSetDevice failed");
  int rc = 0;
  const size_t w0 = size_t(n0) * h->W, w1 = size_t(n1) * h->W;
  auto* st = pbuf<uint64_t>(h, "in", w0 + w1, &rc);
  auto* d = dbuf<uint64_t>(h, "din", w0 + w1, &rc);
  const int nslice = n1 > 0 ? slices_for(h, n0, n1) : 1;
  auto* part = dbuf<unsigned long long>(h, "part", 2 * size_t(n0) * nslice, &rc);
  int* out = dbuf<int>(h, "kout", 4 * size_t(n0), &rc);
  int* res = pbuf<int>(h, "kres", 4 * size_t(n0), &rc);
  if (rc) return rc;
  hipStreamSynchronize(h->stream);
  pack_words(desc0, n0, h->desc_bytes, h->W, st);
  if (n1) pack_words(desc1, n1, h->desc_bytes, h->W, st + w0);
  hipMemcpyAsync(d, st, (w0 + w1) * 8, hipMemcpyHostToDevice, h->stream);
  if ((rc = launch_knn(h, d, nullptr, n0, d + w0, nullptr, n1, part, nslice))) return rc;
  k_knn2_merge<<<(n0 + 255) / 256, 256, 0, h->stream>>>(part, n0, nslice, out);
  hipMemcpyAsync(res, out, 4 * size_t(n0) * sizeof(int), hipMemcpyDeviceToHost, h->stream);
  if (hipStreamSynchronize(h->stream) != hipSuccess) return mfail(SFM_EIO, "matcher kernels failed");
  std::memcpy(best_idx, res, n0 * sizeof(int));
  std::memcpy(best_dist, res + n0, n0 * sizeof(int));
  std::memcpy(second_idx, res + 2 * size_t(n0), n0 * sizeof(int));
  std::memcpy(second_dist, res + 3 * size_t(n0), n0 * sizeof(int));
  return 0;
}

int sfm_matcher_last_time(sfm_matcher* h, double* ms2) {
  if (!h || !ms2) return mfail(SFM_EINVAL, "NULL argument");
  ms2[0] = h->last_knn_ms;
  ms2[1] = h->last_total_ms;
  return 0;
}

// One-shot forms: a cached matcher per (device, calling thread), destroyed
// at thread exit, so repeated calls allocate nothing.
static sfm_matcher* cached_matcher(int32_t device, int32_t desc_bytes, int* rc) {
  struct Cache {
    std::map<std::pair<int, int>, sfm_matcher*> m;
    ~Cache() {
      for (auto& kv : m) sfm_matcher_destroy(kv.second);
    }
  };
  static thread_local Cache cache;
  sfm_matcher*& h = cache.m[{device, desc_bytes}];
  if (!h && (*rc = sfm_matcher_create(device, desc_bytes, &h))) h = nullptr;
  return h;
}

int sfm_knn2_hamming(int32_t device, const uint8_t* desc0, int32_t n0, const uint8_t* desc1, int32_t n1,
                     int32_t desc_bytes, int32_t* best_idx, int32_t* best_dist, int32_t* second_idx,
                     int32_t* second_dist) {
  if (n0 < 0 || n1 < 0 || desc_bytes <= 0 || desc_bytes > 512) return mfail(SFM_EINVAL, "bad sizes");
  if (n0 == 0) return 0;
  int rc = 0;
  sfm_matcher* h = cached_matcher(device, desc_bytes, &rc);
  if (!h) return rc;
  return sfm_matcher_knn2(h, desc0, n0, desc1, n1, best_idx, best_dist, second_idx, second_dist);
}

int sfm_match_features(int32_t device, const double* pts0, const uint8_t* desc0, int32_t n0, const double* pts1,
                       const uint8_t* desc1, int32_t n1, int32_t desc_bytes, double ratio_test, double min_distance,
                       double max_distance, int32_t* idx0, int32_t* idx1, int32_t* n_matches) {
  if (!n_matches) return mfail(SFM_EINVAL, "n_matches is NULL");
  *n_matches = 0;
  if (n0 < 0 || n1 < 0 || desc_bytes <= 0 || desc_bytes > 512) return mfail(SFM_EINVAL, "bad sizes");
  if (n0 == 0 || n1 < 2) return 0;  // reference UB with < 2 train rows: no matches
  int rc = 0;
  sfm_matcher* h = cached_matcher(device, desc_bytes, &rc);
  if (!h) return rc;
  return sfm_matcher_match(h, pts0, desc0, n0, pts1, desc1, n1, ratio_test, min_distance, max_distance, idx0, idx1,
                           n_matches);
}

int sfm_representative_descriptors(int32_t device, const uint8_t* desc, const int32_t* row_off, int32_t n_pts,
                                   int32_t desc_bytes, int32_t* best, uint8_t* out) {
  if (n_pts < 0 || desc_bytes <= 0 || desc_bytes > 512) return mfail(SFM_EINVAL, "bad sizes");
  if (n_pts == 0) return 0;
  if (!desc || !row_off || !best) return mfail(SFM_EINVAL, "NULL argument");
  if (row_off[0] != 0) return mfail(SFM_EINVAL, "row_off[0] must be 0");
  for (int32_t i = 0; i < n_pts; ++i)
    if (row_off[i + 1] <= row_off[i])
      return mfail(SFM_EINVAL, "every point needs at least one descriptor (the reference reads row -1 otherwise)");
  int rc = 0;
  sfm_matcher* h = cached_matcher(device, desc_bytes, &rc);
  if (!h) return rc;
  if (hipSetDevice(device) != hipSuccess) return mfail(SFM_ENODEV, "hipSetDevice failed");
  const int W = h->W;
  const int rows = row_off[n_pts];
  auto* st = pbuf<uint64_t>(h, "in", size_t(rows) * W + size_t(n_pts) + 1, &rc);
  auto* d = dbuf<uint64_t>(h, "din", size_t(rows) * W + size_t(n_pts) + 1, &rc);
  int* r = dbuf<int>(h, "rbest", size_t(n_pts), &rc);
  int* res = pbuf<int>(h, "rres", size_t(n_pts), &rc);
  if (rc) return rc;
  hipStreamSynchronize(h->stream);
  pack_words(desc, rows, desc_bytes, W, st);
  int* so = reinterpret_cast<int*>(st + size_t(rows) * W);
  std::memcpy(so, row_off, (size_t(n_pts) + 1) * sizeof(int));
  hipMemcpyAsync(d, st, (size_t(rows) * W + size_t(n_pts) + 1) * 8, hipMemcpyHostToDevice, h->stream);
  const int* o = reinterpret_cast<const int*>(d + size_t(rows) * W);
  switch (W) {
#define CASE(w) case w: k_repr<w><<<n_pts, 64, 0, h->stream>>>(d, o, n_pts, r); break;
    CASE(1) CASE(2) CASE(4) CASE(8) CASE(16) CASE(32) CASE(64)
#undef CASE
    default: return mfail(SFM_EINVAL, "descriptor width must be <= 512 bytes");
  }
  hipMemcpyAsync(res, r, size_t(n_pts) * sizeof(int), hipMemcpyDeviceToHost, h->stream);
  if (hipStreamSynchronize(h->stream) != hipSuccess) return mfail(SFM_EIO, "kernel or copy failed");
  std::memcpy(best, res, size_t(n_pts) * sizeof(int));
  if (out)
    for (int32_t i = 0; i < n_pts; ++i)
      std::memcpy(out + size_t(i) * desc_bytes, desc + (size_t(row_off[i]) + best[i]) * desc_bytes, desc_bytes);
  return 0;
}


// CSfM::tracking's pose step (CSfM.cpp:533-565) as one call: the previous
// frame's keypoints with a map point (prev_pt3d[i] >= 0) matched against the
// whole current frame (matchFeatures(prevIdx, currIdx), CTracker.cpp:368-417),
// their map points and keypoints gathered on the device, and
// cv::solvePnPRansac on them (sfm_pnp_ransac's kernels) -- one upload, one
// download, one synchronisation.  Fewer than min_matches matches: no PnP
// (*found = 0; the caller's lost-tracking branch, CSfM.cpp:545-551).  Outputs:
// *n_matches, the pose (rvec, tvec; zero when not found) and the inliers as
// (current keypoint, map point) pairs.
int sfm_track_pnp(sfm_matcher* h, sfm_map* map, int32_t n_prev, const int32_t* prev_pt3d, double ratio_test,
                  double min_distance, double max_distance, int32_t min_matches, const double* K9, int32_t iterations,
                  double reproj_err, double confidence, double* rvec, double* tvec, int32_t* found,
                  int32_t* n_matches, int32_t capacity, int32_t* inl_kp, int32_t* inl_pt3d, int32_t* n_inliers) {
  SFM_TRACE("sfm_track_pnp");
  if (!h || !map || !found || !n_matches || !n_inliers || !rvec || !tvec || !K9) return mfail(SFM_EINVAL, "NULL argument");
  *found = 0;
  *n_matches = 0;
  *n_inliers = 0;
  for (int i = 0; i < 3; ++i) rvec[i] = tvec[i] = 0.0;
  if (h->frames_pushed < 2) return mfail(SFM_EINVAL, "push the previous and the current frame first");
  if (!ok_ratio_window(ratio_test, min_distance, max_distance)) return mfail(SFM_EINVAL, "non-finite threshold");
  if (iterations < 0 || iterations > sfm::pnp_max_iters()) return mfail(SFM_EINVAL, "bad iterations");
  if (!(confidence > 0.0 && confidence < 1.0)) return mfail(SFM_EINVAL, "confidence must lie in (0, 1)");
  const MatchFrame& fp = h->frame[h->cur ^ 1];
  const MatchFrame& fc = h->frame[h->cur];
  if (n_prev != fp.n || (n_prev && !prev_pt3d)) return mfail(SFM_EINVAL, "prev_pt3d must hold one entry per previous keypoint");
  int32_t P = 0;
  int mdev = 0;
  const double* X = sfm::map_points_dev(map, &P, &mdev);
  if (mdev != h->device) return mfail(SFM_EINVAL, "the map and the matcher are on different devices");
  std::vector<int32_t> pidx;
  pidx.reserve(size_t(n_prev));
  for (int32_t i = 0; i < n_prev; ++i) {
    if (prev_pt3d[i] >= P) return mfail(SFM_EINVAL, "map point index out of range");
    if (prev_pt3d[i] >= 0) pidx.push_back(i);
  }
  const int n0 = int(pidx.size()), n1 = fc.n;
  if (n0 == 0 || n1 < 2) return 0;  // (as sfm_matcher_match_subset: no matches)
  if (capacity < n0) return mfail(SFM_EINVAL, "capacity below the previous frame's matched keypoints");
  if (hipSetDevice(h->device) != hipSuccess) return mfail(SFM_EIO, "hipSetDevice failed");
  int rc = 0;
  const int iters = iterations > 0 ? iterations : 1;
  const size_t n_up = size_t(n0) + size_t(n1) + size_t(n_prev);
  int* ix = pbuf<int>(h, "tidx", n_up, &rc);
  int* dix = dbuf<int>(h, "dtidx", n_up, &rc);
  // result block (ints): count, (pad x3) | found, best, inliers, pad | model
  // (6 doubles) | inliers [n0] | map points [n0] | keypoints [n0]
  const size_t blk = 8 + 12 + 3 * size_t(n0);
  int* dblk = dbuf<int>(h, "tblk", blk, &rc);
  int* hblk = pbuf<int>(h, "tblkh", blk, &rc);
  double* dobj = dbuf<double>(h, "tobj", 5 * size_t(n0), &rc);
  int* dsub = dbuf<int>(h, "tsub", size_t(sfm::pnp_model_size()) * iters, &rc);
  double* dmodel = dbuf<double>(h, "tmodel", 6 * size_t(iters), &rc);
  int* dcnt = dbuf<int>(h, "tcnt", size_t(iters), &rc);
  if (rc) return rc;
  hipStreamSynchronize(h->stream);  // (the pinned stage may feed an earlier copy)
  std::memcpy(ix, pidx.data(), sizeof(int) * size_t(n0));
  for (int i = 0; i < n1; ++i) ix[n0 + i] = i;  // the whole current frame (currIdx)
  if (n_prev) std::memcpy(ix + n0 + n1, prev_pt3d, sizeof(int) * size_t(n_prev));
  hipMemcpyAsync(dix, ix, sizeof(int) * n_up, hipMemcpyHostToDevice, h->stream);
  int* out = nullptr;
  // undistorted positions (CFrame::getPointsAt, CTracker.cpp:375-376)
  if ((rc = run_match_async(h, fp.desc, dix, fp.pts, n0, fc.desc, dix + n0, fc.pts, n1, ratio_test, min_distance,
                            max_distance, &out)))
    return rc;
  int* inl = dblk + 20;
  int* m3 = inl + n0;
  int* kp = m3 + n0;
  k_track_gather<<<(n0 + 255) / 256, 256, 0, h->stream>>>(out, n0, dix, dix + n0 + n1, X, fc.pts, dobj,
                                                          dobj + 3 * size_t(n0), m3, kp, dblk);
  if ((rc = sfm::pnp_ransac_dev(h->stream, dblk, min_matches, dobj, dobj + 3 * size_t(n0), K9, iterations, reproj_err,
                           confidence, dsub, dmodel, dcnt, dblk + 4, inl)))
    return rc;
  hipMemcpyAsync(hblk, dblk, sizeof(int) * blk, hipMemcpyDeviceToHost, h->stream);
  if (hipStreamSynchronize(h->stream) != hipSuccess) return mfail(SFM_EIO, "tracking kernels failed");
  const int m = hblk[0];
  *n_matches = m;
  if (m < min_matches || !hblk[4]) return 0;
  const double* mdl = reinterpret_cast<const double*>(hblk + 8);
  for (int i = 0; i < 3; ++i) { rvec[i] = mdl[i]; tvec[i] = mdl[3 + i]; }
  const int ni = hblk[6];
  const int* hin = hblk + 20;
  for (int i = 0; i < ni; ++i) {
    inl_kp[i] = hblk[20 + 2 * n0 + hin[i]];
    inl_pt3d[i] = hblk[20 + n0 + hin[i]];
  }
  *n_inliers = ni;
  *found = 1;
  return 0;
}
}  // extern "C"
