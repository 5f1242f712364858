// Per-frame descriptor matcher for gfx950: brute-force Hamming 2-NN
// (replaces the external brisk::BruteForceMatcher::knnMatch, k = 2, called
// at /root/reference/CTracker.cpp:117, 214, 381, 433) and a parallel
// restatement of the reference's sequential acceptance loop
// (CTracker.cpp:221-249, identical at :122-148, :390-416, :441-467):
//
//   for i in queries (in order):
//     accept if d^2 > min^2 && d^2 < max^2 && float(d0)/float(d1) < ratio
//            && (train j0 unmatched || d0 < bestDist[j0])
//     new j0 -> append (i, j0); better -> overwrite the query at j0's slot
//
// Equivalent order-free form (proved in DESIGN.md §5): for each train j the
// surviving query is the FIRST accepted query with the minimum distance, and
// the output slots are ordered by the first accepted query of each j.  Both
// are integer min-reductions (atomicMin on packed keys), so the result is
// bit-exact and independent of scheduling.  Ties inside the 2-NN search go
// to the lower train index (the oracle's restated knnMatch convention).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>
#include "../../include/sfm_amd.h"
#include "ordered_compact.h"

void sfm_internal_set_error(const std::string& msg);  // ba_solver.hip

namespace {

thread_local std::string g_merr;

constexpr int kQ = 64;        // queries per workgroup (one per lane)
constexpr int kTrainTile = 256;

// One lane per query; train descriptors streamed through LDS in tiles.
// Descriptors are handled as 64-bit words; desc_bytes must be a multiple of 8
// (BRISK: 64 bytes) — other widths are zero-padded on the host.
template <int W>
__global__ __launch_bounds__(kQ) void k_knn2(const uint64_t* __restrict__ d0, int n0, const uint64_t* __restrict__ d1,
                                             int n1, int* __restrict__ bi, int* __restrict__ bd,
                                             int* __restrict__ si, int* __restrict__ sd) {
  __shared__ uint64_t tile[kTrainTile * W];
  const int i = blockIdx.x * kQ + threadIdx.x;
  uint64_t q[W];
#pragma unroll
  for (int w = 0; w < W; ++w) q[w] = (i < n0) ? d0[size_t(i) * W + w] : 0ull;
  int b0 = 1 << 30, j0 = -1, b1 = 1 << 30, j1 = -1;
  for (int t0 = 0; t0 < n1; t0 += kTrainTile) {
    const int nt = min(kTrainTile, n1 - t0);
    __syncthreads();
    for (int e = threadIdx.x; e < nt * W; e += kQ) tile[e] = d1[size_t(t0) * W + e];
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
      int d = 0;
#pragma unroll
      for (int w = 0; w < W; ++w) d += __popcll(q[w] ^ tile[t * W + w]);
      const int j = t0 + t;
      if (d < b0) { b1 = b0; j1 = j0; b0 = d; j0 = j; }
      else if (d < b1) { b1 = d; j1 = j; }
    }
  }
  if (i < n0) { bi[i] = j0; bd[i] = b0; si[i] = j1; sd[i] = b1; }
}

// Acceptance test per query + per-train min-reductions:
//   key[j]   = min over accepted queries of (d0 << 32 | i)  -> surviving query
//   first[j] = min over accepted queries of i               -> slot order
__global__ void k_accept(const double* __restrict__ p0, const double* __restrict__ p1, int n0,
                         const int* __restrict__ bi, const int* __restrict__ bd, const int* __restrict__ sd,
                         double ratio_test, double minSq, double maxSq, unsigned long long* __restrict__ key,
                         int* __restrict__ first) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n0) return;
  const int j = bi[i];
  if (j < 0) return;
  const float f0 = float(bd[i]), f1 = float(sd[i]);
  const double ratio = double(f0 / f1);
  const double dx = p0[2 * i] - p1[2 * j], dy = p0[2 * i + 1] - p1[2 * j + 1];
  const double d = dx * dx + dy * dy;
  if (d > minSq && d < maxSq && ratio < ratio_test) {
    atomicMin(&key[j], (static_cast<unsigned long long>(unsigned(bd[i])) << 32) | unsigned(i));
    atomicMin(&first[j], i);
  }
}

struct DevBufs {
  std::vector<void*> ptrs;
  ~DevBufs() { for (void* p : ptrs) hipFree(p); }
  template <typename T>
  T* get(size_t n) {
    void* p = nullptr;
    if (hipMalloc(&p, (n ? n : 1) * sizeof(T)) != hipSuccess) return nullptr;
    ptrs.push_back(p);
    return static_cast<T*>(p);
  }
};

int mfail(int code, const std::string& m) {
  g_merr = m;
  sfm_internal_set_error(m);
  return code;
}

// Pads descriptors to whole 64-bit words.
std::vector<uint64_t> pack_words(const uint8_t* d, int n, int nbytes, int W) {
  std::vector<uint64_t> out(size_t(n) * W, 0ull);
  for (int i = 0; i < n; ++i) std::memcpy(&out[size_t(i) * W], d + size_t(i) * nbytes, nbytes);
  return out;
}

int run_knn(hipStream_t s, int W, const uint64_t* d0, int n0, const uint64_t* d1, int n1, int* bi, int* bd, int* si,
            int* sd) {
  const int grid = (n0 + kQ - 1) / kQ;
  if (grid == 0) return 0;
  switch (W) {
#define CASE(w) case w: k_knn2<w><<<grid, kQ, 0, s>>>(d0, n0, d1, n1, bi, bd, si, sd); break;
    CASE(1) CASE(2) CASE(4) CASE(8) CASE(16) CASE(32) CASE(64)
#undef CASE
    default: return mfail(SFM_EINVAL, "descriptor width must be <= 512 bytes");
  }
  return 0;
}

int words_for(int nbytes) {
  int W = (nbytes + 7) / 8;
  int p = 1;
  while (p < W) p <<= 1;
  return p;
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

extern "C" {

const char* sfm_match_last_error(void) { return g_merr.c_str(); }

int sfm_knn2_hamming(int32_t device, const uint8_t* desc0, int32_t n0, const uint8_t* desc1, int32_t n1,
                     int32_t desc_bytes, int32_t* best_idx, int32_t* best_dist, int32_t* second_idx,
                     int32_t* second_dist) {
  if (n0 < 0 || n1 < 0 || desc_bytes <= 0 || desc_bytes > 512) return mfail(SFM_EINVAL, "bad sizes");
  if (n0 == 0) return 0;
  if (hipSetDevice(device) != hipSuccess) return mfail(SFM_ENODEV, "hipSetDevice failed");
  const int W = words_for(desc_bytes);
  auto h0 = pack_words(desc0, n0, desc_bytes, W), h1 = pack_words(desc1, n1, desc_bytes, W);
  DevBufs b;
  auto* d0 = b.get<uint64_t>(h0.size());
  auto* d1 = b.get<uint64_t>(h1.size());
  int* r = b.get<int>(4 * size_t(n0));
  if (!d0 || !d1 || !r) return mfail(SFM_ENOMEM, "hipMalloc failed");
  hipMemcpy(d0, h0.data(), h0.size() * 8, hipMemcpyHostToDevice);
  if (n1) hipMemcpy(d1, h1.data(), h1.size() * 8, hipMemcpyHostToDevice);
  int rc = run_knn(0, W, d0, n0, d1, n1, r, r + n0, r + 2 * n0, r + 3 * n0);
  if (rc) return rc;
  std::vector<int> out(4 * size_t(n0));
  if (hipMemcpy(out.data(), r, out.size() * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
    return mfail(SFM_EIO, "kernel or copy failed");
  std::memcpy(best_idx, out.data(), n0 * sizeof(int));
  std::memcpy(best_dist, out.data() + n0, n0 * sizeof(int));
  std::memcpy(second_idx, out.data() + 2 * n0, n0 * sizeof(int));
  std::memcpy(second_dist, out.data() + 3 * n0, n0 * sizeof(int));
  return 0;
}

int sfm_match_features(int32_t device, const double* pts0, const uint8_t* desc0, int32_t n0, const double* pts1,
                       const uint8_t* desc1, int32_t n1, int32_t desc_bytes, double ratio_test, double min_distance,
                       double max_distance, int32_t* idx0, int32_t* idx1, int32_t* n_matches) {
  if (!n_matches) return mfail(SFM_EINVAL, "n_matches is NULL");
  *n_matches = 0;
  if (n0 < 0 || n1 < 0 || desc_bytes <= 0 || desc_bytes > 512) return mfail(SFM_EINVAL, "bad sizes");
  if (n0 == 0 || n1 < 2) return 0;  // reference UB with < 2 train rows: no matches
  if (hipSetDevice(device) != hipSuccess) return mfail(SFM_ENODEV, "hipSetDevice failed");
  const int W = words_for(desc_bytes);
  auto h0 = pack_words(desc0, n0, desc_bytes, W), h1 = pack_words(desc1, n1, desc_bytes, W);
  DevBufs b;
  auto* d0 = b.get<uint64_t>(h0.size());
  auto* d1 = b.get<uint64_t>(h1.size());
  auto* p0 = b.get<double>(2 * size_t(n0));
  auto* p1 = b.get<double>(2 * size_t(n1));
  int* r = b.get<int>(4 * size_t(n0));
  auto* key = b.get<unsigned long long>(n1);
  int* first = b.get<int>(n1);
  int* slot = b.get<int>(n0);
  int* out = b.get<int>(2 * size_t(n0) + 1);
  if (!d0 || !d1 || !p0 || !p1 || !r || !key || !first || !slot || !out) return mfail(SFM_ENOMEM, "hipMalloc failed");
  hipStream_t s = 0;
  hipMemcpyAsync(d0, h0.data(), h0.size() * 8, hipMemcpyHostToDevice, s);
  hipMemcpyAsync(d1, h1.data(), h1.size() * 8, hipMemcpyHostToDevice, s);
  hipMemcpyAsync(p0, pts0, 16 * size_t(n0), hipMemcpyHostToDevice, s);
  hipMemcpyAsync(p1, pts1, 16 * size_t(n1), hipMemcpyHostToDevice, s);
  hipMemsetAsync(key, 0xff, 8 * size_t(n1), s);
  hipMemsetAsync(first, 0x7f, 4 * size_t(n1), s);  // 0x7f7f7f7f: overwritten below
  hipMemsetAsync(slot, 0, 4 * size_t(n0), s);
  {
    // first[] must start at INT_MAX exactly
    std::vector<int> inf(n1, 0x7fffffff);
    hipMemcpyAsync(first, inf.data(), 4 * size_t(n1), hipMemcpyHostToDevice, s);
    int rc = run_knn(s, W, d0, n0, d1, n1, r, r + n0, r + 2 * n0, r + 3 * n0);
    if (rc) return rc;
    const double minSq = min_distance * min_distance, maxSq = max_distance * max_distance;
    k_accept<<<(n0 + 255) / 256, 256, 0, s>>>(p0, p1, n0, r, r + n0, r + 3 * n0, ratio_test, minSq, maxSq, key, first);
    sfm::k_mark_first<<<(n1 + 255) / 256, 256, 0, s>>>(n1, first, slot);
    sfm::k_compact_slots<false><<<1, 1024, 0, s>>>(n0, slot, key, out, out + n0, out + 2 * n0);
    std::vector<int> host(2 * size_t(n0) + 1);
    if (hipMemcpy(host.data(), out, host.size() * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
      return mfail(SFM_EIO, "kernel or copy failed");
    const int m = host[2 * n0];
    std::memcpy(idx0, host.data(), m * sizeof(int));
    std::memcpy(idx1, host.data() + n0, m * sizeof(int));
    *n_matches = m;
  }
  return 0;
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
  if (hipSetDevice(device) != hipSuccess) return mfail(SFM_ENODEV, "hipSetDevice failed");
  const int W = words_for(desc_bytes);
  const int rows = row_off[n_pts];
  auto h = pack_words(desc, rows, desc_bytes, W);
  DevBufs b;
  auto* d = b.get<uint64_t>(h.size());
  int* o = b.get<int>(size_t(n_pts) + 1);
  int* r = b.get<int>(size_t(n_pts));
  if (!d || !o || !r) return mfail(SFM_ENOMEM, "hipMalloc failed");
  hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(o, row_off, (size_t(n_pts) + 1) * sizeof(int), hipMemcpyHostToDevice);
  switch (W) {
#define CASE(w) case w: k_repr<w><<<n_pts, 64>>>(d, o, n_pts, r); break;
    CASE(1) CASE(2) CASE(4) CASE(8) CASE(16) CASE(32) CASE(64)
#undef CASE
    default: return mfail(SFM_EINVAL, "descriptor width must be <= 512 bytes");
  }
  if (hipMemcpy(best, r, size_t(n_pts) * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
    return mfail(SFM_EIO, "kernel or copy failed");
  if (out)
    for (int32_t i = 0; i < n_pts; ++i)
      std::memcpy(out + size_t(i) * desc_bytes, desc + (size_t(row_off[i]) + best[i]) * desc_bytes, desc_bytes);
  return 0;
}

}  // extern "C"
