// Device-side problem setup for sfm_ba_set_problem (gfx950).
//
// The reference rebuilds its ceres::Problem on every call
// (/root/reference/CTracker.cpp:672-691: one residual block per observation,
// parameter blocks deduplicated by address), so the drop-in's per-call setup
// is on the critical path of every keyframe BA.  Everything O(N) here runs on
// the GPU from the caller's three observation arrays:
//   * validation (index ranges, finite uv) and the per-camera / per-point
//     observation counts;
//   * point-major order: a stable radix sort on (point, camera) -- ties keep
//     the caller's order, as the host definition did -- and the gathers of
//     uv / camera / point into it; pt_off by an exclusive scan;
//   * camera-major order: a stable radix sort of the point-major ids by
//     camera (points ascending within a camera), padded per camera to whole
//     64-wide wavefront chunks, with the chunk table grouped into 8 point
//     slices (one per XCD, k_jacobian);
//   * the Schur pair lists: for every observation o1 (camera-major), the
//     observations o2 of its point with camera >= c1, o2 != o1, emitted as
//     (block key, point) in (o1 camera-major, o2 ascending) order and stably
//     radix-sorted by block: each block's list is exactly the sequential
//     definition's; CSR offsets by binary search; the blocks by descending
//     pair count for k_schur_pts' wave balance (stable).
// Integer work only; every output is deterministic (no atomics decide an
// order: the counters are commutative integer adds).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <hipcub/hipcub.hpp>
#include <climits>
#include <cmath>
#include "ba_setup.h"

namespace sfm {
namespace {

constexpr int kT = 256;
inline int nblocks(int64_t n) { return int(std::max<int64_t>(1, (n + kT - 1) / kT)); }

// Camera counts go through a per-workgroup LDS histogram (a few hundred
// cameras: one global counter per camera would serialise ~N/C atomics on
// each); point counts are spread over P counters and go straight to memory.
constexpr int kLdsCams = 8192;
__global__ __launch_bounds__(kT) void k_validate(int64_t N, const double* __restrict__ uv,
                                                 const int32_t* __restrict__ cam, const int32_t* __restrict__ pt, int C,
                                                 int P, int32_t* __restrict__ err, int32_t* __restrict__ cam_cnt,
                                                 int32_t* __restrict__ pt_cnt) {
  __shared__ int32_t hist[kLdsCams];
  const bool lds = C <= kLdsCams;
  if (lds)
    for (int c = threadIdx.x; c < C; c += kT) hist[c] = 0;
  __syncthreads();
  for (int64_t i = int64_t(blockIdx.x) * kT + threadIdx.x; i < N; i += int64_t(gridDim.x) * kT) {
    const int c = cam[i], p = pt[i];
    const bool cok = c >= 0 && c < C, pok = p >= 0 && p < P;
    if (!cok) atomicMin(err + 0, int32_t(i));
    if (!pok) atomicMin(err + 1, int32_t(i));
    if (uv) {  // (nullptr: uv still in flight, checked by k_uv_layout)
      const double2 u = reinterpret_cast<const double2*>(uv)[i];
      if (!(isfinite(u.x) && isfinite(u.y))) atomicMin(err + 2, int32_t(i));
    }
    if (cok && pok) {
      if (lds) atomicAdd(hist + c, 1);
      else atomicAdd(cam_cnt + c, 1);
      if (pt_cnt) atomicAdd(pt_cnt + p, 1);  // (nullptr: pt_off from the sorted keys, k_pt_off)
    }
  }
  __syncthreads();
  if (lds)
    for (int c = threadIdx.x; c < C; c += kT)
      if (hist[c]) atomicAdd(cam_cnt + c, hist[c]);
}

__global__ __launch_bounds__(kT) void k_pm_keys(int64_t N, const int32_t* __restrict__ cam,
                                                const int32_t* __restrict__ pt, int C, uint64_t* __restrict__ keys,
                                                int32_t* __restrict__ iota) {
  const int64_t i = int64_t(blockIdx.x) * kT + threadIdx.x;
  if (i >= N) return;
  keys[i] = uint64_t(pt[i]) * uint64_t(C) + uint64_t(cam[i]);
  iota[i] = int32_t(i);
}

__global__ __launch_bounds__(kT) void k_gather_pm(int64_t N, const int32_t* __restrict__ order,
                                                  const double* __restrict__ uv, const int32_t* __restrict__ cam,
                                                  const int32_t* __restrict__ pt, double* __restrict__ uv_pm,
                                                  int32_t* __restrict__ cam_pm, int32_t* __restrict__ pt_s,
                                                  uint32_t* __restrict__ cam_key, int32_t* __restrict__ iota) {
  const int64_t q = int64_t(blockIdx.x) * kT + threadIdx.x;
  if (q >= N) return;
  const int64_t i = order[q];
  if (uv) reinterpret_cast<double2*>(uv_pm)[q] = reinterpret_cast<const double2*>(uv)[i];
  const int c = cam[i];
  cam_pm[q] = c;
  pt_s[q] = pt[i];
  cam_key[q] = uint32_t(c);
  iota[q] = int32_t(q);
}

// Camera-major slot i (runs padded to 64): its point-major observation, the
// point, uv, and the inverse map pos[q] = i.  Padding slots copy the
// camera's last observation (never read back; cam_obs = -1 marks them).
__global__ __launch_bounds__(kT) void k_fill_cm(int64_t N_pad, const int32_t* __restrict__ wcam,
                                                const int32_t* __restrict__ cam_rng,
                                                const int32_t* __restrict__ cam_off,
                                                const int32_t* __restrict__ cm_order,
                                                const int32_t* __restrict__ pt_s, const double* __restrict__ uv_pm,
                                                int32_t* __restrict__ cm_p, double* __restrict__ uv_cm,
                                                int32_t* __restrict__ cam_obs, int32_t* __restrict__ pos) {
  const int64_t i = int64_t(blockIdx.x) * kT + threadIdx.x;
  if (i >= N_pad) return;
  const int c = wcam[i >> 6];
  const int32_t j = int32_t(i - cam_rng[2 * c]);
  const int32_t n_c = cam_off[c + 1] - cam_off[c];
  const int32_t q = cm_order[cam_off[c] + min(j, n_c - 1)];
  cm_p[i] = pt_s[q];
  if (uv_pm) reinterpret_cast<double2*>(uv_cm)[i] = reinterpret_cast<const double2*>(uv_pm)[q];
  cam_obs[i] = j < n_c ? q : -1;
  if (j < n_c) pos[q] = int32_t(i);
}

// Large problems upload uv beside the index layouts (set_problem's deferred
// uv): k_gather_pm / k_fill_cm ran without it, and this pass makes the same
// two copies -- uv_pm[q] = uv[order[q]], camera-major slot i the uv of the
// point-major observation k_fill_cm took (padding: the camera's last one) --
// and k_validate's finite check (first bad caller index into err[2]).
__global__ __launch_bounds__(kT) void k_uv_layout(int64_t N, int64_t N_pad, const int32_t* __restrict__ order,
                                                  const int32_t* __restrict__ wcam,
                                                  const int32_t* __restrict__ cam_rng,
                                                  const int32_t* __restrict__ cam_off,
                                                  const int32_t* __restrict__ cm_order, const double* __restrict__ uv,
                                                  double* __restrict__ uv_pm, double* __restrict__ uv_cm,
                                                  int32_t* __restrict__ err) {
  const int64_t i = int64_t(blockIdx.x) * kT + threadIdx.x;
  if (i < N) {
    const int32_t o = order[i];
    const double2 u = reinterpret_cast<const double2*>(uv)[o];
    reinterpret_cast<double2*>(uv_pm)[i] = u;
    if (!(isfinite(u.x) && isfinite(u.y))) atomicMin(err + 2, o);
  }
  if (i < N_pad) {
    const int c = wcam[i >> 6];
    const int32_t j = int32_t(i - cam_rng[2 * c]);
    const int32_t n_c = cam_off[c + 1] - cam_off[c];
    const int32_t q = cm_order[cam_off[c] + min(j, n_c - 1)];
    reinterpret_cast<double2*>(uv_cm)[i] = reinterpret_cast<const double2*>(uv)[order[q]];
  }
}

// Chunk t of the (camera-major) chunk list: its XCD group is
// the point slice of its first observation (.w holds that observation's
// camera-major index until the gather clears it).
__global__ __launch_bounds__(kT) void k_chunk_keys(int n, const int4* __restrict__ ch,
                                                   const int32_t* __restrict__ cm_order,
                                                   const int32_t* __restrict__ pt_s, int P, uint32_t* __restrict__ key,
                                                   int32_t* __restrict__ iota) {
  const int t = blockIdx.x * kT + threadIdx.x;
  if (t >= n) return;
  const int p0 = pt_s[cm_order[ch[t].w]];
  key[t] = uint32_t(int64_t(p0) * 8 / max(1, P));
  iota[t] = t;
}

__global__ __launch_bounds__(kT) void k_chunk_gather(int n, const int32_t* __restrict__ perm,
                                                     const int4* __restrict__ ch, const uint32_t* __restrict__ key,
                                                     int4* __restrict__ out, int32_t* __restrict__ grp) {
  const int t = blockIdx.x * kT + threadIdx.x;
  if (t < n) {
    const int4 v = ch[perm[t]];
    out[t] = make_int4(v.x, v.y, v.z, 0);
  }
  if (t <= 8) {  // grp[g] = first chunk of group g (lower bound in the sorted keys)
    int lo = 0, hi = n;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (int(key[mid]) < t) lo = mid + 1; else hi = mid;
    }
    grp[t] = lo;
  }
}

// Pairs of observation o1 (entry i of the camera-major list, unpadded; or,
// cm_order == nullptr, point-major observation i): o2 in the point's segment
// with camera >= c1, o2 != o1.  The stable sort by block that follows keeps,
// within a block (c1, c2), the emission order of its o1 -- camera c1's
// observations, in point-major order either way (the camera-major list holds
// each camera's run in point-major order) -- so both emissions give the same
// lists.  Point-major emission reads each point's run from adjacent threads
// (one gather per run instead of one per observation).
__global__ __launch_bounds__(kT) void k_pair_count(int64_t N, const int32_t* __restrict__ cm_order,
                                                   const int32_t* __restrict__ cam_pm,
                                                   const int32_t* __restrict__ pt_s,
                                                   const int32_t* __restrict__ pt_off, int64_t* __restrict__ cnt) {
  const int64_t i = int64_t(blockIdx.x) * kT + threadIdx.x;
  if (i > N) return;
  if (i == N) { cnt[N] = 0; return; }
  const int32_t o1 = cm_order ? cm_order[i] : int32_t(i);
  const int c1 = cam_pm[o1], p = pt_s[o1];
  int64_t k = 0;
  for (int32_t o2 = pt_off[p]; o2 < pt_off[p + 1]; ++o2) k += (cam_pm[o2] >= c1 && o2 != o1) ? 1 : 0;
  cnt[i] = k;
}

__device__ __forceinline__ int64_t row_start(int c1, int C) { return int64_t(c1) * C - int64_t(c1) * (c1 - 1) / 2; }

__global__ __launch_bounds__(kT) void k_pair_fill(int64_t N, const int32_t* __restrict__ cm_order,
                                                  const int32_t* __restrict__ cam_pm, const int32_t* __restrict__ pt_s,
                                                  const int32_t* __restrict__ pt_off, const int64_t* __restrict__ off,
                                                  int C, uint32_t* __restrict__ key, int32_t* __restrict__ val) {
  const int64_t i = int64_t(blockIdx.x) * kT + threadIdx.x;
  if (i >= N) return;
  const int32_t o1 = cm_order ? cm_order[i] : int32_t(i);
  const int c1 = cam_pm[o1], p = pt_s[o1];
  const int64_t rs = row_start(c1, C) - c1;
  int64_t k = off[i];
  for (int32_t o2 = pt_off[p]; o2 < pt_off[p + 1]; ++o2) {
    const int c2 = cam_pm[o2];
    if (c2 >= c1 && o2 != o1) {
      key[k] = uint32_t(rs + c2);
      val[k] = p;
      ++k;
    }
  }
}

// pt_off[p] = first point-major observation of point p: the lower bound of
// p * C in the sorted (point, camera) keys -- the exclusive sum of the point
// counts, without k_validate's 2M scattered count atomics.
__global__ __launch_bounds__(kT) void k_pt_off(int P, const uint64_t* __restrict__ key, int64_t N, int C,
                                               int32_t* __restrict__ pt_off) {
  const int64_t p = int64_t(blockIdx.x) * kT + threadIdx.x;
  if (p > P) return;
  const uint64_t t = uint64_t(p) * uint64_t(C);
  int64_t lo = 0, hi = N;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (key[mid] < t) lo = mid + 1; else hi = mid;
  }
  pt_off[p] = int32_t(lo);
}

// seg[b] = first pair of block b (lower bound of b in the sorted keys).
__global__ __launch_bounds__(kT) void k_seg(int64_t n_blk, const uint32_t* __restrict__ key, int64_t n_pairs,
                                            int32_t* __restrict__ seg) {
  const int64_t b = int64_t(blockIdx.x) * kT + threadIdx.x;
  if (b > n_blk) return;
  int64_t lo = 0, hi = n_pairs;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (int64_t(key[mid]) < b) lo = mid + 1; else hi = mid;
  }
  seg[b] = int32_t(lo);
}

__global__ __launch_bounds__(kT) void k_blk(int C, int2* __restrict__ blk) {
  const int c1 = blockIdx.y;
  const int64_t rs = row_start(c1, C) - c1;
  for (int c2 = c1 + int(blockIdx.x) * kT + int(threadIdx.x); c2 < C; c2 += int(gridDim.x) * kT)
    blk[rs + c2] = make_int2(c1, c2);
}

// ---- k_schur_pts work order (set_problem step 5) ----
// One workgroup: rows' pair totals (block counts when there are no pairs)
// scanned kT rows at a time; row c1 goes to group x = the eighth of the total
// its middle falls in (monotone in c1, so a group is a contiguous block
// range).  grp[x] = the group's first block, grp[8 + x] = its block count.
__global__ __launch_bounds__(kT) void k_bperm_rows(int C, const int32_t* __restrict__ seg, int64_t n_pairs,
                                                   int64_t n_blk, int32_t* __restrict__ row_x,
                                                   int64_t* __restrict__ grp) {
  __shared__ int64_t sc[kT];
  __shared__ int64_t carry;
  __shared__ unsigned long long gfirst[8], gsize[8];
  const int t = threadIdx.x;
  if (t < 8) {
    gfirst[t] = ~0ull;
    gsize[t] = 0;
  }
  if (t == 0) carry = 0;
  __syncthreads();
  const int64_t total = n_pairs > 0 ? n_pairs : n_blk;
  for (int base = 0; base < C; base += kT) {
    const int c1 = base + t;
    int64_t first = 0, nb = 0, w = 0;
    if (c1 < C) {
      first = row_start(c1, C);
      nb = C - c1;
      w = n_pairs > 0 ? int64_t(seg[first + nb]) - seg[first] : nb;
    }
    sc[t] = w;
    __syncthreads();
    for (int o = 1; o < kT; o <<= 1) {
      const int64_t v = t >= o ? sc[t - o] : 0;
      __syncthreads();
      sc[t] += v;
      __syncthreads();
    }
    const int64_t before = carry + sc[t] - w;
    if (c1 < C) {
      const int x = int(min<int64_t>(7, (8 * (before + w / 2)) / max<int64_t>(1, total)));
      row_x[c1] = x;
      atomicMin(&gfirst[x], (unsigned long long)first);
      atomicAdd(&gsize[x], (unsigned long long)nb);
    }
    __syncthreads();
    if (t == kT - 1) carry += sc[kT - 1];
    __syncthreads();
  }
  if (t < 8) {
    grp[t] = gsize[t] ? int64_t(gfirst[t]) : 0;
    grp[8 + t] = int64_t(gsize[t]);
  }
}

// key = (row, descending pair count): a stable sort keeps every row's block
// range in place and orders its blocks longest list first
__global__ __launch_bounds__(kT) void k_bperm_keys(int64_t n_blk, const int2* __restrict__ blk,
                                                   const int32_t* __restrict__ seg, int cbits,
                                                   uint32_t* __restrict__ key, int32_t* __restrict__ iota) {
  const int64_t b = int64_t(blockIdx.x) * kT + threadIdx.x;
  if (b >= n_blk) return;
  const uint32_t cmax = (1u << cbits) - 1u;
  const uint32_t cnt = min(uint32_t(seg[b + 1] - seg[b]), cmax);
  key[b] = (uint32_t(blk[b].x) << cbits) | (cmax - cnt);
  iota[b] = int32_t(b);
}

// group x's i-th block goes to slot ((i / per) * 8 + x) * per + i % per:
// workgroups x, x + 8, x + 16, ... (one XCD under round-robin placement)
__global__ __launch_bounds__(kT) void k_bperm_fill(int64_t n_blk, const int32_t* __restrict__ sorted,
                                                   const int2* __restrict__ blk, const int32_t* __restrict__ row_x,
                                                   const int64_t* __restrict__ grp, int per,
                                                   int32_t* __restrict__ bperm) {
  const int64_t p = int64_t(blockIdx.x) * kT + threadIdx.x;
  if (p >= n_blk) return;
  const int32_t b = sorted[p];
  const int x = row_x[blk[b].x];
  const int64_t i = p - grp[x];
  bperm[((i / per) * 8 + x) * per + i % per] = b;
}

// Host (pinned, device-mapped) -> device copy by a kernel, 16 B per lane
// (bytes a multiple of 16): a small upload that must not queue behind a large
// DMA on the copy engine (set_problem's deferred uv)
__global__ __launch_bounds__(kT) void k_copy_from_host(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                       int64_t n16) {
  for (int64_t i = int64_t(blockIdx.x) * kT + threadIdx.x; i < n16; i += int64_t(gridDim.x) * kT) dst[i] = src[i];
}

__global__ __launch_bounds__(kT) void k_fill32(Fill32Set fs) {
  const Fill32Set::Job f = fs.job[blockIdx.y];
  // 16-B stores for the bulk (device allocations are 256-B aligned), then the tail
  const int64_t n4 = (reinterpret_cast<uintptr_t>(f.p) & 15) ? 0 : f.n / 4;
  const uint4 v4 = make_uint4(f.v, f.v, f.v, f.v);
  const int64_t t0 = int64_t(blockIdx.x) * kT + threadIdx.x, st = int64_t(gridDim.x) * kT;
  for (int64_t i = t0; i < n4; i += st) reinterpret_cast<uint4*>(f.p)[i] = v4;
  for (int64_t i = 4 * n4 + t0; i < f.n; i += st) f.p[i] = f.v;
}

// ---- keyframe-sized problems (set_problem's small path) ----
// The same layouts without radix sorts.  The host knows every count, so
// each order is a scatter into its known segments -- an integer atomic only
// picks a slot -- followed by ordering each segment on its own: the final
// order within a segment is the sorted one whatever slots the atomics gave,
// so every output is the sorted path's, bit for bit (tests/test_gpu_scale.py).

// Observation i into its point's segment (any slot).
__global__ __launch_bounds__(kT) void k_small_pm_scatter(int64_t N, const int32_t* __restrict__ pt,
                                                         const int32_t* __restrict__ pt_off,
                                                         int32_t* __restrict__ fill, int32_t* __restrict__ tmp) {
  const int64_t i = int64_t(blockIdx.x) * kT + threadIdx.x;
  if (i >= N) return;
  const int p = pt[i];
  tmp[pt_off[p] + atomicAdd(fill + p, 1)] = int32_t(i);
}
// Each observation's rank in its point's segment by (camera, caller index)
// -- the stable (point, camera) sort's order -- and the point-major gathers
// at that position (k_gather_pm's).  Segments are short (the host bounds
// them): every lane scans its own.
__global__ __launch_bounds__(kT) void k_small_pm_rank(int64_t N, const int32_t* __restrict__ pt_off,
                                                      const int32_t* __restrict__ tmp,
                                                      const int32_t* __restrict__ cam, const int32_t* __restrict__ pt,
                                                      const double* __restrict__ uv, int32_t* __restrict__ order,
                                                      double* __restrict__ uv_pm, int32_t* __restrict__ cam_pm,
                                                      int32_t* __restrict__ pt_s) {
  const int64_t s = int64_t(blockIdx.x) * kT + threadIdx.x;
  if (s >= N) return;
  const int32_t i = tmp[s];
  const int p = pt[i], c = cam[i];
  const int q0 = pt_off[p], q1 = pt_off[p + 1];
  int rank = 0;
  for (int q = q0; q < q1; ++q) {
    const int32_t j = tmp[q];
    const int cj = cam[j];
    rank += (cj < c || (cj == c && j < i)) ? 1 : 0;
  }
  const int dst = q0 + rank;
  order[dst] = i;
  reinterpret_cast<double2*>(uv_pm)[dst] = reinterpret_cast<const double2*>(uv)[i];
  cam_pm[dst] = c;
  pt_s[dst] = p;
}
// One workgroup per camera: its point-major ids ascending (the stable sort
// by camera of the point-major order) by a stable compaction -- 1024 ids
// at a time, each wave's matches ranked by ballot, the waves in order.
constexpr int kSmallCmMaxSteps = int(kSmallSetupMaxObs / 1024);
__global__ __launch_bounds__(1024) void k_small_cm_compact(int64_t N, const int32_t* __restrict__ cam_pm,
                                                           const int32_t* __restrict__ cam_off,
                                                           int32_t* __restrict__ cm_order) {
  // N <= 64 x 1024 (the small path's bound): thread t looks at observations
  // t, t + 1024, ...; all loads first (one round trip), the hits as bits of
  // one mask, the per-(step, wave) counts scanned once in LDS, then the
  // scatter with the ballots recomputed from the masks.
  __shared__ int cnt[kSmallCmMaxSteps * 16];
  const int c = blockIdx.x, t = threadIdx.x, l = t & 63, w = t >> 6;
  const uint64_t lt = (l == 0) ? 0ull : (~0ull >> (64 - l));
  const int K = int((N + 1023) / 1024);
  uint64_t hits = 0;
#pragma unroll 8
  for (int k = 0; k < K; ++k) {
    const int64_t q = int64_t(k) * 1024 + t;
    if (q < N && cam_pm[q] == c) hits |= 1ull << k;
  }
  for (int k = 0; k < K; ++k) {
    const uint64_t m = __builtin_amdgcn_ballot_w64((hits >> k) & 1);
    if (l == 0) cnt[16 * k + w] = __popcll(m);
  }
  __syncthreads();
  // exclusive scan of the K x 16 counts in (step, wave) order: thread e
  // holds entry e (K x 16 <= 1024)
  __shared__ int wsum[16];
  const int ne = 16 * K;
  const int v = t < ne ? cnt[t] : 0;
  int incl = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(incl, off);
    if (l >= off) incl += o;
  }
  if (l == 63) wsum[w] = incl;
  __syncthreads();
  int wbase = 0;
  for (int u = 0; u < w; ++u) wbase += wsum[u];
  if (t < ne) cnt[t] = wbase + incl - v;
  __syncthreads();
  const int base = cam_off[c];
  for (int k = 0; k < K; ++k) {
    const uint64_t m = __builtin_amdgcn_ballot_w64((hits >> k) & 1);
    if ((hits >> k) & 1) cm_order[base + cnt[16 * k + w] + __popcll(m & lt)] = int32_t(int64_t(k) * 1024 + t);
  }
}
// The chunk table grouped by point slice (k_chunk_keys' key), stable: the
// keys by the whole workgroup into LDS, then wave 0 ranks them, 64 chunks at
// a time, by ballot.
constexpr int kSmallChunks = 2048;
__global__ __launch_bounds__(1024) void k_small_chunks(int n, const int4* __restrict__ ch,
                                                       const int32_t* __restrict__ cm_order,
                                                       const int32_t* __restrict__ pt_s, int P, int4* __restrict__ out,
                                                       int32_t* __restrict__ grp) {
  __shared__ unsigned char key[kSmallChunks];
  for (int t = threadIdx.x; t < n; t += 1024)
    key[t] = (unsigned char)(int64_t(pt_s[cm_order[ch[t].w]]) * 8 / max(1, P));
  __syncthreads();
  if (threadIdx.x >= 64) return;
  const int l = threadIdx.x;
  const uint64_t lt = (l == 0) ? 0ull : (~0ull >> (64 - l));
  int cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int b = 0; b < n; b += 64) {
    const int t = b + l, k = t < n ? int(key[t]) : -1;
#pragma unroll
    for (int g = 0; g < 8; ++g) cnt[g] += __popcll(__builtin_amdgcn_ballot_w64(k == g));
  }
  int start[9];
  start[0] = 0;
#pragma unroll
  for (int g = 0; g < 8; ++g) start[g + 1] = start[g] + cnt[g];
  if (l <= 8) {
    int v = 0;
#pragma unroll
    for (int g = 0; g <= 8; ++g) v = l == g ? start[g] : v;
    grp[l] = v;
  }
  for (int b = 0; b < n; b += 64) {
    const int t = b + l, k = t < n ? int(key[t]) : -1;
    int dst = 0;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const uint64_t m = __builtin_amdgcn_ballot_w64(k == g);
      if (k == g) dst = start[g] + __popcll(m & lt);
      start[g] += __popcll(m);
    }
    if (t < n) {
      const int4 v = ch[t];
      out[dst] = make_int4(v.x, v.y, v.z, 0);
    }
  }
}
// Block b = (c1, c2), c1 <= c2 (row-major over the upper triangle, k_blk's).
__device__ __forceinline__ int2 small_block(int64_t b, int C) {
  int c1 = 0;
  while (c1 + 1 < C && int64_t(c1 + 1) * C - int64_t(c1 + 1) * c1 / 2 <= b) ++c1;
  const int64_t rs = int64_t(c1) * C - int64_t(c1) * (c1 - 1) / 2 - c1;
  return make_int2(c1, int(b - rs));
}
// Camera-major entry i of c1 (o1, point p) in block (c1, c2): the pairs are
// the observations o2 of p with camera c2, o2 != o1.  A point's point-major
// segment is sorted by camera, so they are one run; its length (minus o1
// itself when c2 == c1) is the count, and every pair stores p.  The segment
// is read four entries at a time (independent loads).
__device__ __forceinline__ int small_pairs_of(int i, int c1, int c2, const int32_t* __restrict__ cm_order,
                                              const int32_t* __restrict__ cam_pm, const int32_t* __restrict__ pt_s,
                                              const int32_t* __restrict__ pt_off, int& p) {
  const int32_t o1 = cm_order[i];
  p = pt_s[o1];
  const int q0 = pt_off[p], q1 = pt_off[p + 1];
  int k = 0;
  for (int q = q0; q < q1; q += 4) {
    int cj[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) cj[j] = cam_pm[min(q + j, q1 - 1)];
#pragma unroll
    for (int j = 0; j < 4; ++j) k += (q + j < q1 && cj[j] == c2) ? 1 : 0;
  }
  return k - (c2 == c1 ? 1 : 0);
}
// One workgroup per block: its pair count.
__global__ __launch_bounds__(kT) void k_small_pair_count(int C, const int32_t* __restrict__ cam_off,
                                                         const int32_t* __restrict__ cm_order,
                                                         const int32_t* __restrict__ cam_pm,
                                                         const int32_t* __restrict__ pt_s,
                                                         const int32_t* __restrict__ pt_off, int32_t* __restrict__ cnt) {
  __shared__ int sh[kT / 64];
  const int2 cc = small_block(blockIdx.x, C);
  int k = 0, p;
  for (int i = cam_off[cc.x] + threadIdx.x; i < cam_off[cc.x + 1]; i += kT)
    k += small_pairs_of(i, cc.x, cc.y, cm_order, cam_pm, pt_s, pt_off, p);
  for (int off = 32; off > 0; off >>= 1) k += __shfl_xor(k, off);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = k;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}
// seg = exclusive sum of the n block counts (seg[n] = total), one workgroup.
__global__ __launch_bounds__(1024) void k_small_scan(int64_t n, const int32_t* __restrict__ cnt,
                                                     int32_t* __restrict__ seg) {
  __shared__ int32_t part[1024];
  const int t = threadIdx.x;
  const int64_t per = (n + 1023) / 1024, a = std::min<int64_t>(n, t * per), e = std::min<int64_t>(n, a + per);
  int32_t sum = 0;
  for (int64_t i = a; i < e; ++i) sum += cnt[i];
  part[t] = sum;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int32_t v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int32_t run = part[t] - sum;
  for (int64_t i = a; i < e; ++i) {
    seg[i] = run;
    run += cnt[i];
  }
  if (t == 1023) seg[n] = part[t];
}
// One workgroup per block: its list in (o1 camera-major, o2 point-major)
// order, 256 camera-major entries at a time, positions by a prefix sum.
__global__ __launch_bounds__(kT) void k_small_pair_fill(int C, const int32_t* __restrict__ cam_off,
                                                        const int32_t* __restrict__ cm_order,
                                                        const int32_t* __restrict__ cam_pm,
                                                        const int32_t* __restrict__ pt_s,
                                                        const int32_t* __restrict__ pt_off,
                                                        const int32_t* __restrict__ seg, int32_t* __restrict__ bpts) {
  __shared__ int sc[kT];
  const int2 cc = small_block(blockIdx.x, C);
  const int t = threadIdx.x, i0 = cam_off[cc.x], i1 = cam_off[cc.x + 1];
  int run = seg[blockIdx.x];
  for (int b = i0; b < i1; b += kT) {
    const int i = b + t;
    int p = 0;
    const int k = i < i1 ? small_pairs_of(i, cc.x, cc.y, cm_order, cam_pm, pt_s, pt_off, p) : 0;
    sc[t] = k;
    __syncthreads();
    for (int off = 1; off < kT; off <<= 1) {
      const int v = t >= off ? sc[t - off] : 0;
      __syncthreads();
      sc[t] += v;
      __syncthreads();
    }
    for (int j = 0; j < k; ++j) bpts[run + sc[t] - k + j] = p;
    run += sc[kT - 1];
    __syncthreads();
  }
}

int bits_for(uint64_t max_key) {
  int b = 1;
  while (b < 64 && (max_key >> b) != 0) ++b;
  return b;
}

}  // namespace

size_t setup_sort_bytes(int64_t n, int which) {
  size_t bytes = 0;
  if (n <= 0) return 0;
  if (which == 64)
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, int(n));
  else if (which == 32)
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, int(n));
  else if (which == 1)
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const int32_t*)nullptr, (int32_t*)nullptr, int(n));
  else
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const int64_t*)nullptr, (int64_t*)nullptr, int(n));
  return bytes;
}

hipError_t sort_pairs64(void* tmp, size_t bytes, const uint64_t* kin, uint64_t* kout, const int32_t* vin,
                        int32_t* vout, int64_t n, uint64_t max_key, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, kin, kout, vin, vout, int(n), 0, bits_for(max_key), s);
}
hipError_t sort_pairs32(void* tmp, size_t bytes, const uint32_t* kin, uint32_t* kout, const int32_t* vin,
                        int32_t* vout, int64_t n, uint64_t max_key, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, kin, kout, vin, vout, int(n), 0, bits_for(max_key), s);
}
hipError_t exclusive_sum32(void* tmp, size_t bytes, const int32_t* in, int32_t* out, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, out, int(n), s);
}
hipError_t exclusive_sum64(void* tmp, size_t bytes, const int64_t* in, int64_t* out, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, out, int(n), s);
}

void launch_validate(int64_t N, const double* uv, const int32_t* cam, const int32_t* pt, int C, int P, int32_t* err,
                     int32_t* cam_cnt, int32_t* pt_cnt, hipStream_t s) {
  if (N <= 0) return;
  k_validate<<<std::min(nblocks(N), 1024), kT, 0, s>>>(N, uv, cam, pt, C, P, err, cam_cnt, pt_cnt);
}
void launch_pm_keys(int64_t N, const int32_t* cam, const int32_t* pt, int C, uint64_t* keys, int32_t* iota,
                    hipStream_t s) {
  if (N > 0) k_pm_keys<<<nblocks(N), kT, 0, s>>>(N, cam, pt, C, keys, iota);
}
void launch_gather_pm(int64_t N, const int32_t* order, const double* uv, const int32_t* cam, const int32_t* pt,
                      double* uv_pm, int32_t* cam_pm, int32_t* pt_s, uint32_t* cam_key, int32_t* iota,
                      hipStream_t s) {
  if (N > 0) k_gather_pm<<<nblocks(N), kT, 0, s>>>(N, order, uv, cam, pt, uv_pm, cam_pm, pt_s, cam_key, iota);
}
void launch_fill_cm(int64_t N_pad, const int32_t* wcam, const int32_t* cam_rng, const int32_t* cam_off,
                    const int32_t* cm_order, const int32_t* pt_s, const double* uv_pm, int32_t* cm_p, double* uv_cm,
                    int32_t* cam_obs, int32_t* pos, hipStream_t s) {
  if (N_pad > 0)
    k_fill_cm<<<nblocks(N_pad), kT, 0, s>>>(N_pad, wcam, cam_rng, cam_off, cm_order, pt_s, uv_pm, cm_p, uv_cm, cam_obs,
                                            pos);
}
void launch_uv_layout(int64_t N, int64_t N_pad, const int32_t* order, const int32_t* wcam, const int32_t* cam_rng,
                      const int32_t* cam_off, const int32_t* cm_order, const double* uv, double* uv_pm, double* uv_cm,
                      int32_t* err, hipStream_t s) {
  const int64_t n = std::max(N, N_pad);
  if (n > 0)
    k_uv_layout<<<nblocks(n), kT, 0, s>>>(N, N_pad, order, wcam, cam_rng, cam_off, cm_order, uv, uv_pm, uv_cm, err);
}
void launch_chunk_keys(int n, const int4* ch, const int32_t* cm_order, const int32_t* pt_s, int P, uint32_t* key,
                       int32_t* iota, hipStream_t s) {
  if (n > 0) k_chunk_keys<<<nblocks(n), kT, 0, s>>>(n, ch, cm_order, pt_s, P, key, iota);
}
void launch_chunk_gather(int n, const int32_t* perm, const int4* ch, const uint32_t* key, int4* out, int32_t* grp,
                         hipStream_t s) {
  k_chunk_gather<<<nblocks(std::max(n, 9)), kT, 0, s>>>(n, perm, ch, key, out, grp);
}
void launch_pair_count(int64_t N, const int32_t* cm_order, const int32_t* cam_pm, const int32_t* pt_s,
                       const int32_t* pt_off, int64_t* cnt, hipStream_t s) {
  k_pair_count<<<nblocks(N + 1), kT, 0, s>>>(N, cm_order, cam_pm, pt_s, pt_off, cnt);
}
void launch_pair_fill(int64_t N, const int32_t* cm_order, const int32_t* cam_pm, const int32_t* pt_s,
                      const int32_t* pt_off, const int64_t* off, int C, uint32_t* key, int32_t* val, hipStream_t s) {
  if (N > 0) k_pair_fill<<<nblocks(N), kT, 0, s>>>(N, cm_order, cam_pm, pt_s, pt_off, off, C, key, val);
}
void launch_pt_off(int P, const uint64_t* sorted_keys, int64_t N, int C, int32_t* pt_off, hipStream_t s) {
  k_pt_off<<<nblocks(int64_t(P) + 1), kT, 0, s>>>(P, sorted_keys, N, C, pt_off);
}
void launch_seg(int64_t n_blk, const uint32_t* key, int64_t n_pairs, int32_t* seg, hipStream_t s) {
  k_seg<<<nblocks(n_blk + 1), kT, 0, s>>>(n_blk, key, n_pairs, seg);
}
void launch_copy_from_host(void* dst, const void* src_host_mapped, size_t bytes, hipStream_t s) {
  const int64_t n16 = int64_t(bytes / 16);
  if (n16 > 0)
    k_copy_from_host<<<int(std::min<int64_t>(nblocks(n16), 256)), kT, 0, s>>>(
        static_cast<uint4*>(dst), static_cast<const uint4*>(src_host_mapped), n16);
}
// up to 4 small device -> pinned host copies (4-B words) by one workgroup:
// readbacks that must not queue behind a DMA on the copy engine
__global__ __launch_bounds__(kT) void k_copy_to_host(HostCopySet cs) {
  for (int k = 0; k < cs.n; ++k)
    for (int i = threadIdx.x; i < cs.words[k]; i += kT) cs.dst[k][i] = cs.src[k][i];
}
void launch_copy_to_host(const HostCopySet& cs, hipStream_t s) {
  if (cs.n > 0) k_copy_to_host<<<1, kT, 0, s>>>(cs);
}
void launch_fill32(const Fill32Set& fs, hipStream_t s) {
  if (fs.n == 0) return;
  int64_t mx = 1;
  for (int i = 0; i < fs.n; ++i) mx = std::max(mx, fs.job[i].n);
  const unsigned gx = unsigned(std::min<int64_t>(1024, (mx + kT - 1) / kT));
  k_fill32<<<dim3(gx, unsigned(fs.n)), kT, 0, s>>>(fs);
}
void launch_blk(int C, int2* blk, hipStream_t s) {
  if (C > 0) k_blk<<<dim3(unsigned((C + kT - 1) / kT), unsigned(C)), kT, 0, s>>>(C, blk);
}
void launch_small_pm(int64_t N, const int32_t* pt, const int32_t* cam, const double* uv, const int32_t* pt_off,
                     int32_t* fill, int32_t* tmp, int32_t* order, double* uv_pm, int32_t* cam_pm, int32_t* pt_s,
                     hipStream_t s) {
  if (N <= 0) return;
  k_small_pm_scatter<<<nblocks(N), kT, 0, s>>>(N, pt, pt_off, fill, tmp);
  k_small_pm_rank<<<nblocks(N), kT, 0, s>>>(N, pt_off, tmp, cam, pt, uv, order, uv_pm, cam_pm, pt_s);
}
void launch_small_cm(int64_t N, int C, const int32_t* cam_pm, const int32_t* cam_off, int32_t* cm_order,
                     hipStream_t s) {
  if (N <= 0 || C <= 0 || N > kSmallSetupMaxObs) return;  // (set_problem's small-path bound)
  k_small_cm_compact<<<C, 1024, 0, s>>>(N, cam_pm, cam_off, cm_order);
}
void launch_small_chunks(int n, const int4* ch, const int32_t* cm_order, const int32_t* pt_s, int P, int4* out,
                         int32_t* grp, hipStream_t s) {
  k_small_chunks<<<1, 1024, 0, s>>>(n, ch, cm_order, pt_s, P, out, grp);
}
void launch_small_pairs_count(int C, int64_t n_blk, const int32_t* cam_off, const int32_t* cm_order,
                              const int32_t* cam_pm, const int32_t* pt_s, const int32_t* pt_off, int32_t* cnt,
                              int32_t* seg, hipStream_t s) {
  if (n_blk <= 0) return;
  k_small_pair_count<<<unsigned(n_blk), kT, 0, s>>>(C, cam_off, cm_order, cam_pm, pt_s, pt_off, cnt);
  k_small_scan<<<1, 1024, 0, s>>>(n_blk, cnt, seg);
}
void launch_small_pairs_fill(int C, int64_t n_blk, const int32_t* cam_off, const int32_t* cm_order,
                             const int32_t* cam_pm, const int32_t* pt_s, const int32_t* pt_off, const int32_t* seg,
                             int32_t* bpts, hipStream_t s) {
  if (n_blk > 0) k_small_pair_fill<<<unsigned(n_blk), kT, 0, s>>>(C, cam_off, cm_order, cam_pm, pt_s, pt_off, seg, bpts);
}
int64_t bperm_slots_bound(int64_t n_blk, int per) { return std::max<int64_t>(1, (n_blk + per - 1) / per) * 8 * per; }
hipError_t launch_bperm(int C, int64_t n_blk, int64_t n_pairs, const int32_t* seg, const int2* blk, int per,
                        uint32_t* key_a, uint32_t* key_b, int32_t* iota, int32_t* sorted, int32_t* row_x,
                        int64_t* grp, void* sort_tmp, size_t sort_bytes, int32_t* bperm, hipStream_t s) {
  hipError_t e = hipMemsetAsync(bperm, 0xFF, sizeof(int32_t) * size_t(bperm_slots_bound(n_blk, per)), s);
  if (e != hipSuccess || n_blk <= 0) return e;
  k_bperm_rows<<<1, kT, 0, s>>>(C, seg, n_pairs, n_blk, row_x, grp);
  const int cbits = 32 - bits_for(uint64_t(std::max(1, C)) - 1);
  k_bperm_keys<<<nblocks(n_blk), kT, 0, s>>>(n_blk, blk, seg, cbits, key_a, iota);
  e = sort_pairs32(sort_tmp, sort_bytes, key_a, key_b, iota, sorted, n_blk, ~uint64_t(0) >> 32, s);
  if (e != hipSuccess) return e;
  k_bperm_fill<<<nblocks(n_blk), kT, 0, s>>>(n_blk, sorted, blk, row_x, grp, per, bperm);
  return hipGetLastError();
}

}  // namespace sfm
