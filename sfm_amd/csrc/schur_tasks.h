// Schur-complement work items shared by the standalone kernels
// (ba_kernels.hip: k_schur_row, k_schur_diag) and the fused Schur +
// Cholesky launch (chol_kernels.hip: k_chol_schur_fused).  Each item runs on
// one 256-thread workgroup with LDS supplied by the caller, so the fused
// kernel can overlay it on the Cholesky's tile buffers.
#pragma once
#include <hip/hip_runtime.h>
#include "ba_device.h"

namespace sfm {
namespace {

constexpr int kSchurThreads = 256;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
// Wave sums of 32 values at once by recursive halving (reduce-scatter): at
// each of the 5 exchange distances 32..2 a lane keeps half of its values and
// trades the other half with its partner, then the two lanes of a pair add
// once more.  32 shuffles instead of 32 x 6; lane l returns the sum of
// value l >> 1 over the wave (fixed order: deterministic).
// (The halves are picked with bit masks: a select between two array
// elements becomes a select of addresses and pushes the array to scratch.)
__device__ __forceinline__ double wave_sum32(double (&v)[32], int l) {
#pragma unroll
  for (int h = 16; h >= 1; h >>= 1) {
    const uint64_t m = (l & (2 * h)) ? ~0ull : 0ull;  // exchange distance 2h
#pragma unroll
    for (int j = 0; j < h; ++j) {
      const uint64_t a = __builtin_bit_cast(uint64_t, v[j]), b = __builtin_bit_cast(uint64_t, v[h + j]);
      const double keep = __builtin_bit_cast(double, (b & m) | (a & ~m));
      const double send = __builtin_bit_cast(double, (a & m) | (b & ~m));
      v[j] = keep + __shfl_xor(send, 2 * h);
    }
  }
  return v[0] + __shfl_xor(v[0], 1);
}
__device__ __forceinline__ double2 ld2(const double* p) { return *reinterpret_cast<const double2*>(p); }
__device__ __forceinline__ void st2(double* p, double a, double b) {
  *reinterpret_cast<double2*>(p) = make_double2(a, b);
}
// Streaming (non-temporal) 16-B store for write-once outputs that the same
// kernel never re-reads: on gfx950 the record stream of the Jacobian pass
// runs at ~5.4 TB/s this way against ~3 TB/s with plain stores (measured:
// plain write-allocating stores evict the L2-resident point data the
// gathers need and stall the store path).
typedef double f64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st2_nt(double* p, double a, double b) {
  const f64x2 v = {a, b};
  __builtin_nontemporal_store(v, reinterpret_cast<f64x2*>(p));
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave-cooperative load of the 64 consecutive R-double records that start at
// g into the wave's LDS slice s, returning this lane's record.  A lane-per-
// record load of an AoS array is a 16-B access at an R*8-B stride: every
// instruction touches 64 cache lines (the vector-memory pipeline pays per
// line); these R/2 coalesced 1-KB rows touch 8 each.
template <int R>
__device__ __forceinline__ const double* wave_records(double* s, const double* __restrict__ g, int l) {
  double2 v[R / 2];
#pragma unroll
  for (int k = 0; k < R / 2; ++k) v[k] = ld2(g + 2 * (64 * k + l));
#pragma unroll
  for (int k = 0; k < R / 2; ++k) st2(s + 2 * (64 * k + l), v[k].x, v[k].y);
  wave_sync_lds();
  return s + l * R;
}

// Packed upper-triangle index of a 6x6 symmetric matrix.
__device__ __forceinline__ int up6(int a, int b) {
  if (a > b) { int t = a; a = b; b = t; }
  return a * 6 - (a * (a - 1)) / 2 + (b - a);
}

// ---------------------------------------------------------------------------
constexpr int kRowCh = 448;  // 63 KB of F records per chunk: two workgroups per CU
// S entry store: plain, or write-through (sc1: the line leaves the XCD's L2
// clean) where a latency-critical agent-scope release on the same XCD must
// not write back megabytes of Schur output (fused launch).
template <bool kWT>
__device__ __forceinline__ void st_s(double* p, double v) {
  if (kWT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

// One work item wk = (c1, first block, block count, -) with 256 threads;
// F1: kRowCh * kFRec doubles of LDS (16-B aligned).  kPairs pairs of a
// block are gathered per step (more loads in flight where occupancy is low);
// the contributions are added in pair order whatever kPairs is, so the sums
// are bitwise the same.
template <int kPairs = 2, bool kWT = false>
__device__ __forceinline__ void schur_row_task(int4 wk, const int32_t* __restrict__ seg, const int2* __restrict__ pairs,
                                               const double* __restrict__ frec, const int32_t* __restrict__ cam_rng,
                                               const int2* __restrict__ blk, double* __restrict__ S, int ld,
                                               double* F1) {
  const int t = threadIdx.x;
  const bool has = t < wk.z;
  const int64_t b = int64_t(wk.y) + t;
  int k = has ? seg[b] : 0;
  const int ke = has ? seg[b + 1] : 0;
  double acc[36];
#pragma unroll
  for (int e = 0; e < 36; ++e) acc[e] = 0.0;
  constexpr int kNone = 0x7fffffff;
  int2 pp[kPairs];
#pragma unroll
  for (int q = 0; q < kPairs; ++q) pp[q] = k + q < ke ? pairs[k + q] : make_int2(kNone, 0);
  const int r0 = cam_rng[2 * wk.x], r1 = cam_rng[2 * wk.x + 1];
  for (int base = r0; base < r1; base += kRowCh) {
    const int cnt = min(kRowCh, r1 - base), end = base + cnt;
    __syncthreads();
    {
      const double2* src = reinterpret_cast<const double2*>(frec + size_t(base) * kFRec);
      double2* dst = reinterpret_cast<double2*>(F1);
      for (int e = t; e < cnt * (kFRec / 2); e += kSchurThreads) dst[e] = src[e];
    }
    __syncthreads();
    while (pp[0].x < end) {
      // pairs are sorted by o1: the valid ones of this step are a prefix
      int nv = 1;
#pragma unroll
      for (int q = 1; q < kPairs; ++q) nv += pp[q].x < end ? 1 : 0;
      double G[kPairs][kFRec];
#pragma unroll
      for (int q = 0; q < kPairs; ++q) {
        const int2 qq = q < nv ? pp[q] : pp[0];
        const double wq = q < nv ? 1.0 : 0.0;
        const double* A2 = frec + size_t(qq.y) * kFRec;
#pragma unroll
        for (int f = 0; f < kFRec; f += 2) {
          const double2 x = ld2(A2 + f);
          G[q][f] = x.x * wq; G[q][f + 1] = x.y * wq;
        }
      }
      int2 o1[kPairs];
#pragma unroll
      for (int q = 0; q < kPairs; ++q) o1[q] = q < nv ? pp[q] : pp[0];
      k += nv;
#pragma unroll
      for (int q = 0; q < kPairs; ++q) pp[q] = k + q < ke ? pairs[k + q] : make_int2(kNone, 0);
#pragma unroll
      for (int q = 0; q < kPairs; ++q) {
        const double* A1 = F1 + (o1[q].x - base) * kFRec;
        double a1[kFRec];
#pragma unroll
        for (int f = 0; f < kFRec; f += 2) {
          const double2 x = ld2(A1 + f);
          a1[f] = x.x; a1[f + 1] = x.y;
        }
#pragma unroll
        for (int u = 0; u < 6; ++u)
#pragma unroll
          for (int v = 0; v < 6; ++v)
            acc[6 * u + v] += a1[3 * u] * G[q][3 * v] + a1[3 * u + 1] * G[q][3 * v + 1] + a1[3 * u + 2] * G[q][3 * v + 2];
      }
    }
  }
  if (!has) return;
  const int2 cc = blk[b];
#pragma unroll
  for (int u = 0; u < 6; ++u) {
    double* row = S + size_t(6 * cc.x + u) * ld + 6 * size_t(cc.y);
    if (kWT) {
#pragma unroll
      for (int v = 0; v < 6; ++v) st_s<true>(row + v, -acc[6 * u + v]);
    } else {
#pragma unroll
      for (int v = 0; v < 6; v += 2) st2(row + v, -acc[6 * u + v], -acc[6 * u + v + 1]);
    }
  }
}

// Camera c with 256 threads; lds: kDiagLds doubles (16-B aligned).
constexpr int kDiagLds = (kSchurThreads / 64) * 64 * (kJRec + kMRec) + (kSchurThreads / 64) * 28;
template <bool kWT = false>
__device__ __forceinline__ void schur_diag_task(int c, const int32_t* __restrict__ cam_rng, const int32_t* __restrict__ cam_obs,
                                const double* __restrict__ jrec, const double* __restrict__ mrec,
                                const double* __restrict__ Ucam, const double* __restrict__ diag_c, double radius,
                                int add_diag, double* __restrict__ S, int ld, int n, double* lds) {
  double (*stage)[64 * (kJRec + kMRec)] = reinterpret_cast<double (*)[64 * (kJRec + kMRec)]>(lds);
  double* red = lds + (kSchurThreads / 64) * 64 * (kJRec + kMRec);
  const int i0 = cam_rng[2 * c], i1 = cam_rng[2 * c + 1];
  double dacc[21], rhs[6];
#pragma unroll
  for (int e = 0; e < 21; ++e) dacc[e] = 0.0;
#pragma unroll
  for (int e = 0; e < 6; ++e) rhs[e] = 0.0;
  const int w0 = threadIdx.x >> 6, l0 = threadIdx.x & 63;
  for (int base = i0 + 64 * w0; base < i1; base += kSchurThreads) {
    // camera-major records, streamed through the wave's LDS slice
    const double* J1p = wave_records<kJRec>(stage[w0], jrec + size_t(base) * kJRec, l0);
    const double* M1p = wave_records<kMRec>(stage[w0] + 64 * kJRec, mrec + size_t(base) * kMRec, l0);
    const bool real = base + l0 < i1;
    double J1[12], M1[8];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const double2 v = ld2(J1p + kJC + 2 * k);
      J1[2 * k] = real ? v.x : 0.0; J1[2 * k + 1] = real ? v.y : 0.0;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double2 v = ld2(M1p + 2 * k);
      M1[2 * k] = real ? v.x : 0.0; M1[2 * k + 1] = real ? v.y : 0.0;
    }
    double2 rr = ld2(J1p + kRes);
    if (!real) rr = make_double2(0.0, 0.0);
    wave_sync_lds();
    double F[kFRec];
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      F[3 * u] = J1[u] * M1[0] + J1[6 + u] * M1[3];
      F[3 * u + 1] = J1[u] * M1[1] + J1[6 + u] * M1[4];
      F[3 * u + 2] = J1[u] * M1[2] + J1[6 + u] * M1[5];
    }
    const double e0 = rr.x - M1[6], e1 = rr.y - M1[7];
#pragma unroll
    for (int u = 0; u < 6; ++u) rhs[u] += J1[u] * e0 + J1[6 + u] * e1;
    int q = 0;
#pragma unroll
    for (int u = 0; u < 6; ++u)
#pragma unroll
      for (int v = u; v < 6; ++v, ++q) dacc[q] += F[3 * u] * F[3 * v] + F[3 * u + 1] * F[3 * v + 1] + F[3 * u + 2] * F[3 * v + 2];
  }
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int e = 0; e < 21; ++e) {
    const double v = wave_sum(dacc[e]);
    if (l == 0) red[w * 28 + e] = v;
  }
#pragma unroll
  for (int e = 0; e < 6; ++e) {
    const double v = wave_sum(rhs[e]);
    if (l == 0) red[w * 28 + 21 + e] = v;
  }
  __syncthreads();
  if (threadIdx.x < 36) {
    const int u = threadIdx.x / 6, v = threadIdx.x % 6, q = up6(u, v);
    double tot = red[q];
    for (int w2 = 1; w2 < kSchurThreads / 64; ++w2) tot += red[28 * w2 + q];
    double* sp = S + size_t(6 * c + u) * ld + 6 * size_t(c) + v;
    double val = *sp - tot;
    if (add_diag) {
      val += Ucam[size_t(kUcam) * c + q];
      if (u == v) { const double dd = sqrt(diag_c[6 * size_t(c) + u] / radius); val += dd * dd; }
    }
    st_s<kWT>(sp, val);
  } else if (threadIdx.x < 42) {
    const int u = threadIdx.x - 36;
    double tot = red[21 + u];
    for (int w2 = 1; w2 < kSchurThreads / 64; ++w2) tot += red[28 * w2 + 21 + u];
    st_s<kWT>(S + size_t(6 * c + u) * ld + n, tot);
  }
}

}  // namespace
}  // namespace sfm
