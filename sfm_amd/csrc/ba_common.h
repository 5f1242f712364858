// Small wave-level helpers shared by the bundle-adjustment kernels
// (ba_kernels.hip, chol_kernels.hip, ba_setup.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "ba_device.h"

namespace sfm {
namespace {
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off));
  return v;
}
// One job of a batched scalar reduction (a 1024-thread workgroup, fixed
// order: bitwise reproducible): scal[j.dst] = sum / max of the job's
// partials; `fail` != nullptr also copies the Cholesky failure int into the
// slot after the scalars.  k_reduce_batch and the device LM loop's
// k_reduce_batch_lm (ba_solver.hip) share it.
__device__ __forceinline__ void reduce_batch_job(const double* __restrict__ partials, int64_t max_blocks,
                                                 const ReduceJob& j, double* __restrict__ scal,
                                                 const int* __restrict__ fail, double* sh) {
  const double* src = partials + size_t(j.slot) * max_blocks;
  double v = 0.0;
  for (int i = threadIdx.x; i < j.nb; i += 1024) v = j.op ? fmax(v, src[i]) : v + src[i];
  v = j.op ? wave_max(v) : wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) sh[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double r = sh[0];
    for (int i = 1; i < 16; ++i) r = j.op ? fmax(r, sh[i]) : r + sh[i];
    scal[j.dst] = r;
    if (fail) *reinterpret_cast<int*>(scal + kNumScalars) = *fail;
  }
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

// Packed upper-triangle index of a 6x6 symmetric matrix.
__device__ __forceinline__ int up6(int a, int b) {
  if (a > b) { int t = a; a = b; b = t; }
  return a * 6 - (a * (a - 1)) / 2 + (b - a);
}

}  // namespace
}  // namespace sfm
