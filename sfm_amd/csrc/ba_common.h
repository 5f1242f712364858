// Small wave-level helpers shared by the bundle-adjustment kernels
// (ba_kernels.hip, chol_kernels.hip, ba_setup.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cmath>
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
// sc1: the results stored write-through (sc1), for a consumer in the same
// launch that loads them sc1 after the counter (k_reduce_batch_lm).
__device__ __forceinline__ void reduce_batch_job(const double* __restrict__ partials, int64_t max_blocks,
                                                 const ReduceJob& j, double* __restrict__ scal,
                                                 const int* __restrict__ fail, double* sh, bool sc1 = false) {
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
    if (sc1) {
      __hip_atomic_store(scal + j.dst, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (fail)
        __hip_atomic_store(reinterpret_cast<int*>(scal + kNumScalars), *fail, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    } else {
      scal[j.dst] = r;
      if (fail) *reinterpret_cast<int*>(scal + kNumScalars) = *fail;
    }
  }
}
// Fixed-order block reduction; result valid in thread 0.  `sh` >= 4 doubles.
__device__ __forceinline__ double block_reduce(double v, double* sh, bool is_max) {
  v = is_max ? wave_max(v) : wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  double r = 0.0;
  if (threadIdx.x == 0) {
    const int nw = blockDim.x >> 6;
    r = sh[0];
    for (int i = 1; i < nw; ++i) r = is_max ? fmax(r, sh[i]) : r + sh[i];
  }
  return r;
}

// Rotation matrix R(w) with the branch of ceres::AngleAxisRotatePoint:
// theta^2 > DBL_EPSILON -> Rodrigues; otherwise the first-order map I + [w]x.
// Optionally dR/dw_k (k-major, 3 x row-major 3x3), differentiated through
// the same expressions the Jet evaluation of the reference functor uses.
//
// Contraction is pinned here (not left to the translation unit's flags):
// k_cam_prep (ba_kernels.hip) and the device LM loop's accept fold
// (ba_solver.hip) both call this, and the device loop must equal the host
// loop bitwise.  `fast` is hipcc's default, i.e. the rounding every parity
// scene was pinned with (contract(on) moved the second LM decision of the
// radius-1e15 gauge scene, measured: the scenes' decisions there are
// rounding-decided, tests/test_gpu_lm_branches.py).
__device__ void rotation(const double w[3], double R[9], double* dR) {
#pragma clang fp contract(fast)
  const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  if (th2 > DBL_EPSILON) {
    const double th = sqrt(th2);
    double s, c;
    sincos(th, &s, &c);
    const double ith = 1.0 / th;
    const double u[3] = {w[0] * ith, w[1] * ith, w[2] * ith};
    const double omc = 1.0 - c;
    R[0] = c + omc * u[0] * u[0];        R[1] = -s * u[2] + omc * u[0] * u[1]; R[2] = s * u[1] + omc * u[0] * u[2];
    R[3] = s * u[2] + omc * u[1] * u[0]; R[4] = c + omc * u[1] * u[1];        R[5] = -s * u[0] + omc * u[1] * u[2];
    R[6] = -s * u[1] + omc * u[2] * u[0]; R[7] = s * u[0] + omc * u[2] * u[1]; R[8] = c + omc * u[2] * u[2];
    if (dR) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const double dc = -s * u[k], ds = c * u[k], domc = s * u[k];
        double du[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) du[i] = ((i == k ? 1.0 : 0.0) - u[i] * u[k]) * ith;
        double* D = dR + 9 * k;
        // d/dw_k of: c I + s [u]x + omc u u^T
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j)
            D[3 * i + j] = (i == j ? dc : 0.0) + domc * u[i] * u[j] + omc * (du[i] * u[j] + u[i] * du[j]);
        // skew parts: [a]x = [[0,-a2,a1],[a2,0,-a0],[-a1,a0,0]] with a = ds*u + s*du
        const double a0 = ds * u[0] + s * du[0], a1 = ds * u[1] + s * du[1], a2 = ds * u[2] + s * du[2];
        D[1] -= a2; D[2] += a1; D[3] += a2; D[5] -= a0; D[6] -= a1; D[7] += a0;
      }
    }
  } else {
    R[0] = 1.0;   R[1] = -w[2]; R[2] = w[1];
    R[3] = w[2];  R[4] = 1.0;   R[5] = -w[0];
    R[6] = -w[1]; R[7] = w[0];  R[8] = 1.0;
    if (dR) {
      for (int i = 0; i < 27; ++i) dR[i] = 0.0;
      // d([w]x)/dw_k = [e_k]x
      dR[0 * 9 + 5] = -1.0; dR[0 * 9 + 7] = 1.0;
      dR[1 * 9 + 2] = 1.0;  dR[1 * 9 + 6] = -1.0;
      dR[2 * 9 + 1] = -1.0; dR[2 * 9 + 3] = 1.0;
    }
  }
}

// One camera of the LM step (k_cam_update, and k_chol_small's tail for
// small systems): x_new = x - scale * y, the step's squared length and a
// non-finite flag accumulated into st / bad, the new pose and its rotation
// matrix (camRn: R 9 | t 3).
__device__ __forceinline__ void cam_update_one(int c, const double* __restrict__ cam, const double* __restrict__ ysol,
                                               const double* __restrict__ scale_c, double* __restrict__ cam_new,
                                               double* __restrict__ camRn, double& st, double& bad) {
#pragma clang fp contract(fast)  // (as rotation(): k_cam_update and k_chol_small must agree bitwise)
  double xn[6];
  for (int k = 0; k < 6; ++k) {
    const double y = ysol[6 * c + k];
    if (!isfinite(y)) bad = 1.0;
    const double dx = scale_c[6 * c + k] * (-y);
    xn[k] = cam[6 * c + k] + dx;
    const double d = cam[6 * c + k] - xn[k];
    st += d * d;
    cam_new[6 * c + k] = xn[k];
  }
  double R[9];
  rotation(xn, R, nullptr);
  double* o = camRn + 12 * size_t(c);
  for (int i = 0; i < 9; ++i) o[i] = R[i];
  o[9] = xn[3]; o[10] = xn[4]; o[11] = xn[5];
}
// Wave sums of 32 values at once by recursive halving (reduce-scatter): at
// each of the 5 exchange distances 32..2 a lane keeps half of its values and
// trades the other half with its partner, then the two lanes of a pair add
// once more.  32 shuffles instead of 32 x 6; lane l returns the sum of
// value l >> 1 over the wave (fixed order: deterministic).
// Distances 32 and 16 (24 of the 31 traded values) go through gfx950's
// half-wave / row swaps: swapping the upper half of v[j] with the lower half
// of v[h + j] leaves each lane its own kept value and its partner's in the
// two registers, so no select and no LDS crossbar; the sum is the same pair
// of values either way.  Distances 8..2 trade through ds_bpermute.
// (The halves are picked with bit masks: a select between two array
// elements becomes a select of addresses and pushes the array to scratch.)
__device__ __forceinline__ void swap_halves32(double& x, double& y) {  // x lanes 32..63 <-> y lanes 0..31
  const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(x), __double2loint(y), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(x), __double2hiint(y), false, false);
  x = __hiloint2double(hi[0], lo[0]);
  y = __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ void swap_rows16(double& x, double& y) {  // x odd 16-lane rows <-> y even rows
  const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(x), __double2loint(y), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(x), __double2hiint(y), false, false);
  x = __hiloint2double(hi[0], lo[0]);
  y = __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ double wave_sum32(double (&v)[32], int l) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {  // distance 32: lanes 0..31 keep v[0..16), 32..63 v[16..32)
    swap_halves32(v[j], v[16 + j]);
    v[j] = v[j] + v[16 + j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {  // distance 16: even rows keep v[0..8), odd rows v[8..16)
    swap_rows16(v[j], v[8 + j]);
    v[j] = v[j] + v[8 + j];
  }
#pragma unroll
  for (int h = 4; h >= 1; h >>= 1) {
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

// IEEE divisions by one shared denominator: the compiler's f64 division is
// v_div_scale (denominator) -> v_rcp -> two Newton steps -> v_div_scale
// (numerator) -> q = n r -> e = n - q z -> v_div_fmas (q + e r) ->
// v_div_fixup, i.e. ~11 instructions, the reciprocal part repeated for every
// numerator.  For operands in the normal range div_scale, div_fmas' scaling
// and div_fixup are identities, so refining the reciprocal once and running
// only the numerator's three steps gives the same bits (an observation's
// x/z, y/z and 1/z: 13 instructions instead of ~33).  Outside that range --
// z = 0, denormal or near-overflow operands -- the result differs from the
// division's (NaN for inf at z = 0), and is non-finite or meaningless alike:
// the LM treats either as an invalid step.
struct SharedDiv {
  double z, r;
};
__device__ __forceinline__ SharedDiv shared_div(double z) {
  double r = __builtin_amdgcn_rcp(z);
  double e = fma(-z, r, 1.0);
  r = fma(r, e, r);
  e = fma(-z, r, 1.0);
  r = fma(r, e, r);
  return SharedDiv{z, r};
}
__device__ __forceinline__ double sdiv(const SharedDiv& d, double n) {
  const double q = n * d.r;
  const double e = fma(-d.z, q, n);
  return fma(e, d.r, q);
}
// 1 / z (q = 1 * r = r)
__device__ __forceinline__ double srcp(const SharedDiv& d) { return fma(fma(-d.z, d.r, 1.0), d.r, d.r); }
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
