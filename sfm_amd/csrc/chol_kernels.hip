// Dense reduced-camera Cholesky for gfx950: the replacement of the Eigen
// LLT that Ceres' DenseSchurComplementSolver runs on the reduced camera
// matrix (DENSE_SCHUR, /root/reference/CTracker.cpp:574).
//
// Storage: column-major lower triangle (element (i, j), i >= j, at j*ld + i),
// which is byte-identical to the row-major upper triangle the Schur kernel
// writes.  Row n (= 6C) holds the reduced right-hand side, so factoring the
// augmented matrix performs the forward substitution z = L^-1 rhs for free;
// rows beyond n are identity padding up to a multiple of the 64-wide tile.
//
// Right-looking blocked algorithm, tile 64, three launches per step k:
//   k_chol_potrf : factor tile (k,k) in registers (one workgroup), store
//                  1/L_jj for the substitutions
//   k_chol_trsm  : panel tiles (i,k) <- A_ik L_kk^-T by column substitution
//                  (no barriers: rows are independent)
//   k_chol_syrk  : trailing tiles (i,j) -= L_ik L_jk^T on v_mfma_f64_16x16x4_f64,
//                  operands loaded straight into registers
// and the back substitution L^T y = z (one launch per tile row, each
// workgroup solving the 64x64 diagonal block redundantly).
#include <hip/hip_runtime.h>
#include <cmath>
#include "ba_device.h"

namespace sfm {
namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int NB = kNB;  // 64

// ---------------------------------------------------------------------------
// Pivot: 1/sqrt(d) by the hardware estimate + two Newton steps (full double
// precision), sqrt(d) = d * (1/sqrt(d)).  Keeps the pivot chain short.
__device__ __forceinline__ double rsqrt_nr(double d) {
  double y = __builtin_amdgcn_rsq(d);
  y = y * fma(-0.5 * d * y, y, 1.5);
  y = y * fma(-0.5 * d * y, y, 1.5);
  return y;
}

// Uniform broadcast of lane `src`'s double (two v_readlane_b32 -> SGPRs).
__device__ __forceinline__ double bcast(double v, int src) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
  return __hiloint2double(hi, lo);
}

// POTRF of one 64x64 tile by ONE wavefront.  Lane r holds row r of the tile
// (a[j] = A(r, j), upper part taken from the symmetric lower storage), so
// for column j lane r's own a[j] = A(r, j) = A(j, r) and no column ever has
// to be gathered:
//   pivot  d = a[j] of lane j           (readlane broadcast)
//   l_r    = a[j] / sqrt(d)             (own register: L(r, j))
//   update a[c] -= l_r * L(c, j), c > j (L(c, j) by LDS broadcast reads)
// Fully unrolled (register indices are compile-time), one 64-lane LDS store
// and no barrier per column: the pivot chain is readlane -> rsq -> mul.
__global__ __launch_bounds__(64) void k_chol_potrf(double* __restrict__ A, int ld, int k, int n,
                                                   double* __restrict__ invd, int* __restrict__ fail) {
  __shared__ __attribute__((aligned(16))) double colb[NB];
  const int r = threadIdx.x;
  const int k0 = k * NB;
  double a[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j)
    a[j] = (j <= r) ? A[size_t(k0 + j) * ld + k0 + r] : A[size_t(k0 + r) * ld + k0 + j];
  bool bad = false;
  double myinv = 0.0;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const double d = bcast(a[j], j);
    bad |= !(d > 0.0) && (k0 + j) < n;
    const double inv = rsqrt_nr(d);
    if (r == j) myinv = inv;
    const double l = a[j] * inv;  // L(r, j) for r >= j (r == j: sqrt(d))
    a[j] = l;
    colb[r] = l;
    if (j < NB - 1) {
#pragma unroll
      for (int c = j + 1; c < NB; ++c) a[c] = fma(-l, colb[c], a[c]);
    }
  }
  if (bad && r == 0) atomicOr(fail, 1);
  invd[k0 + r] = myinv;
#pragma unroll
  for (int j = 0; j < NB; ++j)
    if (j <= r) A[size_t(k0 + j) * ld + k0 + r] = a[j];
}

// ---------------------------------------------------------------------------
// Panel tiles (i, k), i > k:  X L_kk^T = B.  One thread per tile row (row r
// of B in registers), one wavefront per tile, four tiles per workgroup
// sharing L_kk in LDS.  Column j: x_j *= 1/L_jj, then x_c -= x_j L(c, j)
// for c > j with L(c, j) read as an LDS broadcast; no cross-lane traffic.
__global__ __launch_bounds__(256) void k_chol_trsm(double* __restrict__ A, int ld, int k, int m,
                                                   const double* __restrict__ invd) {
  __shared__ __attribute__((aligned(16))) double Lc[NB][NB];  // Lc[j][c] = L_kk(c, j)
  __shared__ double id[NB];
  const int t = threadIdx.x, r = t & 63, w = t >> 6;
  const int k0 = k * NB;
  const int tile = 4 * blockIdx.x + w;  // panel tile index (0-based below the diagonal)
  {
    double v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = t + 256 * q, j = e >> 6, c = e & 63;
      v[q] = A[size_t(k0 + j) * ld + k0 + c];
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = t + 256 * q, j = e >> 6, c = e & 63;
      Lc[j][c] = v[q];
    }
  }
  if (t < NB) id[t] = invd[k0 + t];
  const bool active = tile < m;
  const int i0 = (k + 1 + (active ? tile : 0)) * NB;
  double x[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c) x[c] = active ? A[size_t(k0 + c) * ld + i0 + r] : 0.0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    x[j] *= id[j];
    if (j < NB - 1) {
#pragma unroll
      for (int c = j + 1; c < NB; ++c) x[c] = fma(-x[j], Lc[j][c], x[c]);
    }
  }
  if (active) {
#pragma unroll
    for (int c = 0; c < NB; ++c) A[size_t(k0 + c) * ld + i0 + r] = x[c];
  }
}

// ---------------------------------------------------------------------------
// Trailing update of tile (i, j), k < j <= i:  A_ij -= L_ik L_jk^T.
// Computed transposed, D[c][r] = sum_l L_jk[c][l] L_ik[r][l], so the MFMA's
// D column (lane & 15) walks the tile's rows: each register of the
// accumulator maps to 16 consecutive doubles of one column of A (128 B).
// v_mfma_f64_16x16x4_f64 lane maps (cdna_hip_programming.md §3):
//   A[i = l&15][k = l>>4], B[k = l>>4][j = l&15], D col = l&15, row = (l>>4) + 4*reg.
// Operands go straight from L2 into registers (no LDS): wave w owns the
// 32x32 quadrant (c in 32*(w>>1).., r in 32*(w&1)..) and loads all 64 k
// of its 2+2 fragments before the MFMA chain.
__global__ __launch_bounds__(256) void k_chol_syrk(double* __restrict__ A, int ld, int k) {
  int i, j;
  {
    const int b = blockIdx.x;
    int ii = int((sqrt(8.0 * b + 1.0) - 1.0) * 0.5);
    while ((ii + 1) * (ii + 2) / 2 <= b) ++ii;
    while (ii * (ii + 1) / 2 > b) --ii;
    i = k + 1 + ii;
    j = k + 1 + (b - ii * (ii + 1) / 2);
  }
  const int k0 = k * NB, i0 = i * NB, j0 = j * NB;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int cb = 32 * (w >> 1), rb = 32 * (w & 1);
  const int lr = lane & 15, lk = lane >> 4;
  if (i == j && cb > rb) return;  // strictly-upper quadrant of a diagonal tile: never read
  double xa[2][16], yb[2][16];
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) {
    const size_t colbase = size_t(k0 + 4 * ks + lk) * ld;
#pragma unroll
    for (int a = 0; a < 2; ++a) xa[a][ks] = A[colbase + j0 + cb + 16 * a + lr];
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) yb[bb][ks] = A[colbase + i0 + rb + 16 * bb + lr];
  }
  double cv[2][2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int bb = 0; bb < 2; ++bb)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg)
        cv[a][bb][reg] = A[size_t(j0 + cb + 16 * a + lk + 4 * reg) * ld + i0 + rb + 16 * bb + lr];
  f64x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) acc[a][bb] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int ks = 0; ks < 16; ++ks)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int bb = 0; bb < 2; ++bb)
        acc[a][bb] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[a][ks], yb[bb][ks], acc[a][bb], 0, 0, 0);
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int bb = 0; bb < 2; ++bb)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg)
        A[size_t(j0 + cb + 16 * a + lk + 4 * reg) * ld + i0 + rb + 16 * bb + lr] = cv[a][bb][reg] - acc[a][bb][reg];
}

// z <- row n of the factor (z = L^-1 rhs), y <- 0
__global__ void k_copy_z(const double* __restrict__ A, int ld, int n, double* __restrict__ z, double* __restrict__ y) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < ld) {
    z[j] = (j < n) ? A[size_t(j) * ld + n] : 0.0;
    y[j] = 0.0;
  }
}

// One step of the blocked back substitution L^T y = z, tile k (descending).
// Every workgroup loads L_kk (all loads in flight at once), wavefront 0
// solves L_kk^T y_k = z_k (redundant across workgroups; workgroup 0 stores
// y_k), then thread l of workgroup b updates z_j, j = 256b + l < k0:
//   z_j -= sum_r L(k0 + r, j) y_k[r]
// from its column's 64 contiguous doubles, prefetched before the solve.
__global__ __launch_bounds__(256) void k_backsolve_step(const double* __restrict__ A, int ld, int n, int k,
                                                        const double* __restrict__ invd, double* __restrict__ z,
                                                        double* __restrict__ y) {
  __shared__ double Lt[NB][NB + 1];  // Lt[r][j] = L_kk(r, j)
  __shared__ double yk[NB];
  const int k0 = k * NB;
  const int nreal = (n - k0) < NB ? (n - k0) : NB;
  const int t = threadIdx.x, lane = t & 63;
  const int j = blockIdx.x * 256 + t;
  const bool upd = j < k0;
  double col[NB];
  if (upd) {
#pragma unroll
    for (int q = 0; q < NB / 2; ++q) {
      const double2 v2 = *reinterpret_cast<const double2*>(A + size_t(j) * ld + k0 + 2 * q);
      col[2 * q] = v2.x;
      col[2 * q + 1] = v2.y;
    }
  }
  {
    double v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = t + 256 * q, jj = e >> 6, r = e & 63;
      v[q] = A[size_t(k0 + jj) * ld + k0 + r];
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = t + 256 * q, jj = e >> 6, r = e & 63;
      Lt[r][jj] = (r >= jj) ? v[q] : 0.0;
    }
  }
  __syncthreads();
  if (t < 64) {
    // lane r holds z_r; descending columns, y_j broadcast by readlane
    double v = (lane < nreal) ? z[k0 + lane] * invd[k0 + lane] : 0.0;
    const double idl = (lane < nreal) ? invd[k0 + lane] : 0.0;
#pragma unroll
    for (int jj = NB - 1; jj >= 0; --jj) {
      if (jj < nreal) {
        const double yj = bcast(v, jj);
        if (lane < jj) v = fma(-Lt[jj][lane] * idl, yj, v);
      }
    }
    if (lane >= nreal) v = 0.0;
    yk[lane] = v;
    if (blockIdx.x == 0 && lane < nreal) y[k0 + lane] = v;
  }
  __syncthreads();
  if (upd) {
    double s = 0.0;
#pragma unroll
    for (int r = 0; r < NB; ++r) s += col[r] * yk[r];
    z[j] -= s;
  }
}

}  // namespace

void launch_cholesky(const DevProblem& d, hipStream_t s) {
  (void)hipMemsetAsync(d.fail, 0, sizeof(int), s);
  for (int k = 0; k < d.nblk; ++k) {
    k_chol_potrf<<<1, 64, 0, s>>>(d.S, d.ld, k, d.n, d.invL, d.fail);
    const int m = d.nblk - k - 1;
    if (m == 0) break;
    k_chol_trsm<<<(m + 3) / 4, 256, 0, s>>>(d.S, d.ld, k, m, d.invL);
    k_chol_syrk<<<m * (m + 1) / 2, 256, 0, s>>>(d.S, d.ld, k);
  }
}

void launch_backsolve(const DevProblem& d, hipStream_t s) {
  k_copy_z<<<(d.ld + 255) / 256, 256, 0, s>>>(d.S, d.ld, d.n, d.zwork, d.ysol);
  const int nb_real = (d.n + NB - 1) / NB;
  for (int k = nb_real - 1; k >= 0; --k)
    k_backsolve_step<<<k > 0 ? (k + 3) / 4 : 1, 256, 0, s>>>(d.S, d.ld, d.n, k, d.invL, d.zwork, d.ysol);
}

}  // namespace sfm
