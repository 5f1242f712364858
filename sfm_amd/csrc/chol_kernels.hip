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
//   k_chol_potrf : factor tile (k,k) in registers (one wavefront) and form
//                  its inverse W_k = L_kk^-1 (stored for the next two)
//   k_chol_trsm  : panel tiles (i,k) <- A_ik W_k^T on MFMA
//   k_chol_syrk  : trailing tiles (i,j) -= L_ik L_jk^T on v_mfma_f64_16x16x4_f64,
//                  operands loaded straight into registers
// and the back substitution L^T y = z (one launch per tile row, y_k = W_k^T z_k
// recomputed by each workgroup, then the update of the rows above).
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

// POTRF of one 64x64 tile plus the tile inverse W = L^-1, two wavefronts.
// Wave 0 factors: lane r holds row r of the tile (a[j] = A(r, j), upper part
// taken from the symmetric lower storage), so for column j lane r's own
// a[j] = A(j, r):
//   pivot  d = a[j] of lane j           (readlane broadcast)
//   l_r    = a[j] / sqrt(d)             (own register: L(r, j))
//   update a[c] -= l_r * L(c, j), c > j (L(c, j) by LDS broadcast reads)
// and leaves every column L(:, j) in LDS.  L = E_0 E_1 ... E_63 with E_j the
// identity whose column j is L(:, j), so wave 1 forms W = E_63^-1 ... E_0^-1
// from those columns, one block of 8 behind wave 0: lane m holds column m
// of W (w[c] = W(c, m)) and applies w[j] *= 1/L(j, j); w[c] -= L(c, j) w[j].
// W turns the panel solve and the back substitution into products
// (k_chol_trsm, k_backsolve_step) with no per-column chain outside this
// kernel.  Fully unrolled; the broadcast reads of a column are issued
// together.  Pivots at or beyond n (augmented row, identity padding) are
// taken as 1 so the padding stays finite; they are never read back.
constexpr int kPotrfBlk = 8;
__global__ __launch_bounds__(128) void k_chol_potrf(double* __restrict__ A, int ld, int k, int n,
                                                    double* __restrict__ Winv, int* __restrict__ fail) {
  __shared__ __attribute__((aligned(16))) double Lcol[NB * NB];  // Lcol[j][c] = L(c, j)
  __shared__ double invs[NB];
  const int r = threadIdx.x & 63;
  const int k0 = k * NB;
  if (threadIdx.x < 64) {
    double a[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j)
      a[j] = (j <= r) ? A[size_t(k0 + j) * ld + k0 + r] : A[size_t(k0 + r) * ld + k0 + j];
    bool bad = false;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      double d = bcast(a[j], j);
      if ((k0 + j) < n) bad |= !(d > 0.0);
      else d = 1.0;
      const double inv = rsqrt_nr(d);
      const double l = a[j] * inv;  // L(r, j) for r >= j (r == j: sqrt(d))
      a[j] = l;
      Lcol[j * NB + r] = l;
      invs[j] = inv;
      if (j < NB - 1) {
        double lc[NB];
#pragma unroll
        for (int c = (j + 1) & ~1; c < NB; c += 2) {
          const double2 v2 = *reinterpret_cast<const double2*>(&Lcol[j * NB + c]);
          lc[c] = v2.x;
          lc[c + 1] = v2.y;
        }
#pragma unroll
        for (int c = j + 1; c < NB; ++c) a[c] = fma(-l, lc[c], a[c]);
      }
      if (j % kPotrfBlk == kPotrfBlk - 1) __syncthreads();
    }
    if (bad && r == 0) atomicOr(fail, 1);
#pragma unroll
    for (int j = 0; j < NB; ++j)
      if (j <= r) A[size_t(k0 + j) * ld + k0 + r] = a[j];
  } else {
    double w[NB];
#pragma unroll
    for (int c = 0; c < NB; ++c) w[c] = (c == r) ? 1.0 : 0.0;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (j % kPotrfBlk == 0) __syncthreads();
      w[j] *= invs[j];
      if (j < NB - 1) {
        double lc[NB];
#pragma unroll
        for (int c = (j + 1) & ~1; c < NB; c += 2) {
          const double2 v2 = *reinterpret_cast<const double2*>(&Lcol[j * NB + c]);
          lc[c] = v2.x;
          lc[c + 1] = v2.y;
        }
#pragma unroll
        for (int c = j + 1; c < NB; ++c) w[c] = fma(-lc[c], w[j], w[c]);
      }
    }
    // W column-major (Wc[m][c] = W(c, m)); lane m writes 64 contiguous doubles
    double* Wk = Winv + size_t(k) * NB * NB + size_t(r) * NB;
#pragma unroll
    for (int c = 0; c < NB; c += 2) *reinterpret_cast<double2*>(Wk + c) = double2{w[c], w[c + 1]};
  }
}

// ---------------------------------------------------------------------------
// Panel tile (i, k), i > k:  X L_kk^T = B  ->  X = B W^T, one workgroup per
// tile on v_mfma_f64_16x16x4_f64, computed transposed like k_chol_syrk:
// D[c][r] = sum_m W(c, m) B(r, m).  X overwrites B in place, so every wave
// finishes its MFMA chain (all operand loads consumed) before any store.
__global__ __launch_bounds__(256) void k_chol_trsm(double* __restrict__ A, int ld, int k,
                                                   const double* __restrict__ Winv) {
  const int k0 = k * NB, i0 = (k + 1 + blockIdx.x) * NB;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int cb = 32 * (w >> 1), rb = 32 * (w & 1);
  const int lr = lane & 15, lk = lane >> 4;
  const double* Wk = Winv + size_t(k) * NB * NB;
  double xa[2][16], yb[2][16];
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) {
    const int m = 4 * ks + lk;
#pragma unroll
    for (int a = 0; a < 2; ++a) xa[a][ks] = Wk[m * NB + cb + 16 * a + lr];
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) yb[bb][ks] = A[size_t(k0 + m) * ld + i0 + rb + 16 * bb + lr];
  }
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
  __syncthreads();
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int bb = 0; bb < 2; ++bb)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg)
        A[size_t(k0 + cb + 16 * a + lk + 4 * reg) * ld + i0 + rb + 16 * bb + lr] = acc[a][bb][reg];
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

// One step of the blocked back substitution L^T y = z, tile k (descending):
// y_k = W^T z_k (a 64x64 product, recomputed by every workgroup; workgroup 0
// stores it), then thread l of workgroup b updates z_j, j = 256b + l < k0:
//   z_j -= sum_r L(k0 + r, j) y_k[r]
// from its column's 64 contiguous doubles, prefetched first.
__global__ __launch_bounds__(256) void k_backsolve_step(const double* __restrict__ A, int ld, int n, int k,
                                                        const double* __restrict__ Winv, double* __restrict__ z,
                                                        double* __restrict__ y) {
  __shared__ double zk[NB];
  __shared__ double part[4][NB];
  __shared__ double yk[NB];
  const int k0 = k * NB;
  const int nreal = (n - k0) < NB ? (n - k0) : NB;
  const int t = threadIdx.x, r = t & 63, q = t >> 6;
  const int j = blockIdx.x * 256 + t;
  const bool upd = j < k0;
  double col[NB];
  if (upd) {
#pragma unroll
    for (int p = 0; p < NB / 2; ++p) {
      const double2 v2 = *reinterpret_cast<const double2*>(A + size_t(j) * ld + k0 + 2 * p);
      col[2 * p] = v2.x;
      col[2 * p + 1] = v2.y;
    }
  }
  // y_k[r] = sum_c W(c, r) z_k[c], W(c, r) = Wc[r][c]; quarter q sums c in [16q, 16q + 16)
  const double* Wr = Winv + size_t(k) * NB * NB + size_t(r) * NB + 16 * q;
  double wv[16];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const double2 v2 = *reinterpret_cast<const double2*>(Wr + 2 * p);
    wv[2 * p] = v2.x;
    wv[2 * p + 1] = v2.y;
  }
  if (t < NB) zk[t] = (t < nreal) ? z[k0 + t] : 0.0;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int p = 0; p < 16; ++p) s = fma(wv[p], zk[16 * q + p], s);
  part[q][r] = s;
  __syncthreads();
  if (t < NB) {
    const double v = (t < nreal) ? (part[0][t] + part[1][t]) + (part[2][t] + part[3][t]) : 0.0;
    yk[t] = v;
    if (blockIdx.x == 0 && t < nreal) y[k0 + t] = v;
  }
  __syncthreads();
  if (upd) {
    double acc = 0.0;
#pragma unroll
    for (int rr = 0; rr < NB; ++rr) acc = fma(col[rr], yk[rr], acc);
    z[j] -= acc;
  }
}

}  // namespace

void launch_cholesky(const DevProblem& d, hipStream_t s) {
  (void)hipMemsetAsync(d.fail, 0, sizeof(int), s);
  for (int k = 0; k < d.nblk; ++k) {
    k_chol_potrf<<<1, 128, 0, s>>>(d.S, d.ld, k, d.n, d.invL, d.fail);
    const int m = d.nblk - k - 1;
    if (m == 0) break;
    k_chol_trsm<<<m, 256, 0, s>>>(d.S, d.ld, k, d.invL);
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
