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
// Right-looking blocked algorithm, tile 64:
//   k_chol_diag  : factor the diagonal tile and invert it (one workgroup)
//   k_chol_gemm  : TRSM of the panel as a GEMM with inv(L_kk)^T and the
//                  SYRK/GEMM trailing update, on v_mfma_f64_16x16x4_f64
// and the back substitution L^T y = z with the stored tile inverses.
#include <hip/hip_runtime.h>
#include <cmath>
#include "ba_device.h"

namespace sfm {
namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int NB = kNB;        // 64
constexpr int kPad = 80;       // LDS row stride (doubles): rows 2 apart land 32 banks apart

// Factor the 64x64 diagonal tile k (in place) and write its inverse.
// Left-looking by column; 4 lanes per row share each dot product.
__global__ __launch_bounds__(256) void k_chol_diag(double* __restrict__ A, int ld, int k, int n,
                                                   double* __restrict__ invL, int* __restrict__ fail) {
  __shared__ double L[NB][NB + 1];
  __shared__ double Xs[NB][NB + 1];
  const int k0 = k * NB;
  const int tid = threadIdx.x;
  for (int e = tid; e < NB * NB; e += 256) {
    const int j = e / NB, i = e - j * NB;
    L[i][j] = (i >= j) ? A[size_t(k0 + j) * ld + k0 + i] : 0.0;
    Xs[i][j] = 0.0;
  }
  __syncthreads();
  const int rsub = tid >> 2, part = tid & 3;
  for (int j = 0; j < NB; ++j) {
    const int i = j + rsub;
    double s = 0.0;
    if (i < NB)
      for (int kk = part; kk < j; kk += 4) s += L[i][kk] * L[j][kk];
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    const double v = (i < NB) ? L[i][j] - s : 0.0;
    if (part == 0 && i == j) {
      if (!(v > 0.0) && (k0 + j) < n) atomicOr(fail, 1);
      L[j][j] = sqrt(v);
    }
    __syncthreads();
    if (part == 0 && i > j && i < NB) L[i][j] = v / L[j][j];
    __syncthreads();
  }
  // inverse of the lower-triangular tile: column c by forward substitution
  const int c = tid >> 2;
  for (int i = 0; i < NB; ++i) {
    if (i >= c) {
      double s = 0.0;
      for (int kk = c + part; kk < i; kk += 4) s += L[i][kk] * Xs[kk][c];
      s += __shfl_xor(s, 1);
      s += __shfl_xor(s, 2);
      if (part == 0) Xs[i][c] = ((i == c ? 1.0 : 0.0) - s) / L[i][i];
    }
    __syncthreads();
  }
  for (int e = tid; e < NB * NB; e += 256) {
    const int j = e / NB, i = e - j * NB;
    if (i >= j) A[size_t(k0 + j) * ld + k0 + i] = L[i][j];
    invL[size_t(k) * NB * NB + size_t(j) * NB + i] = Xs[i][j];
  }
}

// C-tile GEMM on f64 MFMA:  D[c][r] = sum_l Xt[c][l] * Yt[r][l]  (64x64x64)
//   mode 0 (TRSM):  tile (i, k) <- A_ik * inv(L_kk)^T : X = invL_k, Y = A_ik
//   mode 1 (SYRK):  tile (i, j) -= L_ik * L_jk^T      : X = L_jk,  Y = L_ik
// Output element (r, c) of tile (ti, tj) lives at A[(tj*64 + c)*ld + ti*64 + r].
// v_mfma_f64_16x16x4_f64 lane maps (cdna_hip_programming.md §3): A[i=l&15][k=l>>4],
// B[k=l>>4][j=l&15], D col = l&15, row = (l>>4) + 4*reg.
__global__ __launch_bounds__(256) void k_chol_gemm(double* __restrict__ A, int ld, int k, int nblk, int mode,
                                                   const double* __restrict__ invL) {
  __shared__ double TX[NB * kPad];  // [l][c]
  __shared__ double TY[NB * kPad];  // [l][r]
  int ti, tj;
  const int b = blockIdx.x;
  if (mode == 0) {
    ti = k + 1 + b; tj = k;
  } else {
    // lower-triangular enumeration of the trailing tiles: b -> (i, j), j <= i
    int i = int((sqrt(8.0 * b + 1.0) - 1.0) * 0.5);
    while ((i + 1) * (i + 2) / 2 <= b) ++i;
    while (i * (i + 1) / 2 > b) --i;
    const int j = b - i * (i + 1) / 2;
    ti = k + 1 + i; tj = k + 1 + j;
  }
  const int k0 = k * NB, i0 = ti * NB, j0 = tj * NB;
  const int tid = threadIdx.x;
  for (int e = tid; e < NB * NB; e += 256) {
    const int l = e / NB, r = e - l * NB;
    // column l of the panel (global column k0 + l), rows r
    TY[l * kPad + r] = A[size_t(k0 + l) * ld + i0 + r];
    if (mode == 0) TX[l * kPad + r] = invL[size_t(k) * NB * NB + size_t(l) * NB + r];  // invL[c=r][l] col-major: (row r? see below)
    else TX[l * kPad + r] = A[size_t(k0 + l) * ld + j0 + r];
  }
  __syncthreads();
  const int lane = tid & 63, w = tid >> 6;
  const int cb = 32 * (w >> 1), rb = 32 * (w & 1);
  f64x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) acc[a][bb] = f64x4{0.0, 0.0, 0.0, 0.0};
  const int lr = lane & 15, lk = lane >> 4;
#pragma unroll 4
  for (int ks = 0; ks < NB / 4; ++ks) {
    const int l = ks * 4 + lk;
    double xa[2], yb[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) xa[a] = TX[l * kPad + cb + 16 * a + lr];
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) yb[bb] = TY[l * kPad + rb + 16 * bb + lr];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int bb = 0; bb < 2; ++bb) acc[a][bb] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[a], yb[bb], acc[a][bb], 0, 0, 0);
  }
  if (mode == 0) __syncthreads();  // in-place TRSM: every wave has finished reading before anyone writes (reads are LDS)
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int bb = 0; bb < 2; ++bb)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int c = cb + 16 * a + lk + 4 * reg;
        const int r = rb + 16 * bb + lr;
        double* dst = A + size_t(j0 + c) * ld + i0 + r;
        if (mode == 0) *dst = acc[a][bb][reg];
        else *dst -= acc[a][bb][reg];
      }
}

// z <- row n of the factor (z = L^-1 rhs), y <- 0
__global__ void k_copy_z(const double* __restrict__ A, int ld, int n, double* __restrict__ z, double* __restrict__ y) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < ld) {
    z[j] = (j < n) ? A[size_t(j) * ld + n] : 0.0;
    y[j] = 0.0;
  }
}

// One step of the blocked back substitution L^T y = z, block k (descending):
// every workgroup forms y_k = inv(L_kk)^T z_k (rows < n only); workgroup 0
// stores it; then each workgroup subtracts the block's contribution from 64
// earlier unknowns:  z_j -= sum_r L[k0 + r][j] y_k[r]   for j < k0.
__global__ __launch_bounds__(256) void k_backsolve_step(const double* __restrict__ A, int ld, int n, int k,
                                                        const double* __restrict__ invL, double* __restrict__ z,
                                                        double* __restrict__ y) {
  __shared__ double yk[NB];
  const int k0 = k * NB;
  const int nreal = (n - k0) < NB ? (n - k0) : NB;
  const int tid = threadIdx.x;
  {
    const int c = tid >> 2, part = tid & 3;
    const double* col = invL + size_t(k) * NB * NB + size_t(c) * NB;  // column c of inv(L_kk)
    double s = 0.0;
    if (c < nreal)
      for (int r = c + part; r < nreal; r += 4) s += col[r] * z[k0 + r];
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    if (part == 0) yk[c] = (c < nreal) ? s : 0.0;
  }
  __syncthreads();
  if (blockIdx.x == 0 && tid < nreal) y[k0 + tid] = yk[tid];
  const int lane = tid & 63, w = tid >> 6;
  const int jbase = blockIdx.x * NB;
  for (int jj = w; jj < NB; jj += 4) {
    const int j = jbase + jj;
    if (j >= k0) break;
    double v = (lane < nreal) ? A[size_t(j) * ld + k0 + lane] * yk[lane] : 0.0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) z[j] -= v;
  }
}

}  // namespace

void launch_cholesky(const DevProblem& d, hipStream_t s) {
  hipMemsetAsync(d.fail, 0, sizeof(int), s);
  for (int k = 0; k < d.nblk; ++k) {
    k_chol_diag<<<1, 256, 0, s>>>(d.S, d.ld, k, d.n, d.invL, d.fail);
    const int m = d.nblk - k - 1;
    if (m == 0) break;
    k_chol_gemm<<<m, 256, 0, s>>>(d.S, d.ld, k, d.nblk, 0, d.invL);
    k_chol_gemm<<<m * (m + 1) / 2, 256, 0, s>>>(d.S, d.ld, k, d.nblk, 1, d.invL);
  }
}

void launch_backsolve(const DevProblem& d, hipStream_t s) {
  k_copy_z<<<(d.ld + 255) / 256, 256, 0, s>>>(d.S, d.ld, d.n, d.zwork, d.ysol);
  const int nb_real = (d.n + NB - 1) / NB;
  for (int k = nb_real - 1; k >= 0; --k) {
    const int grid = k == 0 ? 1 : k;  // k*64 earlier unknowns, 64 per workgroup
    k_backsolve_step<<<grid, 256, 0, s>>>(d.S, d.ld, d.n, k, d.invL, d.zwork, d.ysol);
  }
}

}  // namespace sfm
