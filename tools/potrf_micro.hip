// Diagnostic build (not product code): cycles per column step of the tile
// POTRF, stamped with s_memtime / s_memrealtime around the column loop.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cmath>
#define NB 64
__global__ __launch_bounds__(256) void potrf_stamped(double* A, int ld, double* invd, unsigned long long* stamps) {
  __shared__ double col[NB];
  __shared__ double piv_s[2];
  __shared__ double idl[NB];
  const int t = threadIdx.x, rb = t >> 4, cb = t & 15;
  double a[4][4];
  for (int x = 0; x < 4; ++x) for (int y = 0; y < 4; ++y) {
    const int r = 4 * rb + x, c = 4 * cb + y;
    a[x][y] = (r >= c) ? A[size_t(c) * ld + r] : 0.0;
  }
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (int j = 0; j < NB; ++j) {
    const int jb = j >> 2, jy = j & 3;
    if (rb == jb && cb == jb) {
      double d = 0.0;
      for (int x = 0; x < 4; ++x) if (x == jy) d = a[x][x];
      const double p = sqrt(d);
      piv_s[0] = p; piv_s[1] = 1.0 / p; idl[j] = 1.0 / p;
    }
    __syncthreads();
    if (cb == jb && rb >= jb) {
      const double p = piv_s[0], ip = piv_s[1];
      for (int x = 0; x < 4; ++x) {
        const int r = 4 * rb + x; double cv = 0.0;
        for (int y = 0; y < 4; ++y) {
          const double nv = (r > j) ? a[x][y] * ip : p;
          const bool sel = (y == jy) && (r >= j);
          a[x][y] = sel ? nv : a[x][y];
          cv = (y == jy) ? nv : cv;
        }
        col[r] = (r >= j) ? cv : 0.0;
      }
    }
    __syncthreads();
    if (cb <= rb && 4 * cb + 3 > j) {
      double lr[4], lc[4];
      for (int x = 0; x < 4; ++x) lr[x] = col[4 * rb + x];
      for (int y = 0; y < 4; ++y) lc[y] = col[4 * cb + y];
      for (int y = 0; y < 4; ++y) lc[y] = (4 * cb + y > j) ? lc[y] : 0.0;
      for (int x = 0; x < 4; ++x) for (int y = 0; y < 4; ++y) a[x][y] = fma(-lr[x], lc[y], a[x][y]);
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  if (t == 0) { stamps[0] = t1 - t0; stamps[1] = w1 - w0; }
  if (t < NB) invd[t] = idl[t];
  for (int x = 0; x < 4; ++x) for (int y = 0; y < 4; ++y) {
    const int r = 4 * rb + x, c = 4 * cb + y;
    if (r >= c) A[size_t(c) * ld + r] = a[x][y];
  }
}

__global__ __launch_bounds__(256) void trsm_stamped(double* A, int ld, const double* invd, unsigned long long* stamps) {
  __shared__ double Lt[NB][NB + 1];
  __shared__ double id[NB];
  const int t = threadIdx.x;
  for (int e = t; e < NB * NB; e += 256) { const int j = e >> 6, c = e & 63; Lt[j][c] = (c >= j) ? A[size_t(j) * ld + c] : 0.0; }
  if (t < NB) id[t] = invd[t];
  const int r = t >> 2, p = t & 3;
  double x[16];
  for (int m = 0; m < 16; ++m) x[m] = A[size_t(p + 4 * m) * ld + 64 + r];
  __syncthreads();
  const int lane = t & 63, base = lane & ~3;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int j = 0; j < NB; ++j) {
    const int jm = j >> 2, jp = j & 3;
    const double s = id[j];
    double v = 0.0;
#pragma unroll
    for (int m = 0; m < 16; ++m) { const bool own = (p == jp) && (m == jm); const double xs = x[m] * s; x[m] = own ? xs : x[m]; v = own ? xs : v; }
    const double xj = __shfl(v, base + jp);
    double l[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) l[m] = Lt[j][p + 4 * m];
#pragma unroll
    for (int m = 0; m < 16; ++m) { const double upd = fma(-xj, l[m], x[m]); x[m] = (p + 4 * m == j) ? x[m] : upd; }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) stamps[2] = t1 - t0;
  for (int m = 0; m < 16; ++m) A[size_t(p + 4 * m) * ld + 64 + r] = x[m];
}
__global__ void empty_kernel(int* p) { if (threadIdx.x == 0 && p) *p = 1; }
int main() {
  const int ld = 64;
  std::vector<double> h(ld * ld, 0.0);
  for (int i = 0; i < 64; ++i) for (int j = 0; j <= i; ++j) h[j * ld + i] = (i == j) ? 100.0 : 0.5;
  double *A, *invd; unsigned long long* st; int* e;
  hipMalloc(&A, h.size() * 8); hipMalloc(&invd, 64 * 8); hipMalloc(&st, 16); hipMalloc(&e, 4);
  hipEvent_t a0, a1; hipEventCreate(&a0); hipEventCreate(&a1);
  for (int rep = 0; rep < 5; ++rep) {
    hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipEventRecord(a0);
    potrf_stamped<<<1, 256>>>(A, ld, invd, st);
    hipEventRecord(a1); hipEventSynchronize(a1);
    float ms; hipEventElapsedTime(&ms, a0, a1);
    unsigned long long s[2]; hipMemcpy(s, st, 16, hipMemcpyDeviceToHost);
    printf("potrf: event %.1f us, loop %llu cycles, %llu ticks@100MHz (%.1f us) -> clock %.2f GHz, %.0f cycles/column\n",
           ms * 1e3, s[0], s[1], s[1] / 100.0, s[0] / (s[1] / 100.0) / 1e3, s[0] / 64.0);
  }
  {
    std::vector<double> h2(128 * 128, 0.0);
    for (int i = 0; i < 128; ++i) for (int j = 0; j <= i; ++j) h2[j * 128 + i] = (i == j) ? 100.0 : 0.5;
    double* A2; hipMalloc(&A2, h2.size() * 8); hipMemcpy(A2, h2.data(), h2.size() * 8, hipMemcpyHostToDevice);
    potrf_stamped<<<1, 256>>>(A2, 128, invd, st);
    for (int rep = 0; rep < 4; ++rep) {
      hipEventRecord(a0);
      trsm_stamped<<<1, 256>>>(A2, 128, invd, st);
      hipEventRecord(a1); hipEventSynchronize(a1);
      float ms; hipEventElapsedTime(&ms, a0, a1);
      unsigned long long s[3]; hipMemcpy(s, st, 24, hipMemcpyDeviceToHost);
      printf("trsm: event %.1f us, loop %llu cycles, %.0f cycles/column\n", ms * 1e3, s[2], s[2] / 64.0);
    }
  }
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(a0);
    for (int i = 0; i < 100; ++i) empty_kernel<<<1, 64>>>(e);
    hipEventRecord(a1); hipEventSynchronize(a1);
    float ms; hipEventElapsedTime(&ms, a0, a1);
    printf("100 empty dependent kernels: %.1f us each\n", ms * 10);
  }
  return 0;
}
