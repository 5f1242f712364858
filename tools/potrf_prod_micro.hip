#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define NB 64
__device__ __forceinline__ double rsqrt_nr(double d) {
  double y = __builtin_amdgcn_rsq(d);
  y = y * fma(-0.5 * d * y, y, 1.5);
  y = y * fma(-0.5 * d * y, y, 1.5);
  return y;
}

// POTRF of one 64x64 tile.  Wavefront w holds rows 16w..16w+15; lane c holds
// column c: a[i] = A(16w + i, c).  Column j = 16 jw + ji is processed with
// ji unrolled (register indices are compile-time) inside a rolled loop over
// jw (keeps the body in the instruction cache):
//   1. the pivot lane (wave jw, lane j) forms 1/sqrt(a_jj) -> LDS
//   2. lane j of every wave scales its 16 rows of column j -> LDS column
//   3. every lane applies the rank-1 update to its 16 rows of column c > j
template <int V>
__global__ __launch_bounds__(256) void k_chol_potrf(double* __restrict__ A, int ld, int k, int n,
                                                    double* __restrict__ invd, int* __restrict__ fail, unsigned long long* st) {
  __shared__ double colb[NB];
  __shared__ double ids[NB];
  __shared__ double piv_s[2];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int k0 = k * NB;
  double a[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = A[size_t(k0 + lane) * ld + k0 + 16 * w + i];
  int bad = 0;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int jw = 0; jw < 4; ++jw) {
#pragma unroll
    for (int ji = 0; ji < 16; ++ji) {
      const int j = 16 * jw + ji;
      if (w == jw && lane == j) {
        const double d = a[ji];
        if (!(d > 0.0)) bad |= (k0 + j) < n;
        const double inv = rsqrt_nr(d);
        piv_s[0] = d * inv;
        piv_s[1] = inv;
        ids[j] = inv;
      }
      __syncthreads();
      if (V >= 2 && lane == j) {
        const double p = piv_s[0], inv = piv_s[1];
        if (V == 4) {
#pragma unroll
          for (int i = 0; i < 16; ++i) { const int r = 16 * w + i; a[i] = (r > j) ? a[i] * inv : ((r == j) ? p : 0.0); }
        } else if (V == 5) {
#pragma unroll
          for (int i = 0; i < 16; ++i) colb[16 * w + i] = a[i];
        } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int r = 16 * w + i;
          a[i] = (r > j) ? a[i] * inv : ((r == j) ? p : 0.0);
          colb[r] = a[i];
        }
        }
      }
      __syncthreads();
      const double lc = (lane > j) ? colb[lane] : 0.0;
      if (V >= 3 && 16 * w + 15 > j) {
#pragma unroll
        for (int i = 0; i < 16; ++i) a[i] = fma(-colb[16 * w + i], lc, a[i]);
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) st[0] = t1 - t0;
  if (bad) atomicOr(fail, 1);
  __syncthreads();
  if (t < NB) invd[k0 + t] = ids[t];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int r = 16 * w + i;
    if (r >= lane) A[size_t(k0 + lane) * ld + k0 + r] = a[i];
  }
}


int main() {
  const int ld = 64;
  std::vector<double> h(ld * ld, 0.0);
  for (int i = 0; i < 64; ++i) for (int j = 0; j <= i; ++j) h[j * ld + i] = (i == j) ? 100.0 : 0.5;
  double *A, *invd; unsigned long long* st; int* f;
  hipMalloc(&A, h.size() * 8); hipMalloc(&invd, 64 * 8); hipMalloc(&st, 16); hipMalloc(&f, 4);
  hipEvent_t a0, a1; hipEventCreate(&a0); hipEventCreate(&a1);
  for (int rep = 0; rep < 15; ++rep) {
    hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipEventRecord(a0);
    if (rep % 5 == 3) k_chol_potrf<4><<<1, 256>>>(A, ld, 0, 64, invd, f, st);
    if (rep % 5 == 4) k_chol_potrf<5><<<1, 256>>>(A, ld, 0, 64, invd, f, st);
    if (rep % 5 == 0) k_chol_potrf<1><<<1, 256>>>(A, ld, 0, 64, invd, f, st);
    if (rep % 5 == 1) k_chol_potrf<2><<<1, 256>>>(A, ld, 0, 64, invd, f, st);
    if (rep % 5 == 2) k_chol_potrf<3><<<1, 256>>>(A, ld, 0, 64, invd, f, st);
    hipEventRecord(a1); hipEventSynchronize(a1);
    float ms; hipEventElapsedTime(&ms, a0, a1);
    unsigned long long s; hipMemcpy(&s, st, 8, hipMemcpyDeviceToHost);
    printf("V%d potrf:", (rep % 5) + 1); printf(" event %.1f us, loop %llu cycles = %.0f cycles/column\n", ms * 1e3, s, s / 64.0);
  }
}
