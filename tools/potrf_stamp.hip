#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
#define NB 64
typedef double f64x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ double rsqrt_nr(double d) {
  double y = __builtin_amdgcn_rsq(d);
  y = y * fma(-0.5 * d * y, y, 1.5);
  y = y * fma(-0.5 * d * y, y, 1.5);
  return y;
}
__device__ __forceinline__ double bcast(double v, int src) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
  return __hiloint2double(hi, lo);
}
constexpr int kPotrfBlk = 8;
template <bool kFull>  // kFull: every pivot of the tile is a real one (k0 + 64 <= n)
__global__ __launch_bounds__(128) void k_chol_potrf(double* __restrict__ A, int ld, int k, int n,
                                                    double* __restrict__ Winv, int* __restrict__ fail, long long* st) {
  long long ts[NB + 3];
  ts[0] = __builtin_amdgcn_s_memtime();
  __shared__ __attribute__((aligned(16))) double Lcol[NB * NB];  // Lcol[j][c] = L(c, j)
  __shared__ double invs[NB];
  const int r = threadIdx.x & 63;
  const int k0 = k * NB;
  if (threadIdx.x < 64) {
    // Only the lower part (j <= r) is ever read back: the strict upper
    // entries of a row never feed a pivot or an L value, so they are not
    // loaded (all loads coalesced) and their updates are don't-cares.
    double a[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const double v = A[size_t(k0 + j) * ld + k0 + r];  // unconditional: no exec-mask blocks
      a[j] = (j <= r) ? v : 0.0;
    }
    bool bad = false;
    double d = bcast(a[0], 0);
    ts[1] = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (kFull || (k0 + j) < n) bad |= !(d > 0.0);
      if (!kFull && (k0 + j) >= n) d = 1.0;
      const double inv = rsqrt_nr(d);
      const double l = a[j] * inv;  // L(r, j) for r >= j (r == j: sqrt(d))
      a[j] = l;
      Lcol[j * NB + r] = l;
      invs[j] = inv;
      if (j < NB - 1) {
        // the next pivot is lane j+1's own a[j+1] - L(j+1, j)^2: one
        // readlane, no LDS on the pivot chain
        d = bcast(fma(-l, l, a[j + 1]), j + 1);
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
      ts[2 + j] = __builtin_amdgcn_s_memtime();
      if (j % kPotrfBlk == kPotrfBlk - 1) __syncthreads();
    }
    if (bad && r == 0) atomicOr(fail, 1);
#pragma unroll
    for (int j = 0; j < NB; ++j) A[size_t(k0 + j) * ld + k0 + r] = a[j];  // strict upper: don't-care
    ts[NB + 2] = __builtin_amdgcn_s_memtime();
    if (r == 0) for (int q = 0; q < NB + 3; ++q) st[q] = ts[q];
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


int main() {
  const int n = 64, ld = 64;
  std::vector<double> M(n * n), A(n * n);
  unsigned s = 1;
  for (auto& v : M) { s = s * 1664525u + 1013904223u; v = (s >> 8) / 16777216.0 - 0.5; }
  for (int i = 0; i < n; ++i) for (int j = 0; j < n; ++j) {
    double acc = (i == j) ? n : 0.0;
    for (int q = 0; q < n; ++q) acc += M[i * n + q] * M[j * n + q];
    A[j * ld + i] = acc;
  }
  double *dA, *dW; int* df; long long* dst;
  hipMalloc(&dA, 8 * n * n); hipMalloc(&dW, 8 * n * n); hipMalloc(&df, 4); hipMalloc(&dst, 8 * 128);
  for (int rep = 0; rep < 3; ++rep) {
    hipMemcpy(dA, A.data(), 8 * n * n, hipMemcpyHostToDevice);
    k_chol_potrf<true><<<1, 128>>>(dA, ld, 0, 1000, dW, df, dst);
    hipDeviceSynchronize();
  }
  std::vector<long long> st(NB + 3);
  hipMemcpy(st.data(), dst, 8 * (NB + 3), hipMemcpyDeviceToHost);
  printf("load %lld  cols:", st[1] - st[0]);
  for (int j = 0; j < NB; ++j) printf(" %lld", st[2 + j] - (j ? st[1 + j] : st[1]));
  printf("\nstore %lld total %lld\n", st[NB + 2] - st[NB + 1], st[NB + 2] - st[0]);
  // verify L L^T = A on the lower triangle
  std::vector<double> L(n * n);
  hipMemcpy(L.data(), dA, 8 * n * n, hipMemcpyDeviceToHost);
  double err = 0;
  for (int i = 0; i < n; ++i) for (int j = 0; j <= i; ++j) {
    double acc = 0; for (int q = 0; q <= j; ++q) acc += L[q * ld + i] * L[q * ld + j];
    err = fmax(err, fabs(acc - A[j * ld + i]));
  }
  printf("err %.3e\n", err);
}
