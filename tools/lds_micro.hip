// Diagnostic microbenchmark (not product code): cost of single-lane LDS
// stores between barriers.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int V>
__global__ __launch_bounds__(256) void k(double* out, unsigned long long* st) {
  __shared__ __attribute__((aligned(16))) double colb[256 * 16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  double a[16];
  for (int i = 0; i < 16; ++i) a[i] = out[t * 16 + i];
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int jw = 0; jw < 4; ++jw) {
#pragma unroll
    for (int ji = 0; ji < 16; ++ji) {
      const int j = 16 * jw + ji;
      __syncthreads();
      if (V == 1 && lane == j) { for (int i = 0; i < 16; ++i) colb[16 * w + i] = a[i]; }
      if (V == 2) { for (int i = 0; i < 16; ++i) colb[16 * t + i] = a[i]; }
      if (V == 3 && lane == 0) { for (int i = 0; i < 16; ++i) colb[16 * w + i] = a[i]; }
      if (V == 4 && lane == j) { a[0] += 1.0; }
      __syncthreads();
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) st[V] = t1 - t0;
  for (int i = 0; i < 16; ++i) out[t * 16 + i] = a[i] + colb[t];
}
int main() {
  double* o; unsigned long long* st; hipMalloc(&o, 256 * 16 * 8); hipMalloc(&st, 64); hipMemset(o, 0, 256*16*8);
  for (int r = 0; r < 2; ++r) {
    k<0><<<1, 256>>>(o, st); k<1><<<1, 256>>>(o, st); k<2><<<1, 256>>>(o, st); k<3><<<1, 256>>>(o, st); k<4><<<1, 256>>>(o, st);
    unsigned long long h[5]; hipMemcpy(h, st, 40, hipMemcpyDeviceToHost);
    printf("2 barriers only: %.0f | lane==j 16 stores: %.0f | all lanes 16 stores: %.0f | lane0 16 stores: %.0f | lane==j add: %.0f  (cycles/iter)\n",
           h[0] / 64.0, h[1] / 64.0, h[2] / 64.0, h[3] / 64.0, h[4] / 64.0);
  }
}
