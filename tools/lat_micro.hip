// Diagnostic microbenchmark (not product code): latencies of the primitives
// on the Cholesky pivot chain, in shader clocks (s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(256) void lat(double* out, unsigned long long* st, double seed) {
  __shared__ double sh[256];
  const int t = threadIdx.x;
  double x = seed + t;
  unsigned long long t0, t1;
  // 1. dependent f64 FMA chain
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < 100; ++i) x = fma(x, 0.999999, 1e-9);
  asm volatile("s_waitcnt vmcnt(0)" :: "v"(x));
  t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) st[0] = t1 - t0;
  // 2. dependent rsq chain
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < 100; ++i) x = __builtin_amdgcn_rsq(x) + 0.5;
  asm volatile("" :: "v"(x));
  t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) st[1] = t1 - t0;
  // 3. barrier only (4 waves)
  __syncthreads();
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 100; ++i) __syncthreads();
  t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) st[2] = t1 - t0;
  // 4. LDS write -> barrier -> read of another wave's value, dependent
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 100; ++i) {
    sh[t] = x;
    __syncthreads();
    x = sh[(t + 64) & 255] * 0.5 + 1.0;
    __syncthreads();
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) st[3] = t1 - t0;
  // 5. dependent ds_bpermute (shfl) chain
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 100; ++i) x = __shfl(x, (t + 1) & 63) + 1.0;
  asm volatile("" :: "v"(x));
  t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) st[4] = t1 - t0;
  // 6. dependent readfirstlane-style broadcast (v_readlane to SGPR) chain
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 100; ++i) {
    const unsigned lo = __builtin_amdgcn_readlane(__double2loint(x), 5);
    const unsigned hi = __builtin_amdgcn_readlane(__double2hiint(x), 5);
    x = __hiloint2double(hi, lo) * 0.5 + 1.0;
  }
  asm volatile("" :: "v"(x));
  t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) st[5] = t1 - t0;
  out[t] = x;
}
int main() {
  double* o; unsigned long long* st; hipMalloc(&o, 256 * 8); hipMalloc(&st, 64);
  const char* names[] = {"fma_f64 dependent", "rsq_f64+add dependent", "s_barrier (4 waves)", "LDS wr->bar->rd->bar", "ds_bpermute dependent", "readlane x2 dependent"};
  for (int r = 0; r < 3; ++r) {
    lat<<<1, 256>>>(o, st, 1.0 + r);
    unsigned long long h[6]; hipMemcpy(h, st, 48, hipMemcpyDeviceToHost);
    for (int i = 0; i < 6; ++i) printf("%-26s %7.1f cycles/iter\n", names[i], h[i] / 100.0);
    printf("--\n");
  }
  return 0;
}
