// Cold-cache HBM probe: each timed pass runs right after a 512-MB read of an
// unrelated buffer (MALL/L2 hold none of the pass's lines), as a kernel meets
// memory inside an LM iteration; back-to-back (warm) passes beside it.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d2v __attribute__((ext_vector_type(2)));
__global__ void k_write(d2v* __restrict__ p, size_t n, int nt) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    d2v v = {double(i), 1.0};
    if (nt) __builtin_nontemporal_store(v, p + i); else p[i] = v;
  }
}
__global__ void k_read(const d2v* __restrict__ p, size_t n, double* out) {
  double s = 0;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    d2v v = p[i];
    s += v.x + v.y;
  }
  if (s == 12345.678) out[0] = s;
}
int main() {
  const size_t bytes = 320ull << 20, n = bytes / 16, tb = 512ull << 20;
  d2v *a, *b, *t; double* o;
  hipMalloc(&a, bytes); hipMalloc(&b, bytes); hipMalloc(&t, tb); hipMalloc(&o, 8);
  hipMemset(a, 0, bytes); hipMemset(t, 0, tb);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int cold : {0, 1})
    for (int v = 0; v < 3; ++v) {
      float sum = 0.f, ms;
      const int reps = 8;
      for (int r = 0; r < reps + 1; ++r) {
        if (cold) k_read<<<4096, 256>>>(t, tb / 16, o);
        hipEventRecord(e0);
        if (v < 2) k_write<<<4096, 256>>>(a, n, v);
        else k_read<<<4096, 256>>>(a, n, o);
        hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
        if (r) sum += ms;
      }
      const double us = sum / reps * 1e3;
      printf("%-5s %-9s %8.1f us %8.1f GB/s\n", cold ? "cold" : "warm", v == 0 ? "write" : v == 1 ? "write_nt" : "read",
             us, bytes / (us * 1e-6) / 1e9);
    }
  return 0;
}
