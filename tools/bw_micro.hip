// HBM bandwidth probe: streaming write / read / copy of 320 MB with 16-B lanes.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k_write(double2* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
    p[i] = make_double2(double(i), 1.0);
}
__global__ void k_write_nt(double2* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
    {
      typedef double d2v __attribute__((ext_vector_type(2)));
      d2v v = {double(i), 1.0};
      __builtin_nontemporal_store(v, reinterpret_cast<d2v*>(p) + i);
    }
}
__global__ void k_read(const double2* __restrict__ p, size_t n, double* out) {
  double s = 0;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    double2 v = p[i];
    s += v.x + v.y;
  }
  if (s == 12345.678) out[0] = s;
}
__global__ void k_copy(const double2* __restrict__ a, double2* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) b[i] = a[i];
}
int main1() {
  const size_t bytes = 320ull << 20, n = bytes / 16;
  double2 *a, *b; double* o;
  hipMalloc(&a, bytes); hipMalloc(&b, bytes); hipMalloc(&o, 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int grid : {1024, 2048, 4096, 8192}) {
    float ms;
    for (int v = 0; v < 4; ++v) {
      float best = 1e9;
      for (int r = 0; r < 5; ++r) {
        hipEventRecord(e0);
        if (v == 0) k_write<<<grid, 256>>>(a, n);
        if (v == 1) k_write_nt<<<grid, 256>>>(a, n);
        if (v == 2) k_read<<<grid, 256>>>(a, n, o);
        if (v == 3) k_copy<<<grid, 256>>>(a, b, n);
        hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      const double gb = (v == 3 ? 2.0 : 1.0) * bytes / 1e9;
      printf("grid %5d %-9s %8.1f GB/s\n", grid, v == 0 ? "write" : v == 1 ? "write_nt" : v == 2 ? "read" : "copy", gb / (best * 1e-3));
    }
  }
}
// (appended) write 10-KB runs: one wave per run, run order sequential or permuted
__global__ void k_runs(double2* __restrict__ p, int nruns, int stride_perm, int per_wave) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, l = threadIdx.x & 63;
  const int nw = (gridDim.x * blockDim.x) >> 6;
  for (int r = wave; r < nruns; r += nw) {
    const int run = stride_perm ? int((long long)r * stride_perm % nruns) : r;
    double2* d = p + size_t(run) * 640;
    for (int k = 0; k < 10; ++k) d[64 * k + l] = make_double2(double(r), double(k));
  }
}
int main2() {
  const int nruns = 31250;
  double2* a; hipMalloc(&a, size_t(nruns) * 10240);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int perm : {0, 7919, 12345}) for (int grid : {1024, 4096}) {
    float best = 1e9, ms;
    for (int r = 0; r < 5; ++r) {
      hipEventRecord(e0); k_runs<<<grid, 256>>>(a, nruns, perm, 0); hipEventRecord(e1);
      hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
    }
    printf("runs perm %5d grid %5d  %.1f us  %.1f GB/s\n", perm, grid, best * 1e3, nruns * 10240.0 / (best * 1e-3) / 1e9);
  }
  return 0;
}
int main() { main2(); return 0; }
