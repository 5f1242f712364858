// HBM reference measurement for bench.py: a STREAM copy (read + write bytes
// per second) with 16-B vector accesses, the form MI355X_MICROARCH.md quotes
// its measured 6.29 TB/s for.  It is the denominator beside the 8 TB/s spec
// for the "fraction of achievable HBM" statements of DESIGN.md; nothing on the
// BA path calls it.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <string>
#include "../../include/sfm_amd.h"

void sfm_internal_set_error(const std::string& msg);

namespace {

typedef float v4f __attribute__((ext_vector_type(4)));  // one 16-B access

// Each thread moves kU 16-B elements per round, all loads issued before the
// stores; consecutive lanes take consecutive 16-B elements (fully coalesced
// 1-KiB wave accesses).
template <int kU, bool kNT>
__global__ __launch_bounds__(256) void k_stream_copy(const v4f* __restrict__ a, v4f* __restrict__ b, int64_t n) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x * kU;
  for (int64_t base = int64_t(blockIdx.x) * blockDim.x * kU + threadIdx.x; base < n; base += stride) {
    v4f v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = base + int64_t(u) * blockDim.x;
      if (i < n) v[u] = kNT ? __builtin_nontemporal_load(a + i) : a[i];
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = base + int64_t(u) * blockDim.x;
      if (i < n) {
        if (kNT) __builtin_nontemporal_store(v[u], b + i);
        else b[i] = v[u];
      }
    }
  }
}

}  // namespace

extern "C" int sfm_bench_stream_copy(int32_t device, int64_t bytes, int32_t reps, double* best_gbs) {
  if (bytes < (1 << 20) || reps < 1 || !best_gbs) {
    sfm_internal_set_error("sfm_bench_stream_copy: bytes >= 1 MiB, reps >= 1");
    return SFM_EINVAL;
  }
  if (hipSetDevice(device) != hipSuccess) {
    sfm_internal_set_error("sfm_bench_stream_copy: hipSetDevice failed");
    return SFM_ENODEV;
  }
  hipDeviceProp_t prop;
  int cus = 256;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0) cus = prop.multiProcessorCount;
  const int64_t n = bytes / 16;
  v4f *a = nullptr, *b = nullptr;
  if (hipMalloc(&a, n * 16) != hipSuccess || hipMalloc(&b, n * 16) != hipSuccess) {
    if (a) (void)hipFree(a);
    sfm_internal_set_error("sfm_bench_stream_copy: hipMalloc failed");
    return SFM_ENOMEM;
  }
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  (void)hipMemsetAsync(a, 0, n * 16, s);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  double best = 0.0;
  // a few grid / unroll shapes, best of `reps` each (the figure is the best
  // copy the device sustains, not a property of one launch shape)
  const int grids[4] = {cus * 2, cus * 4, cus * 8, cus * 16};
  for (int g : grids)
    for (int u = 0; u < 4; ++u)
      for (int r = 0; r <= reps; ++r) {
        (void)hipEventRecord(e0, s);
        if (u == 0) k_stream_copy<4, true><<<g, 256, 0, s>>>(a, b, n);
        else if (u == 1) k_stream_copy<8, true><<<g, 256, 0, s>>>(a, b, n);
        else if (u == 2) k_stream_copy<4, false><<<g, 256, 0, s>>>(a, b, n);
        else k_stream_copy<8, false><<<g, 256, 0, s>>>(a, b, n);
        (void)hipEventRecord(e1, s);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r > 0 && ms > 0.f) best = std::max(best, 2.0 * double(n) * 16.0 / (double(ms) * 1e-3) / 1e9);
      }
  const hipError_t err = hipStreamSynchronize(s);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipStreamDestroy(s);
  (void)hipFree(a);
  (void)hipFree(b);
  if (err != hipSuccess) {
    sfm_internal_set_error(std::string("sfm_bench_stream_copy: ") + hipGetErrorString(err));
    return SFM_EIO;
  }
  *best_gbs = best;
  return 0;
}
