// FETCH_SIZE / WRITE_SIZE calibration on known byte counts, in the access
// widths the BA kernels use (MI355X_MICROARCH.md "HBM": only wide streamed
// reads and 16-B streamed stores are calibrated there).  Every kernel touches
// each byte of its range once, over a 1 GiB table (past the 256 MiB Infinity
// Cache), so the algorithmic byte count is the HBM byte count.
//   hipcc --offload-arch=gfx950 -O3 tools/pmc_calib.hip -o tools/pmc_calib
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace... see tools/pmc_calib.sh
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// streamed 16 B per lane
__global__ void cal_read16(const double2* __restrict__ a, size_t n, double* out) {
  double s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    double2 v = a[i]; s += v.x + v.y;
  }
  if (s == 1.2345) out[0] = s;
}
// streamed 8 B per lane
__global__ void cal_read8(const double* __restrict__ a, size_t n, double* out) {
  double s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
  if (s == 1.2345) out[0] = s;
}
// random 128-B records, 8 lanes x 16 B per record (k_schur_pts / k_obs_prep shape)
__global__ void cal_gather128(const double2* __restrict__ a, const uint32_t* __restrict__ idx, size_t nrec, double* out) {
  double s = 0;
  size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (size_t i = t; i < nrec * 8; i += (size_t)gridDim.x * blockDim.x) {
    double2 v = a[(size_t)idx[i >> 3] * 8 + (i & 7)]; s += v.x + v.y;
  }
  if (s == 1.2345) out[0] = s;
}
// random 128-B records, one lane reads a whole record as 8 x 16 B
__global__ void cal_gather128_lane(const double2* __restrict__ a, const uint32_t* __restrict__ idx, size_t nrec, double* out) {
  double s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nrec; i += (size_t)gridDim.x * blockDim.x) {
    const double2* r = a + (size_t)idx[i] * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) { double2 v = r[k]; s += v.x + v.y; }
  }
  if (s == 1.2345) out[0] = s;
}
// random 64-B lines, one 8-B double per lane from each (sparse gather: 8 of 64 B used)
__global__ void cal_gather8(const double* __restrict__ a, const uint32_t* __restrict__ idx, size_t n, double* out) {
  double s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[(size_t)idx[i] * 8];
  if (s == 1.2345) out[0] = s;
}
// streamed 16 B stores
__global__ void cal_write16(double2* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = make_double2(i, 1.0);
}
// streamed 8 B stores
__global__ void cal_write8(double* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = (double)i;
}
// random 128-B record stores, 8 lanes x 16 B
__global__ void cal_scatter128(double2* __restrict__ a, const uint32_t* __restrict__ idx, size_t nrec) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nrec * 8; i += (size_t)gridDim.x * blockDim.x)
    a[(size_t)idx[i >> 3] * 8 + (i & 7)] = make_double2(i, 2.0);
}

int main() {
  const size_t bytes = size_t(1) << 30;          // 1 GiB table
  const size_t nrec = bytes / 128;               // 8 Mi records of 128 B
  double2* a; double* out; uint32_t* idx;
  CK(hipMalloc(&a, bytes)); CK(hipMalloc(&out, 64)); CK(hipMalloc(&idx, nrec * 4));
  CK(hipMemset(a, 0, bytes));
  std::vector<uint32_t> h(nrec);
  for (size_t i = 0; i < nrec; ++i) h[i] = (uint32_t)i;
  std::mt19937 rng(7); std::shuffle(h.begin(), h.end(), rng);
  CK(hipMemcpy(idx, h.data(), nrec * 4, hipMemcpyHostToDevice));
  const int G = 4096, B = 256;
  for (int rep = 0; rep < 3; ++rep) {
    cal_read16<<<G, B>>>(a, bytes / 16, out);
    cal_read8<<<G, B>>>((const double*)a, bytes / 8, out);
    cal_gather128<<<G, B>>>(a, idx, nrec, out);
    cal_gather128_lane<<<G, B>>>(a, idx, nrec, out);
    cal_gather8<<<G, B>>>((const double*)a, idx, nrec, out);
    cal_write16<<<G, B>>>(a, bytes / 16);
    cal_write8<<<G, B>>>((double*)a, bytes / 8);
    cal_scatter128<<<G, B>>>(a, idx, nrec);
  }
  CK(hipDeviceSynchronize());
  // algorithmic bytes per launch (the index array adds 32 MiB read to the gathers)
  printf("known bytes: read16/read8/gather128/gather128_lane = %zu (+%zu idx on gathers), gather8 = %zu lines x 64 B = %zu B used 8 B/line (+idx), "
         "write16/write8/scatter128 = %zu\n", bytes, nrec * 4, nrec, nrec * 64, bytes);
  CK(hipFree(a)); CK(hipFree(out)); CK(hipFree(idx));
  return 0;
}
