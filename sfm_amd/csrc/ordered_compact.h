// Order-preserving compaction of a sequential "first accepted query opens a
// slot, a better query overwrites the slot's query" resolution, shared by the
// descriptor matcher (CTracker.cpp:221-249) and the optical-flow association
// (CTracker.cpp:520-545).  Per train/detected index j the caller has
// reduced:
//   key[j]   64-bit key whose low word encodes the surviving query
//   first[j] the first accepted query (INT_MAX: none) -> slot order
// k_mark + k_compact then emit (query, j) pairs in slot order.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace sfm {
namespace {  // one copy per translation unit

// slot_train[i] = j + 1 if query i is the first accepted query of train j.
__global__ void k_mark_first(int n1, const int* __restrict__ first, int* __restrict__ slot_train) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n1 && first[j] != 0x7fffffff) slot_train[first[j]] = j + 1;
}

// Ordered compaction (single workgroup, prefix sum over the query order).
// kInvert: the key's low word holds 0xffffffff - query (latest query wins
// ties under atomicMin) instead of the query itself.
template <bool kInvert>
__global__ __launch_bounds__(1024) void k_compact_slots(int n0, const int* __restrict__ slot_train,
                                                        const unsigned long long* __restrict__ key,
                                                        int* __restrict__ idx0, int* __restrict__ idx1,
                                                        int* __restrict__ count) {
  __shared__ int sums[1024];
  __shared__ int base;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  for (int c0 = 0; c0 < n0; c0 += 1024) {
    const int i = c0 + threadIdx.x;
    const int f = (i < n0 && slot_train[i] > 0) ? 1 : 0;
    sums[threadIdx.x] = f;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const int v = threadIdx.x >= off ? sums[threadIdx.x - off] : 0;
      __syncthreads();
      sums[threadIdx.x] += v;
      __syncthreads();
    }
    if (f) {
      const int pos = base + sums[threadIdx.x] - 1;
      const int j = slot_train[i] - 1;
      const unsigned lo = unsigned(key[j] & 0xffffffffull);
      idx0[pos] = kInvert ? int(0xffffffffu - lo) : int(lo);
      idx1[pos] = j;
    }
    __syncthreads();
    if (threadIdx.x == 1023) base += sums[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) *count = base;
}

}  // namespace
}  // namespace sfm
