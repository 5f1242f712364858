// Microbenchmark + check of the walker's 64x64 tile POTRF (chol_kernels.hip
// potrf_tile: 16-column panels, lane-per-row pivot chain).  One workgroup,
// the tile in LDS as in k_chol_fused, `reps` POTRFs back to back on fresh
// copies, timed with s_memrealtime (100 MHz).  Output: us per POTRF, max
// |L - L_ref|, |W - W_ref| and a bitwise checksum of L and W (to compare
// builds of chol_kernels.hip).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/potrf_tile_micro.hip -o tools/potrf_tile_micro
// (CHOL_SRC=<path> selects another copy of the kernel file.)
#ifndef CHOL_SRC
#include "../sfm_amd/csrc/chol_kernels.hip"
#else
#include CHOL_SRC
#endif
#include <cstdint>
#include <cstring>

// Measured on MI355X (round 2): potrf_tile 9.8 us per tile; an 8-column
// variant with a redundant in-register diagonal factor ran 17.1 us.
namespace sfm {
namespace {
__global__ __launch_bounds__(256) void k_bench(const double* __restrict__ A, double* __restrict__ L,
                                               double* __restrict__ W, unsigned long long* st, int reps, int n) {
  __shared__ double T[NB * TS];
  __shared__ double Wl[NB * TS];
  __shared__ double scr[4][256];
  __shared__ int rdy;
  const int t = threadIdx.x;
  unsigned long long tot = 0;
  bool bad = false;
  for (int rep = 0; rep < reps; ++rep) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = t + 256 * q, c = e >> 6, r = e & 63;
      T[c * TS + r] = A[c * 64 + r];
    }
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bad |= potrf_tile<true>(T, Wl, scr, 0, n, nullptr, nullptr, nullptr, 0, &rdy);
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    tot += t1 - t0;
    __syncthreads();
  }
  if (t == 0) { st[0] = tot; st[1] = bad; }
#ifdef POTRF_STAMPS
  if (t < 4 * 32) st[2 + t] = g_st[t >> 5][t & 31];
#endif
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = t + 256 * q, c = e >> 6, r = e & 63;
    L[c * 64 + r] = T[c * TS + r];
    W[c * 64 + r] = Wl[c * TS + r];
  }
}
}  // namespace
}  // namespace sfm

int main() {
  const int n = 64, reps = 50;
  std::vector<double> A(n * n);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (s >> 8) / double(1 << 24) - 0.5; };
  std::vector<double> B(n * n);
  for (auto& v : B) v = rnd();
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double acc = 0;
      for (int k = 0; k < n; ++k) acc += B[i * n + k] * B[j * n + k];
      A[j * n + i] = acc + (i == j ? 4.0 : 0.0);  // column-major, SPD
    }
  // reference L (lower) and W = L^-1
  std::vector<double> Lr(n * n, 0.0), Wr(n * n, 0.0);
  for (int j = 0; j < n; ++j) {
    double d = A[j * n + j];
    for (int k = 0; k < j; ++k) d -= Lr[k * n + j] * Lr[k * n + j];
    Lr[j * n + j] = std::sqrt(d);
    for (int i = j + 1; i < n; ++i) {
      double v = A[j * n + i];
      for (int k = 0; k < j; ++k) v -= Lr[k * n + i] * Lr[k * n + j];
      Lr[j * n + i] = v / Lr[j * n + j];
    }
  }
  for (int j = 0; j < n; ++j) {
    Wr[j * n + j] = 1.0 / Lr[j * n + j];
    for (int i = j + 1; i < n; ++i) {
      double sacc = 0;
      for (int k = j; k < i; ++k) sacc += Lr[k * n + i] * Wr[j * n + k];
      Wr[j * n + i] = -sacc / Lr[i * n + i];
    }
  }
  double *dA, *dL, *dW;
  unsigned long long* dst;
  hipMalloc(&dA, n * n * 8); hipMalloc(&dL, n * n * 8); hipMalloc(&dW, n * n * 8); hipMalloc(&dst, 8 * (2 + 128));
  hipMemcpy(dA, A.data(), n * n * 8, hipMemcpyHostToDevice);
  for (int v : {16, 16}) {
    sfm::k_bench<<<1, 256>>>(dA, dL, dW, dst, reps, n);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
    unsigned long long st[2 + 128];
    std::vector<double> L(n * n), W(n * n);
    hipMemcpy(st, dst, 8 * (2 + 128), hipMemcpyDeviceToHost);
#ifdef POTRF_STAMPS
    // clocks since panel 0 start of wave 0, last rep, per wave and stamp
    const long long z = (long long)st[2 + 0];
    for (int w = 0; w < 4; ++w) {
      printf("wave %d:", w);
      for (int id = 0; id < 18; ++id) printf(" %lld", (long long)st[2 + 32 * w + id] - z);
      printf("\n");
    }
#endif
    hipMemcpy(L.data(), dL, n * n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(W.data(), dW, n * n * 8, hipMemcpyDeviceToHost);
    double eL = 0, eW = 0;
    for (int j = 0; j < n; ++j)
      for (int i = j; i < n; ++i) {
        eL = std::max(eL, std::fabs(L[j * n + i] - Lr[j * n + i]) / std::fabs(Lr[j * n + j]));
        eW = std::max(eW, std::fabs(W[j * n + i] - Wr[j * n + i]) * std::fabs(Lr[i * n + i]));
      }
    // W upper part of each 16x16 diagonal block must be zero (MFMA operand)
    double up = 0;
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < j; ++i)
        if (i / 16 == j / 16) up = std::max(up, std::fabs(W[j * n + i]));
    uint64_t h = 1469598103934665603ull;
    for (int k = 0; k < n * n; ++k) {
      uint64_t a, b;
      std::memcpy(&a, &L[k], 8);
      std::memcpy(&b, &W[k], 8);
      if ((k % n) >= (k / n)) h = (h ^ a) * 1099511628211ull;  // lower triangle of L
      h = (h ^ b) * 1099511628211ull;
    }
    printf("potrf_tile%-2d  %.2f us per tile (s_memrealtime 100 MHz)  max rel |L-Lref| %.2e  |W-Wref| %.2e  W-upper %.1e  bad %llu  checksum %016llx\n",
           v, st[0] / 100.0 / reps, eL, eW, up, st[1], (unsigned long long)h);
  }
  return 0;
}
