// Clock count of the POTRF panel loop (chol_kernels.hip potrf_tile, panels
// 1..3: wave 0, lane r = row r, 16 pivots) in isolation, with ablations that
// remove one ingredient at a time (wrong results; timing only):
//   V0  production form
//   V1  no LDS in the loop (column broadcasts from registers)
//   V2  no deferred column updates at all
//   V3  no readlanes (pivot and l1 taken from the lane's own registers)
//   V4  chain only (rsqrt, l, dn, readlane)
//   V5  production, scheduling barrier only between the chain and the updates
//   V6  production, no scheduling barriers
//   V7  production, scheduling barrier only at the end of each step
//   V8  production with the chain through 1/d (rcp) instead of l = p rsqrt(d)
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/panel_micro.hip -o tools/panel_micro
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int TS = 65;

__device__ __forceinline__ double rsqrt_nr(double d) {
  const double y = __builtin_amdgcn_rsq(d);
  const double e = fma(-d * y, y, 1.0);
  return fma(y * e, fma(e, 0.375, 0.5), y);
}
__device__ __forceinline__ double rcp_nr(double d) {
  const double y = __builtin_amdgcn_rcp(d);
  const double e = fma(-d, y, 1.0);
  return fma(y, fma(e, e, e), y);
}
__device__ __forceinline__ double bcast(double v, int src) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
  return __hiloint2double(hi, lo);
}

template <int V>
__device__ __forceinline__ void panel(double* T, int g0, bool& bad) {
  const int r = threadIdx.x & 63;
  const bool wl = r < 16;
  double p[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) p[j] = wl ? ((j == r) ? 1.0 : 0.0) : T[(g0 + j) * TS + r];
  double d = V == 3 ? p[0] + 4.0 : bcast(p[0], g0);
  double lp = 0.0, lcp[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) lcp[c] = 0.0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int g = g0 + j;
    bad |= !(d > 0.0);
    const double inv = rsqrt_nr(d);
    double dn = 0.0, l1 = 0.0;
    if (V == 8 && j < 15) {  // chain through 1/d: dn = (p[j+1] - lp^2) - p[j]^2 / d
      const double rr = rcp_nr(d);
      const double psq = p[j] * p[j];
      const double dg = j >= 1 ? fma(-lp, lp, p[j + 1]) : p[j + 1];
      dn = bcast(fma(-psq, rr, dg), g + 1);
    }
    const double l = p[j] * inv;
    p[j] = l;
    if (j < 15) {
      const double dg = j >= 1 ? fma(-lp, lp, p[j + 1]) : p[j + 1];
      if (V == 8) {
        l1 = bcast(l, g + 1);
      } else if (V == 3) {
        dn = fma(-l, l, dg) + 4.0;
        l1 = l * 0.5;
      } else {
        dn = bcast(fma(-l, l, dg), g + 1);
        l1 = bcast(l, g + 1);
      }
    }
    if (V != 6 && V != 7) __builtin_amdgcn_sched_barrier(0);
    if (V != 4) {
      if (V != 1) T[g * TS + r] = l;
      if (V != 2 && j >= 1 && j < 15) {
#pragma unroll
        for (int c = j + 1; c < 16; ++c) p[c] = fma(-lp, lcp[c], p[c]);
      }
      if (j < 15) {
        p[j + 1] = fma(-l, l1, p[j + 1]);
        if (j < 14 && V != 2) {
#pragma unroll
          for (int c = j + 2; c < 16; ++c) lcp[c] = V == 1 ? p[c] * 0.25 : T[g * TS + g0 + c];
        }
      }
    }
    if (j < 15) {
      lp = l;
      d = dn;
    }
    if (V != 5 && V != 6) __builtin_amdgcn_sched_barrier(0);
  }
  if (wl)
#pragma unroll
    for (int c = 0; c < 16; ++c) T[(g0 + r) * TS + g0 + c] = p[c];
}

template <int V>
__global__ __launch_bounds__(64) void k_panel(const double* A, double* out, long long* clk, int reps) {
  __shared__ double T[64 * TS];
  const int t = threadIdx.x;
  bool bad = false;
  long long tot = 0;
  for (int rep = 0; rep < reps; ++rep) {
    for (int q = 0; q < 64; ++q) T[q * TS + t] = A[q * 64 + t];
    __syncthreads();
    const long long t0 = clock64();
    panel<V>(T, 16, bad);
    const long long t1 = clock64();
    tot += t1 - t0;
    __syncthreads();
  }
  out[t] = T[20 * TS + t] + (bad ? 1.0 : 0.0);
  if (t == 0) clk[V] = tot;
}

int main() {
  const int n = 64, reps = 20;
  double hA[64 * 64];
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) hA[j * n + i] = (i == j) ? 100.0 : 0.01 * ((i * 7 + j * 3) % 11);
  double *A, *out;
  long long* clk;
  hipMalloc(&A, sizeof(hA));
  hipMalloc(&out, 64 * 8);
  hipMalloc(&clk, 16 * 8);
  hipMemcpy(A, hA, sizeof(hA), hipMemcpyHostToDevice);
  const char* nm[] = {"production", "no LDS", "no deferred updates", "no readlanes", "chain only",
                      "barrier A|B only", "no barriers", "barrier end only", "rcp chain"};
  for (int pass = 0; pass < 2; ++pass) {
    k_panel<0><<<1, 64>>>(A, out, clk, reps);
    k_panel<1><<<1, 64>>>(A, out, clk, reps);
    k_panel<2><<<1, 64>>>(A, out, clk, reps);
    k_panel<3><<<1, 64>>>(A, out, clk, reps);
    k_panel<4><<<1, 64>>>(A, out, clk, reps);
    k_panel<5><<<1, 64>>>(A, out, clk, reps);
    k_panel<6><<<1, 64>>>(A, out, clk, reps);
    k_panel<7><<<1, 64>>>(A, out, clk, reps);
    k_panel<8><<<1, 64>>>(A, out, clk, reps);
    hipDeviceSynchronize();
    long long h[9];
    hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
    for (int v = 0; v < 9; ++v) printf("V%d %-22s %7.1f clk per pivot\n", v, nm[v], double(h[v]) / reps / 16);
  }
  return 0;
}
