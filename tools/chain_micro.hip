// Diagnostic microbenchmark (not product code): wall-clock latency of the
// primitives on the POTRF pivot chain (chol_kernels.hip potrf_tile), one
// wave, dependent loops of ITER steps timed with hipEvents after a warm-up
// launch (so the clocks have ramped), reported in ns per step.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/chain_micro.hip -o tools/chain_micro
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITER = 20000;

__device__ __forceinline__ double bcast(double v, int src) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
  return __hiloint2double(hi, lo);
}

template <int kMode>
__global__ __launch_bounds__(64) void chain(double* out, double seed, double a, int src) {
  const int t = threadIdx.x;
  double x = seed + 1e-3 * t, y = 1.0 + 1e-4 * t;
  for (int i = 0; i < ITER; ++i) {
    if constexpr (kMode == 0) {  // dependent fp64 FMA
      x = fma(x, a, 1e-9);
    } else if constexpr (kMode == 1) {  // dependent v_rsq_f64 (+ fma to stay in range)
      x = fma(__builtin_amdgcn_rsq(x), a, 0.75);
    } else if constexpr (kMode == 2) {  // dependent readlane pair + fma
      x = fma(bcast(x, src), a, 1e-9);
    } else if constexpr (kMode == 3) {  // the pivot chain: rsq, third-order step, l, d', readlane pair
      const double yy = __builtin_amdgcn_rsq(x);
      const double e = fma(-x * yy, yy, 1.0);
      const double inv = fma(yy * e, fma(e, 0.375, 0.5), yy);
      const double l = y * inv;
      x = bcast(fma(-l, l, 2.0 * x), src);
    } else if constexpr (kMode == 4) {  // the chain without the refinement
      const double inv = __builtin_amdgcn_rsq(x);
      const double l = y * inv;
      x = bcast(fma(-l, l, 2.0 * x), src);
    } else if constexpr (kMode == 5) {  // dependent v_sqrt_f64 + v_rcp_f64
      x = fma(__builtin_amdgcn_rcp(__builtin_amdgcn_sqrt(x)), a, 0.75);
    } else if constexpr (kMode == 6) {  // fp32 rsq in the chain (precision experiment)
      const double yy = double(__builtin_amdgcn_rsqf(float(x)));
      const double e = fma(-x * yy, yy, 1.0);
      const double inv = fma(yy * e, fma(e, 0.375, 0.5), yy);
      const double l = y * inv;
      x = bcast(fma(-l, l, 2.0 * x), src);
    }
  }
  out[t] = x;
}

template <int kMode>
float run(double* o, hipEvent_t e0, hipEvent_t e1) {
  chain<kMode><<<1, 64>>>(o, 1.0, 0.999999, 3);
  hipEventRecord(e0);
  chain<kMode><<<1, 64>>>(o, 1.0, 0.999999, 3);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e6f / ITER;
}

__global__ void spin(double* o) {  // clock warm-up
  double x = threadIdx.x;
  for (int i = 0; i < 2000000; ++i) x = fma(x, 0.9999999, 1e-9);
  o[threadIdx.x] = x;
}

int main() {
  double* o;
  hipMalloc(&o, 1024 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  spin<<<256, 256>>>(o);
  hipDeviceSynchronize();
  const char* names[] = {"fma_f64", "rsq_f64 + fma", "readlane x2 + fma", "pivot chain (rsq, refine, l, d', readlane x2)",
                         "pivot chain, no refinement", "sqrt_f64 + rcp_f64 + fma", "pivot chain, f32 rsq seed"};
  for (int r = 0; r < 2; ++r) {
    float v[7] = {run<0>(o, e0, e1), run<1>(o, e0, e1), run<2>(o, e0, e1), run<3>(o, e0, e1),
                  run<4>(o, e0, e1), run<5>(o, e0, e1), run<6>(o, e0, e1)};
    for (int i = 0; i < 7; ++i) printf("%-48s %7.2f ns per step\n", names[i], v[i]);
    printf("--\n");
  }
  return 0;
}
