// Dependent-latency probe for the pivot chain of the dense Cholesky
// (chol_kernels.hip potrf_tile): one wave, clock counts of dependent chains
// of the operations the chain is made of.  Build + run (GPU box):
//   hipcc -O3 --offload-arch=gfx950 tools/lat_probe.hip -o tools/lat_probe && tools/lat_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int R = 512;

__device__ __forceinline__ double bcast(double v, int src) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double rsqrt_nr(double d) {
  const double y = __builtin_amdgcn_rsq(d);
  const double e = fma(-d * y, y, 1.0);
  return fma(y * e, fma(e, 0.375, 0.5), y);
}

__global__ void k_probe(const double* in, double* out, long long* clk, int which) {
  __shared__ double lds[256];
  const int lane = threadIdx.x;
  double x = in[lane], a = in[64 + lane], b = in[128 + lane];
  f64x4 acc = {x, a, b, x};
  f64x4 acc2 = acc, acc3 = acc, acc4 = acc;
  lds[lane] = x;
  __syncthreads();
  const long long t0 = clock64();
  switch (which) {
    case 0:  // dependent fma
      for (int i = 0; i < R; ++i) x = fma(x, a, b);
      break;
    case 1:  // dependent mul
      for (int i = 0; i < R; ++i) x = x * a;
      break;
    case 2:  // dependent rsq (raw)
      for (int i = 0; i < R; ++i) x = __builtin_amdgcn_rsq(x);
      break;
    case 3:  // fma + 64-bit readlane broadcast (the chain's bcast)
      for (int i = 0; i < R; ++i) x = bcast(fma(x, a, b), i & 63);
      break;
    case 4:  // LDS round trip: write by every lane, read another lane's word
      for (int i = 0; i < R; ++i) {
        lds[lane] = x;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        x = lds[(lane + 1) & 63] * a;
      }
      break;
    case 5:  // dependent MFMA f64 16x16x4
      for (int i = 0; i < R; ++i) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
      break;
    case 6:  // 4 independent MFMA chains (issue rate)
      for (int i = 0; i < R / 4; ++i) {
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, x, acc2, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, acc3, 0, 0, 0);
        acc4 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, b, acc4, 0, 0, 0);
      }
      break;
    case 7:  // the pivot step: rsqrt + third-order step, l = p * inv, dn = fma, bcast
      for (int i = 0; i < R; ++i) {
        const double inv = rsqrt_nr(x);
        const double l = a * inv;
        x = bcast(fma(-l, l, b + 4.0), i & 63);
      }
      break;
    case 8:  // reciprocal chain: rcp + 3-op third-order step + fma + bcast (LDL form)
      for (int i = 0; i < R; ++i) {
        const double y = __builtin_amdgcn_rcp(x);
        const double e = fma(-x, y, 1.0);
        const double r = fma(y, fma(e, e, e), y);
        x = bcast(fma(-a * a, r, b + 4.0), i & 63);
      }
      break;
    case 9:  // independent fma issue rate (8 chains)
    {
      double y0 = x, y1 = a, y2 = b, y3 = x + 1, y4 = a + 1, y5 = b + 1, y6 = x + 2, y7 = a + 2;
      for (int i = 0; i < R / 8; ++i) {
        y0 = fma(y0, a, b); y1 = fma(y1, a, b); y2 = fma(y2, a, b); y3 = fma(y3, a, b);
        y4 = fma(y4, a, b); y5 = fma(y5, a, b); y6 = fma(y6, a, b); y7 = fma(y7, a, b);
      }
      x = y0 + y1 + y2 + y3 + y4 + y5 + y6 + y7;
      break;
    }
  }
  const long long t1 = clock64();
  out[lane] = x + acc[0] + acc[1] + acc[2] + acc[3] + acc2[0] + acc3[1] + acc4[2];
  if (lane == 0) clk[which] = t1 - t0;
}

int main() {
  double h_in[192];
  for (int i = 0; i < 64; ++i) { h_in[i] = 1.0 + 1e-3 * i; h_in[64 + i] = 0.999; h_in[128 + i] = 1e-3; }
  double *in, *out;
  long long* clk;
  hipMalloc(&in, sizeof(h_in));
  hipMalloc(&out, 64 * sizeof(double));
  hipMalloc(&clk, 16 * sizeof(long long));
  hipMemcpy(in, h_in, sizeof(h_in), hipMemcpyHostToDevice);
  const char* names[] = {"fma dep", "mul dep", "rsq dep", "fma+readlane", "lds round trip", "mfma f64 dep",
                         "mfma f64 4 indep", "pivot step (rsq form)", "pivot step (rcp form)", "fma 8 indep"};
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  std::printf("device %s, clockRate %d kHz (clock64 = shader clock)\n", p.name, p.clockRate);
  for (int w = 0; w < 10; ++w) {
    k_probe<<<1, 64>>>(in, out, clk, w);  // warm
    k_probe<<<1, 64>>>(in, out, clk, w);
    hipDeviceSynchronize();
    long long c = 0;
    hipMemcpy(&c, clk + w, sizeof(c), hipMemcpyDeviceToHost);
    std::printf("%-24s %8.1f clk per step\n", names[w], double(c) / R);
  }
  return 0;
}
