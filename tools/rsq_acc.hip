// Accuracy of v_rsq_f64 (raw and with 1 / 2 Newton steps) against 1/sqrt in double.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
__global__ void k(const double* d, double* o0, double* o1, double* o2, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double x = d[i];
  double y = __builtin_amdgcn_rsq(x);
  o0[i] = y;
  y = y * fma(-0.5 * x * y, y, 1.5);
  o1[i] = y;
  y = y * fma(-0.5 * x * y, y, 1.5);
  o2[i] = y;
}
int main() {
  const int n = 1 << 20;
  std::vector<double> d(n), o0(n), o1(n), o2(n);
  unsigned long long s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    d[i] = std::ldexp(1.0 + (s >> 11) * 0x1.0p-53, int(s % 60) - 30);
  }
  double *dd, *a, *b, *c;
  hipMalloc(&dd, 8 * n); hipMalloc(&a, 8 * n); hipMalloc(&b, 8 * n); hipMalloc(&c, 8 * n);
  hipMemcpy(dd, d.data(), 8 * n, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(dd, a, b, c, n);
  hipMemcpy(o0.data(), a, 8 * n, hipMemcpyDeviceToHost);
  hipMemcpy(o1.data(), b, 8 * n, hipMemcpyDeviceToHost);
  hipMemcpy(o2.data(), c, 8 * n, hipMemcpyDeviceToHost);
  double e0 = 0, e1 = 0, e2 = 0;
  for (int i = 0; i < n; ++i) {
    const long double r = 1.0L / std::sqrt((long double)d[i]);
    e0 = std::fmax(e0, double(std::fabs((o0[i] - r) / r)));
    e1 = std::fmax(e1, double(std::fabs((o1[i] - r) / r)));
    e2 = std::fmax(e2, double(std::fabs((o2[i] - r) / r)));
  }
  std::printf("max rel err: rsq %.3e  +1NR %.3e  +2NR %.3e  (ulp %.3e)\n", e0, e1, e2, 0x1.0p-53);
}
