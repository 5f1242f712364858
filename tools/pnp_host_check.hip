// Host build of the device EPnP (pnp_kernels.hip's __host__ __device__
// routines) on the subsets of the oracle's RANSAC trace, to compare the
// kernel's arithmetic with oracle/pnp_oracle.py on the CPU:
//   hipcc -O2 -std=c++17 -ffp-contract=off tools/pnp_host_check.hip -o tools/pnp_host_check
// stdin: fu fv uc vc n, then n lines "X Y Z u v" (float32-exact values);
// stdout: R (9) t (3) of epnp5 on the n (= 5) points.
#include "../sfm_amd/csrc/pnp_kernels.hip"
#include <cstdio>
void sfm_internal_set_error(const std::string&) {}
int main() {
  sfm::PnPCam k;
  int n;
  if (scanf("%lf %lf %lf %lf %d", &k.fu, &k.fv, &k.uc, &k.vc, &n) != 5 || n != 5) return 1;
  sfm::EpnpIn in;
  for (int p = 0; p < n; ++p) {
    double X, Y, Z, u, v;
    if (scanf("%lf %lf %lf %lf %lf", &X, &Y, &Z, &u, &v) != 5) return 1;
    in.pw[p][0] = X; in.pw[p][1] = Y; in.pw[p][2] = Z;
    const float xn = float((u - k.uc) * (1.0 / k.fu)), yn = float((v - k.vc) * (1.0 / k.fv));
    in.us[p][0] = double(xn) * k.fu + k.uc;
    in.us[p][1] = double(yn) * k.fv + k.vc;
  }
  double R[9], t[3];
  sfm::epnp5(in, k, nullptr, R, t);
  for (int i = 0; i < 9; ++i) printf("%.17g ", R[i]);
  for (int i = 0; i < 3; ++i) printf("%.17g ", t[i]);
  printf("\n");
  return 0;
}
