# Patch for tools/mkvar.sh (file pnp_kernels.hip): stamps inside the beta
# cases of k_pnp_epnp -> g_pstamp[(hypothesis * 3 + wave) * 8 + slot]:
# 0 case start, 1 after the least squares (cv::solve SVD), 2 after
# Gauss-Newton, 3 after compute_R_and_t; read by sfm_debug_pstamps.
def _rep(s, old, new, cnt=1):
    assert s.count(old) == cnt, ("patch_pnp_stamps2: anchor count", old, s.count(old))
    return s.replace(old, new)
s = _rep(s, "__host__ __device__ void rodrigues_v2m(", """__device__ unsigned long long g_pstamp[64 * 3 * 8];
#if defined(__HIP_DEVICE_COMPILE__)
#define PSTAMP(slot) do { if ((threadIdx.x & 63) == 0 && blockIdx.x < 64) g_pstamp[(blockIdx.x * 3 + (threadIdx.x >> 6)) * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define PSTAMP(slot) do {} while (0)
#endif
__host__ __device__ void rodrigues_v2m(""")
s = _rep(s, "    gauss_newton(L, rho, be);\n    return r_and_t(in, alpha, ut, be, k, R, t);\n",
         "    PSTAMP(1);\n    gauss_newton(L, rho, be);\n    PSTAMP(2);\n    const double e_ = r_and_t(in, alpha, ut, be, k, R, t);\n    PSTAMP(3);\n    return e_;\n", 3)
s = _rep(s, """  const double (&rho)[6] = cm.rho;
  if (N == 0) {""", """  const double (&rho)[6] = cm.rho;
  PSTAMP(0);
  if (N == 0) {""")
s += '''
extern "C" int sfm_debug_pstamps(unsigned long long* out, int n) {
  if (n > 64 * 3 * 8) n = 64 * 3 * 8;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(sfm::g_pstamp), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -5;
}
'''
