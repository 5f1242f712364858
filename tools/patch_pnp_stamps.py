# Patch for tools/mkvar.sh (file pnp_kernels.hip): s_memrealtime stamps in
# k_pnp_epnp -> g_pstamp[(hypothesis * 3 + wave) * 8 + slot] (100 MHz):
# 0 start, 1 M^T M built (before the 12x12 SVD), 2 after the SVD, 3 common
# part done, 4 case done; read by sfm_debug_pstamps (tools/pnp_stamps.py).
def _rep(s, old, new):
    assert s.count(old) == 1, "patch_pnp_stamps: anchor not found:\n" + old
    return s.replace(old, new)
s = _rep(s, "__host__ __device__ void rodrigues_v2m(", """__device__ unsigned long long g_pstamp[64 * 3 * 8];
#define PSTAMP(slot) do { if ((threadIdx.x & 63) == 0 && blockIdx.x < 64) g_pstamp[(blockIdx.x * 3 + (threadIdx.x >> 6)) * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); } while (0)
__host__ __device__ void rodrigues_v2m(""")
s = _rep(s, "    cv_svd12_lanes(u, lds, ut);\n", "    PSTAMP(1);\n    cv_svd12_lanes(u, lds, ut);\n    PSTAMP(2);\n")
s = _rep(s, """  EpnpCommon cm;
  epnp5_common(in, k, lds[w], cm);
  double R[9], t[3], r[3];
  const double e = epnp5_case(w, in, k, cm, R, t);""", """  PSTAMP(0);
  EpnpCommon cm;
  epnp5_common(in, k, lds[w], cm);
  PSTAMP(3);
  double R[9], t[3], r[3];
  const double e = epnp5_case(w, in, k, cm, R, t);
  PSTAMP(4);""")
s += '''
extern "C" int sfm_debug_pstamps(unsigned long long* out, int n) {
  if (n > 64 * 3 * 8) n = 64 * 3 * 8;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(sfm::g_pstamp), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -5;
}
'''
