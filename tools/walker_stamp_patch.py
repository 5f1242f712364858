# Patch for tools/mkvar.sh (file chol_kernels.hip): s_memrealtime stamps at the
# diagonal walker's phase boundaries -> g_wstamp[step][slot] (100 MHz clock),
# read back by sfm_debug_stamps (tools/walker_phases.py).
def _rep(s, old, new):
    assert s.count(old) >= 1, "walker_stamp_patch: anchor not found:\n" + old
    return s.replace(old, new, 1)


s = _rep(s, 'namespace sfm {\nnamespace {\n', '''namespace sfm {
__device__ unsigned long long g_wstamp[64 * 16];
namespace {
#define WSTAMP(j, k) do { if (threadIdx.x == 0 && (j) < 64) g_wstamp[(j) * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
''')
s = _rep(s, '''  for (int j = 0; j < nb; ++j) {
    const int j0 = j * NB;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = t + 256 * q, c = e >> 6, r = e & 63;
      T[c * TS + r] = nx[q];
    }''', '''  for (int j = 0; j < nb; ++j) {
    const int j0 = j * NB;
    WSTAMP(j, 0);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = t + 256 * q, c = e >> 6, r = e & 63;
      T[c * TS + r] = nx[q];
    }''')
s = _rep(s, '''    const bool bad = (j0 + NB <= n) ? potrf_tile<true>(T, Wl, scr, j0, n, dl) : potrf_tile<false>(T, Wl, scr, j0, n, dl);
    if (bad) atomicOr(fail, 1);''', '''    WSTAMP(j, 1);
    const bool bad = (j0 + NB <= n) ? potrf_tile<true>(T, Wl, scr, j0, n, dl) : potrf_tile<false>(T, Wl, scr, j0, n, dl);
    WSTAMP(j, 2);
    if (bad) atomicOr(fail, 1);''')
s = _rep(s, '''    if (j + 1 == nb) break;
    // subdiagonal tile''', '''    WSTAMP(j, 3);
    if (j + 1 == nb) break;
    // subdiagonal tile''')
s = _rep(s, '''    block_wait(Pf + (j + 1) * nb + j, epoch, fail);
    load_tile(T, A, ld, i0, j0);''', '''    block_wait(Pf + (j + 1) * nb + j, epoch, fail);
    WSTAMP(j, 4);
    load_tile(T, A, ld, i0, j0);''')
s = _rep(s, '''    block_wait(Pf + (j + 1) * nb + j + 1, epoch, fail);''', '''    block_wait(Pf + (j + 1) * nb + j + 1, epoch, fail);
    WSTAMP(j, 5);''')
s = _rep(s, '''    trsm_lds(T, Wl, x, lane);
    put_tile(Ls, x, lane);''', '''    trsm_lds(T, Wl, x, lane);
    put_tile(Ls, x, lane);
    WSTAMP(j, 6);''')
s = _rep(s, '''    block_publish_wt(F + (j + 1) * nb + j, epoch);
  }
}''', '''    block_publish_wt(F + (j + 1) * nb + j, epoch);
    WSTAMP(j, 7);
  }
}''')
s += '''
extern "C" int sfm_debug_stamps(unsigned long long* out, int n) {
  if (n > 64 * 16) n = 64 * 16;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(sfm::g_wstamp), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -5;
}
'''

# POTRF internals: after each panel (slots 8..11), after each trailing update (12..14), after W row 3 (15)
s = _rep(s, """    __syncthreads();
    // ---- trailing update of column block b+1""", """    __syncthreads();
    WSTAMP(k0 / 64, 8 + b);
    // ---- trailing update of column block b+1""")
s = _rep(s, """      if (w < 3 - b) trail_block(T, g0, b + 1 + w, b + 1, lane);
      __syncthreads();""", """      if (w < 3 - b) trail_block(T, g0, b + 1 + w, b + 1, lane);
      __syncthreads();
      WSTAMP(k0 / 64, 12 + b);""")
s = _rep(s, """  if (w >= 1) w_row3_finish(Wl, scr[w], w - 1, lane);
  __syncthreads();
  return bad;""", """  if (w >= 1) w_row3_finish(Wl, scr[w], w - 1, lane);
  __syncthreads();
  WSTAMP(k0 / 64, 15);
  return bad;""")
