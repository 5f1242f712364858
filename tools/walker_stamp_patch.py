# Patch for tools/mkvar.sh (file chol_kernels.hip): s_memrealtime stamps at the
# diagonal walker's phase boundaries -> g_wstamp[step][slot] (100 MHz clock),
# read back by sfm_debug_stamps (tools/walker_phases.py).
s = s.replace('namespace sfm {\nnamespace {\n', '''namespace sfm {
__device__ unsigned long long g_wstamp[64 * 16];
namespace {
#define WSTAMP(j, k) do { if (threadIdx.x == 0 && (j) < 64) g_wstamp[(j) * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
''', 1)
s = s.replace('''  for (int j = 0; j < nb; ++j) {
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
    }''', 1)
s = s.replace('''    const bool bad = (j0 + NB <= n) ? potrf_tile<true>(T, Wl, scr, j0, n) : potrf_tile<false>(T, Wl, scr, j0, n);
    if (bad) atomicOr(fail, 1);''', '''    WSTAMP(j, 1);
    const bool bad = (j0 + NB <= n) ? potrf_tile<true>(T, Wl, scr, j0, n) : potrf_tile<false>(T, Wl, scr, j0, n);
    WSTAMP(j, 2);
    if (bad) atomicOr(fail, 1);''', 1)
s = s.replace('''    if (j + 1 == nb) break;
    // subdiagonal tile''', '''    WSTAMP(j, 3);
    if (j + 1 == nb) break;
    // subdiagonal tile''', 1)
s = s.replace('''    block_wait(Pf + (j + 1) * nb + j, epoch, fail);
    load_tile(T, A, ld, i0, j0);''', '''    block_wait(Pf + (j + 1) * nb + j, epoch, fail);
    WSTAMP(j, 4);
    load_tile(T, A, ld, i0, j0);''', 1)
s = s.replace('''    block_wait(Pf + (j + 1) * nb + j + 1, epoch, fail);''', '''    block_wait(Pf + (j + 1) * nb + j + 1, epoch, fail);
    WSTAMP(j, 5);''', 1)
s = s.replace('''    trsm_lds(T, Wl, x, lane);
    put_tile(Ls, x, lane);''', '''    trsm_lds(T, Wl, x, lane);
    put_tile(Ls, x, lane);
    WSTAMP(j, 6);''', 1)
s = s.replace('''    block_publish_wt(F + (j + 1) * nb + j, epoch);
  }
}''', '''    block_publish_wt(F + (j + 1) * nb + j, epoch);
    WSTAMP(j, 7);
  }
}''', 1)
s += '''
extern "C" int sfm_debug_stamps(unsigned long long* out, int n) {
  if (n > 64 * 16) n = 64 * 16;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(sfm::g_wstamp), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -5;
}
'''

# POTRF internals: after each panel (slots 8..11), after each trailing update (12..14), after W row 3 (15)
s = s.replace("""      if (r < 16)
#pragma unroll
        for (int c = 0; c < 16; ++c) Wl[(g0 + r) * TS + g0 + c] = wc[c];
    } else if (b >= 2 && w - 1 < b - 1) {""", """      if (r < 16)
#pragma unroll
        for (int c = 0; c < 16; ++c) Wl[(g0 + r) * TS + g0 + c] = wc[c];
    } else if (b >= 2 && w - 1 < b - 1) {""", 1)
s = s.replace("""    __syncthreads();
    // ---- trailing update: blocks (I, J), b < J <= I <= 3 ----""", """    __syncthreads();
    WSTAMP(k0 / 64, 8 + b);
    // ---- trailing update: blocks (I, J), b < J <= I <= 3 ----""", 1)
s = s.replace("""        for (int rr = 0; rr < 4; ++rr) T[(16 * J + j) * TS + 16 * I + 4 * rr + kk] -= acc[rr];
      }
      __syncthreads();
    }
  }""", """        for (int rr = 0; rr < 4; ++rr) T[(16 * J + j) * TS + 16 * I + 4 * rr + kk] -= acc[rr];
      }
      __syncthreads();
      WSTAMP(k0 / 64, 12 + b);
    }
  }""", 1)
s = s.replace("""  if (w < 3) w_offdiag(T, Wl, scr[w], 3, w, lane);
  __syncthreads();
  return bad;""", """  if (w < 3) w_offdiag(T, Wl, scr[w], 3, w, lane);
  __syncthreads();
  WSTAMP(k0 / 64, 15);
  return bad;""", 1)
