// Dense reduced-camera Cholesky for gfx950: the replacement of the Eigen
// LLT that Ceres' DenseSchurComplementSolver runs on the reduced camera
// matrix (DENSE_SCHUR, /root/reference/CTracker.cpp:574).
//
// Storage: column-major lower triangle (element (i, j), i >= j, at j*ld + i),
// which is byte-identical to the row-major upper triangle the Schur kernel
// writes.  Row n (= 6C) holds the reduced right-hand side, so factoring the
// augmented matrix performs the forward substitution z = L^-1 rhs for free;
// rows beyond n are identity padding up to a multiple of the 64-wide tile.
//
// Blocked algorithm, tile 64, in ONE persistent launch (k_chol_fused): a
// diagonal walker factors tile (k,k) (POTRF on v_mfma_f64_16x16x4_f64 with a
// register pivot chain) and forms W_k = L_kk^-1; helper workgroups
// accumulate the off-diagonal tiles' updates on MFMA and finish them with
// X = T W_k^T.  Then the back substitution L^T y = z in one launch with
// flag-chained block rows (k_backsolve).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstdlib>
#include "ba_device.h"
#include "ba_common.h"

namespace sfm {
#ifdef SFM_CHOL_STAMPS
// Development build only (tools/chol_stamps.sh): s_memrealtime (100 MHz)
// stamps of the diagonal walker's phases, g_wstamp[step][slot], and the
// helpers' publication times of the tiles the walker awaits, g_hstamp[i][j]
// (slot 0: partial tile, slot 1: final tile).  Read by sfm_debug_stamps.
__device__ unsigned long long g_wstamp[256 * 16];
__device__ unsigned long long g_hstamp[128 * 128 * 2];
__device__ unsigned long long g_pstamp[256 * 4];  // per wave: the end of its panel-3 work
__device__ unsigned long long g_bstamp[256 * 8];  // k_backsolve per block row (sfm_debug_bstamps)
#define BSTAMP(b, k)                                                                          \
  do {                                                                                        \
    if (threadIdx.x == 0 && (b) < 256) g_bstamp[(b) * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define WSTAMP(j, k)                                                                          \
  do {                                                                                        \
    if (threadIdx.x == 0 && (j) < 256) g_wstamp[(j) * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define WSTAMPV(j, k, v)                                       \
  do {                                                         \
    if (threadIdx.x == 0 && (j) < 256) g_wstamp[(j) * 16 + (k)] = (v); \
  } while (0)
#define PSTAMP(j, w)                                                                                      \
  do {                                                                                                    \
    if ((threadIdx.x & 63) == 0 && (j) < 256) g_pstamp[(j) * 4 + (w)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define HSTAMP(i, j, k)                                                                                         \
  do {                                                                                                          \
    if (threadIdx.x == 0 && (i) < 128 && (j) < 128) g_hstamp[((i) * 128 + (j)) * 2 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define WSTAMP(j, k) do { } while (0)
#define WSTAMPV(j, k, v) do { } while (0)
#define HSTAMP(i, j, k) do { } while (0)
#define PSTAMP(j, w) do { } while (0)
#define BSTAMP(b, k) do { } while (0)
#endif
namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int NB = kNB;  // 64

// ---------------------------------------------------------------------------
// Pivot: 1/sqrt(d) by the hardware estimate + two Newton steps (full double
// precision), sqrt(d) = d * (1/sqrt(d)).  Keeps the pivot chain short.
__device__ __forceinline__ double rsqrt_nr(double d) {
  // v_rsq_f64 is good to ~5e-8; one third-order step
  //   y1 = y0 (1 + e/2 + 3e^2/8),  e = 1 - d y0^2
  // reaches full precision with four dependent operations (two Newton
  // steps would take six).
  const double y = __builtin_amdgcn_rsq(d);
  const double e = fma(-d * y, y, 1.0);
  return fma(y * e, fma(e, 0.375, 0.5), y);
}

// Uniform broadcast of lane `src`'s double (two v_readlane_b32 -> SGPRs).
__device__ __forceinline__ double bcast(double v, int src) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
  return __hiloint2double(hi, lo);
}

// POTRF of one 64x64 tile plus its inverse W = L^-1, four wavefronts,
// blocked in 16-column panels so that the per-pivot work is small and the
// bulk of the flops runs on MFMA.  For panel b = 0..3 (columns 16b..16b+15):
//   wave 0     factors the panel column by column, lane r = row r holding
//              its 16 panel entries in registers.  The pivot chain is
//              readlane-only: the next pivot is lane g+1's own a - l*l and
//              L(g+1, g) reaches every lane by readlane; the other columns'
//              L(c, g) come from the column just written to LDS.  Lanes
//              0..15 also carry the columns of W_bb = L_bb^-1 through the
//              same eliminations (w_j *= 1/L_jj, w_c -= L_cj w_j).
//   waves 1-3  meanwhile form row b-1 of W off the diagonal,
//              W_{b-1,J} = -W_{b-1,b-1} sum_{K=J}^{b-2} L_{b-1,K} W_KJ (MFMA).
//   all waves  then apply the trailing update C_IJ -= P_I P_J^T to the 16x16
//              blocks right of and below the panel (v_mfma_f64_16x16x4_f64).
// Row 3 of W closes the kernel.  Pivots at or beyond n (augmented row,
// identity padding) are taken as 1 so the padding stays finite; they are
// never read back.  The strictly upper part of the stored tile is a
// don't-care (never read by any kernel).
constexpr int TS = NB + 1;  // LDS column stride (doubles) of the tile images

// D (16x16) += sum_{k<16} A(i, k) B(k, j) with A(i, k) = Ap[i*ai + k*ak],
// B(k, j) = Bp[k*bk + j*bj] (LDS).  Lane l's reg r holds D(4r + (l>>4), l&15).
// The eight LDS operands are read before the first MFMA (one wait, not one
// LDS round trip per MFMA: left to itself the compiler interleaved
// read -> wait -> MFMA under the walker's register pressure); the MFMA
// order, and so every sum, is unchanged.
__device__ __forceinline__ f64x4 mfma16(const double* Ap, int ai, int ak, const double* Bp, int bk, int bj, f64x4 acc,
                                        int lane) {
  const int i = lane & 15, kk = lane >> 4;
  double a[4], b[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = 4 * s + kk;
    a[s] = Ap[i * ai + k * ak];
    b[s] = Bp[k * bk + i * bj];
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) asm volatile("" : "+v"(a[s]), "+v"(b[s]));
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], acc, 0, 0, 0);
  return acc;
}

// W_IJ = -W_II sum_{K=J}^{I-1} L_IK W_KJ, by one wavefront (scr: its 16x16 scratch).
__device__ __forceinline__ void w_offdiag(const double* T, double* Wl, double* scr, int I, int J, int lane) {
  f64x4 acc = {0.0, 0.0, 0.0, 0.0};
  for (int K = J; K < I; ++K)  // A(i,k) = L(16I+i, 16K+k), B(k,j) = W(16K+k, 16J+j)
    acc = mfma16(T + (16 * K) * TS + 16 * I, 1, TS, Wl + (16 * J) * TS + 16 * K, 1, TS, acc, lane);
  const int j = lane & 15, kk = lane >> 4;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) scr[(4 * rr + kk) * 16 + j] = acc[rr];  // row-major T1(i, j)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  f64x4 acc2 = {0.0, 0.0, 0.0, 0.0};  // A(i,k) = W(16I+i, 16I+k), B(k,j) = T1(k, j)
  acc2 = mfma16(Wl + (16 * I) * TS + 16 * I, 1, TS, scr, 16, 1, acc2, lane);
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) Wl[(16 * J + j) * TS + 16 * I + 4 * rr + kk] = -acc2[rr];
}

// W_00 = L_00^-1 from the panel-0 factor in T and the pivots' inverses inv
// [16], lane m < 16 forming column m with the very operations wave 0's panel
// carried it with before (per entry: the column updates k = 0 .. c-1 as
// fma(-L(c,k), w_k, .) in k order, then the scaling by inv_c): bitwise the
// same W_00, off the pivot chain (panel 0 went 2.43 -> see DESIGN.md §5).
__device__ __forceinline__ void trtri16(const double* T, double* Wl, const double* inv, int lane) {
  if (lane >= 16) return;
  double w[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    double acc = (c == lane) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 0; k < c; ++k) acc = fma(-T[k * TS + c], w[k], acc);
    w[c] = acc * inv[c];
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) Wl[lane * TS + c] = w[c];
}

// Row 3 of W in two halves, so that the sum runs during panel 3:
// scr = sum_{K=J}^{2} L_3K W_KJ (needs only L rows 48.. of panels 0-2 and W
// rows 0-2), then W_3J = -W_33 scr once panel 3 is out.  Same MFMA order
// as w_offdiag(T, Wl, scr, 3, J): bitwise the same W.
__device__ __forceinline__ void w_row3_sum(const double* T, const double* Wl, double* scr, int J, int lane) {
  f64x4 acc = {0.0, 0.0, 0.0, 0.0};
  for (int K = J; K < 3; ++K) acc = mfma16(T + (16 * K) * TS + 48, 1, TS, Wl + (16 * J) * TS + 16 * K, 1, TS, acc, lane);
  const int j = lane & 15, kk = lane >> 4;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) scr[(4 * rr + kk) * 16 + j] = acc[rr];
}
__device__ __forceinline__ void w_row3_finish(double* Wl, const double* scr, int J, int lane) {
  f64x4 acc2 = {0.0, 0.0, 0.0, 0.0};
  acc2 = mfma16(Wl + 48 * TS + 48, 1, TS, scr, 16, 1, acc2, lane);
  const int j = lane & 15, kk = lane >> 4;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) Wl[(16 * J + j) * TS + 48 + 4 * rr + kk] = -acc2[rr];
}

// The walker's last update T -= Ls Ls^T (Ls = L_j,j-1 in LDS) of the lower
// 16x16 blocks (I, J) = (Ib[q], Jb[q]), q < nq, by one wavefront; the MFMA
// chains of the blocks are interleaved (same k order per block as a chain).
// last_update_acc forms the products only (acc), last_update_apply
// subtracts them (the walker forms column block 0's at the end of the
// previous step, beside the drain of L_j,j-1's stores).
template <int kMax>
__device__ __forceinline__ void last_update_acc(const double* Ls, const int* Ib, const int* Jb, int nq, int lane,
                                                f64x4 (&acc)[kMax]);
template <int kMax>
__device__ __forceinline__ void last_update_apply(double* T, const int* Ib, const int* Jb, int nq, int lane,
                                                  const f64x4 (&acc)[kMax]) {
  const int li = lane & 15, kk = lane >> 4;
#pragma unroll
  for (int q = 0; q < kMax; ++q)
    if (q < nq)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) T[(16 * Jb[q] + li) * TS + 16 * Ib[q] + 4 * rr + kk] -= acc[q][rr];
}
template <int kMax>
__device__ __forceinline__ void last_update(double* T, const double* Ls, const int* Ib, const int* Jb, int nq, int lane) {
  f64x4 acc[kMax];
  last_update_acc<kMax>(Ls, Ib, Jb, nq, lane, acc);
  last_update_apply<kMax>(T, Ib, Jb, nq, lane, acc);
}
template <int kMax>
__device__ __forceinline__ void last_update_acc(const double* Ls, const int* Ib, const int* Jb, int nq, int lane,
                                                f64x4 (&acc)[kMax]) {
  const int li = lane & 15, kk = lane >> 4;
#pragma unroll
  for (int q = 0; q < kMax; ++q) acc[q] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int M = 0; M < 4; ++M) {
    // a column block's operands first, then its MFMAs (same order per block)
    double a[4][kMax], b[4][kMax];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const double* row = Ls + (16 * M + 4 * s4 + kk) * TS + li;
#pragma unroll
      for (int q = 0; q < kMax; ++q)
        if (q < nq) {
          a[s4][q] = row[16 * Ib[q]];
          b[s4][q] = row[16 * Jb[q]];
        }
    }
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int q = 0; q < kMax; ++q)
        if (q < nq) asm volatile("" : "+v"(a[s4][q]), "+v"(b[s4][q]));
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int q = 0; q < kMax; ++q)
        if (q < nq) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s4][q], b[s4][q], acc[q], 0, 0, 0);
  }
}

// Trailing update of the 16x16 block (I, J) by the panel at columns g0..g0+15,
// one wavefront: C_IJ -= P_I P_J^T.
__device__ __forceinline__ void trail_block(double* T, int g0, int I, int J, int lane) {
  const double* P = T + g0 * TS;  // P(row, kk) = L(row, g0 + kk) = P[kk*TS + row]
  f64x4 acc = {0.0, 0.0, 0.0, 0.0};
  // A(i, k) = L(16I + i, g0 + k), B(k, j) = L(16J + j, g0 + k)
  acc = mfma16(P + 16 * I, 1, TS, P + 16 * J, TS, 1, acc, lane);
  const int j = lane & 15, kk = lane >> 4;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) T[(16 * J + j) * TS + 16 * I + 4 * rr + kk] -= acc[rr];
}

// The factorisation proper, on the tile image T in LDS (256 threads; Wl is
// cleared here).  Returns this thread's bad-pivot flag; ends with a barrier.
// Ls != nullptr: the walker's last update of the blocks right of column
// block 0 is still due (the walker applied it to column block 0 only);
// waves 1-3 apply it while wave 0 factors panel 0, before the trailing
// update of panel 0 touches those blocks (every block keeps its update
// order: bitwise the same factor).
// pf_sub != nullptr: wave 2 (idle in panel 2) polls the flag of the
// walker's next partial tile (j+1, j) during panel 2 and leaves in rdy[0]
// whether it is out; if so, waves 1-3 issue their loads of that tile
// (pre.load(), to registers) at the top of their panel-3 work, and the walker
// writes them to its LDS image after the POTRF (pre.store()): the memory
// latency -- 2-3 us under the helpers' traffic, stamped -- runs beside panel
// 3 and the W row.  Wave 3 polls the next diagonal partial tile's flag
// (pf_diag) at the top of panel 3 and leaves it in rdy[1].  (The loads are
// sc1 loads of sc1-stored bytes behind a relaxed poll and a barrier: no agent
// acquire, MI355X_MICROARCH.md "Valid forms", row 1.)  Panel 3 is peeled out
// of the panel loop so that the prefetched registers are live from there on
// only.
struct NoPrefetch {
  __device__ void load() {}
  __device__ void w_early(const double*, int) {}
};

// Wave 0's factorisation of panel b >= 1 (columns g0 = 16 b ..): rows r < g0
// are above the diagonal (don't-care), so lanes 0..15 carry W_bb column r in
// p itself: the elimination applies the same operations to [A_panel | I] rows
// (p[j] *= inv, p[c] -= p[j] L(g0+c, g)), so one FMA stream updates both --
// half the pivot work of the separate wc[] registers.  Their T writes land in
// the tile's strictly upper part, which nothing reads.
template <bool kFull>
__device__ __forceinline__ void panel_w0(double* T, double* Wl, int g0, int k0, int n, int lane, bool& bad) {
  const int r = lane;
  const bool wl = r < 16;
  double p[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) p[j] = wl ? ((j == r) ? 1.0 : 0.0) : T[(g0 + j) * TS + r];
  double d = bcast(p[0], g0);
  // column j's LDS-fed updates (p[c], c >= j + 2) are applied one step
  // late, right before they are first needed, so the LDS round trip
  // overlaps the next pivot's rsqrt chain; every p[c] still takes its
  // column updates in column order (bitwise the eager form)
  double lp = 0.0, lcp[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) lcp[c] = 0.0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int g = g0 + j;
    if (kFull || k0 + g < n) bad |= !(d > 0.0);
    else d = 1.0;
    const double inv = rsqrt_nr(d);
    const double l = p[j] * inv;
    p[j] = l;
    T[g * TS + r] = l;
    if (j >= 1 && j < 15) {
#pragma unroll
      for (int c = j + 1; c < 16; ++c) p[c] = fma(-lp, lcp[c], p[c]);  // column j - 1
    }
    if (j < 15) {
      const double dn = bcast(fma(-l, l, p[j + 1]), g + 1);
      const double l1 = bcast(l, g + 1);
      p[j + 1] = fma(-l, l1, p[j + 1]);
      if (j < 14) {
#pragma unroll
        for (int c = j + 2; c < 16; ++c) lcp[c] = T[g * TS + g0 + c];
      }
      lp = l;
      d = dn;
    }
  }
  if (wl)
#pragma unroll
    for (int c = 0; c < 16; ++c) Wl[(g0 + r) * TS + g0 + c] = p[c];
}

template <bool kFull, class Pre>  // kFull: every pivot of the tile is a real one (k0 + 64 <= n)
__device__ __forceinline__ bool potrf_tile(double* T, double* Wl, double (*scr)[256], int k0, int n,
                                           const double* Ls, const int* pf_sub, const int* pf_diag, int epoch,
                                           int* rdy, Pre& pre) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = t + 256 * q, c = e >> 6, r = e & 63;
    Wl[c * TS + r] = 0.0;
  }
  if (t == 0) rdy[2] = rdy[3] = 0;  // panel 3's W_20 hand-off (wave 3 -> wave 1), its late-poll bits
  __syncthreads();
  bool bad = false;
  for (int b = 0; b < 3; ++b) {
    const int g0 = 16 * b;
    if (w == 0 && b > 0) {
      panel_w0<kFull>(T, Wl, g0, k0, n, lane, bad);
    } else if (w == 0) {
      // ---- panel 0 factorisation: lane r = row r.  W_00 is not carried here
      // (no rows above the panel to carry it in): the pivots' inverses go to
      // scr[0] and wave 2 forms W_00 during panel 1 (trtri16) ----
      const int r = lane;
      double p[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) p[j] = T[(g0 + j) * TS + r];
      double d = bcast(p[0], g0);
      double lp = 0.0, lcp[16];  // deferred LDS-fed updates, as in panels 1..3
#pragma unroll
      for (int c = 0; c < 16; ++c) lcp[c] = 0.0;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int g = g0 + j;
        if (kFull || k0 + g < n) bad |= !(d > 0.0);
        else d = 1.0;
        const double inv = rsqrt_nr(d);
        const double l = p[j] * inv;  // L(r, g) for r >= g (r == g: sqrt(d))
        p[j] = l;
        T[g * TS + r] = l;
        if (r == 0) scr[0][j] = inv;
        if (j >= 1 && j < 15) {
#pragma unroll
          for (int c = j + 1; c < 16; ++c) p[c] = fma(-lp, lcp[c], p[c]);  // column j - 1
        }
        if (j < 15) {
          // critical path by readlane only: the next pivot (lane g+1's own
          // a - l*l) and the next column's L(g+1, g) for every lane
          const double dn = bcast(fma(-l, l, p[j + 1]), g + 1);
          const double l1 = bcast(l, g + 1);
          p[j + 1] = fma(-l, l1, p[j + 1]);
          if (j < 14) {
#pragma unroll
            for (int c = j + 2; c < 16; ++c) lcp[c] = T[g * TS + g0 + c];
          }
          lp = l;
          d = dn;
        }
      }
    } else if (b == 0) {
      if (Ls != nullptr) {
        // deferred last update: wave 1 blocks (1,1) (2,2), wave 2 (2,1) (3,2),
        // wave 3 (3,1) (3,3)  [(I, J)]
        const int Ib[2] = {w, w + 1 < 4 ? w + 1 : 3}, Jb[2] = {1, w == 1 ? 2 : (w == 2 ? 2 : 3)};
        last_update<2>(T, Ls, Ib, Jb, 2, lane);
      }
    } else if (b == 1) {
      // panel 0's trailing update of blocks (2,2) (3,2) (3,3) [waves 1, 2, 3]
      trail_block(T, 0, w == 1 ? 2 : 3, w == 3 ? 3 : 2, lane);
      if (w == 2) trtri16(T, Wl, scr[0], lane);  // W_00 (read by wave 1 in panel 2)
    } else if (w == 1) {
      w_offdiag(T, Wl, scr[w], 1, 0, lane);  // row 1 of W (its diagonal block is done)
    } else if (w == 3) {
      trail_block(T, 16, 3, 3, lane);  // panel 1's trailing update of block (3,3)
    } else if (pf_sub != nullptr) {  // (b == 2, wave 2)
      // a second poll ~0.55 us later when the first misses: the tile is out
      // ~5.4 us into the step, panel 2 starts at ~5.1 us (stamped), and a
      // poll's round trip (~1 us) still ends within the panel (1.8 us)
      bool f = __hip_atomic_load(pf_sub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
      if (!__builtin_amdgcn_readfirstlane(int(f))) {
        __builtin_amdgcn_s_sleep(20);
        f = __hip_atomic_load(pf_sub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
      }
      rdy[0] = f;
    }
    __syncthreads();
    WSTAMP(k0 / NB, 2 + b);
    // ---- trailing update of column block b+1 (the next panel's); the
    // blocks right of it follow during the next panel (look-ahead) ----
    if (w < 3 - b) trail_block(T, g0, b + 1 + w, b + 1, lane);
    // (b = 2: a third poll of the subdiagonal partial tile by idle wave 2)
    if (b == 2 && w == 2 && pf_sub != nullptr && __builtin_amdgcn_readfirstlane(rdy[0]) == 0)
      rdy[0] = __hip_atomic_load(pf_sub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
    __syncthreads();
    WSTAMP(k0 / NB, 6 + b);
  }
  // ---- panel 3 (peeled) ----
  if (w == 0) {
    panel_w0<kFull>(T, Wl, 48, k0, n, lane, bad);
    PSTAMP(k0 / NB, 0);
  } else {
    // the walker's next partial tiles: the diagonal tile's poll, then the
    // prefetch's loads go out first (the poll ahead of them: vmcnt is one
    // in-order counter, so its value waits only for itself), its result is
    // written at the end
    int dflag = 0;
    if (w == 3 && pf_diag != nullptr) dflag = __hip_atomic_load(pf_diag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (pf_sub != nullptr) {
      if (__builtin_amdgcn_readfirstlane(rdy[0]) != 0) {
        pre.load();
      } else if (__hip_atomic_load(pf_sub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch) {
        // missed by the earlier polls: each wave polls once more and loads its
        // share; the prefetch counts only if all three saw the tile (bits in
        // rdy[3]; otherwise the walker reloads it whole)
        pre.load();
        if (lane == 0) __hip_atomic_fetch_or(&rdy[3], 1 << w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    // row 2 of W, then the sums of row 3 (wave w: column block J = w - 1).
    // W_20 is formed by wave 3 (its own row-3 sum is one product) and handed
    // to wave 1 by an LDS flag: wave 1 forms its sum's K = 0, 1 products
    // meanwhile and adds K = 2 last, as the chain always did (bitwise the
    // same W; wave 1 carried 6 of the panel's 11 16x16x16 products and ended
    // after wave 0, stamped)
    if (w == 3) {
      w_offdiag(T, Wl, scr[3], 2, 0, lane);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) __hip_atomic_store(&rdy[2], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      w_row3_sum(T, Wl, scr[3], 2, lane);
    } else if (w == 2) {
      w_offdiag(T, Wl, scr[2], 2, 1, lane);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      w_row3_sum(T, Wl, scr[2], 1, lane);
    } else {
      f64x4 acc = {0.0, 0.0, 0.0, 0.0};
      acc = mfma16(T + 48, 1, TS, Wl, 1, TS, acc, lane);
      acc = mfma16(T + 16 * TS + 48, 1, TS, Wl + 16, 1, TS, acc, lane);
      while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&rdy[2], __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_WORKGROUP)) == 0)
        __builtin_amdgcn_s_sleep(1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      acc = mfma16(T + 32 * TS + 48, 1, TS, Wl + 32, 1, TS, acc, lane);
      const int j = lane & 15, kk = lane >> 4;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) scr[1][(4 * rr + kk) * 16 + j] = acc[rr];
    }
    if (w == 3 && pf_diag != nullptr) rdy[1] = dflag == epoch;
    PSTAMP(k0 / NB, w);
  }
  __syncthreads();
  WSTAMP(k0 / NB, 5);
  // ---- W row 3 off the diagonal: the products with W_33 ----
  // (wave 0, idle here: the stores of W rows 0-2, final since panel 3)
  if (w >= 1) w_row3_finish(Wl, scr[w], w - 1, lane);
  else pre.w_early(Wl, lane);
  __syncthreads();
  WSTAMP(k0 / NB, 9);
  return bad;
}

// ---------------------------------------------------------------------------
// The whole factorisation in ONE persistent launch (left-looking tiles,
// device-scope flags instead of kernel boundaries).
//
// Workgroup 0 walks the diagonal -- the critical path -- and never waits for
// a launch: for j = 0, 1, ...
//   T_jj (updated by the helpers for k <= j-2)  -= L_j,j-1 L_j,j-1^T
//   POTRF -> L_jj, W_j = L_jj^-1
//   L_j+1,j = T_j+1,j W_j^T  (kept in LDS for the next update)
// Every other workgroup is a helper that takes tiles (i, j), column-major,
// from an atomic ticket and accumulates T_ij = A_ij - sum_k L_ik L_jk^T in
// MFMA registers as the L columns become final (flags F).  Tiles (j, j)
// (one update short) and (j+1, j) hand the partial tile to the walker
// (flag P); every other tile finishes with its TRSM against W_j (F(j,j)).
// Tickets are taken in an order in which every dependency was taken
// earlier, and roles go by start order (the walker is the first workgroup
// to run, a helper takes tasks only once running), so every awaited tile
// belongs to a running workgroup and the waits drain whatever the residency;
// every wait is bounded anyway (a timeout sets fail bit value 4; the back
// substitution's own timeout sets 2).
// Polls are relaxed agent-scope atomic loads (coherent across the XCDs'
// L2s); the acquire fence comes once, after the flag is seen.  (An acquire
// load per poll would invalidate the poller's L2 on every spin.)
constexpr long kFlagSpins = 1L << 20;

__device__ __forceinline__ bool spin_until(const int* f, int epoch) {
  long spins = 0;
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
    if (++spins > kFlagSpins) return false;
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// Branches around barriers are kept SCALAR: "this is wave 0" is tested on
// readfirstlane(threadIdx.x) (an SGPR), and everything inside runs on all 64
// lanes (same flag, same value).  A per-lane `if (threadIdx.x == 0)` inside a
// loop that also holds barriers lets the compiler split the loop by lane
// masks, so that lanes 1..63 of wave 0 pass the barrier without lane 0
// (seen on gfx950: a hang on a stale ticket).
__device__ __forceinline__ bool wave0() { return __builtin_amdgcn_readfirstlane(threadIdx.x) < 64; }

// Wave 0 waits for one flag, then the block proceeds (acquire by wave 0; the
// barrier orders the other waves' loads after it).
__device__ __forceinline__ void block_wait(const int* f, int epoch, int* fail) {
  if (wave0()) {
    if (!spin_until(f, epoch)) atomicOr(fail, 4);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the invalidate completes asynchronously
  }
  __syncthreads();
}

// Write-through publication (MI355X_MICROARCH.md: a producer that stores
// every handed-off byte sc1 and drains every wave before the flag needs no
// agent release; the consumers keep their acquire): every tile the walker
// and the helpers hand off, so no publication pays an L2 write-back (the
// release form, buffer_wbl2 + drain, wrote back the XCD's whole L2).
__device__ __forceinline__ void st_wt(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void block_publish_wt(int* f, int epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (wave0()) __hip_atomic_store(f, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave 0 finds how many of k = k_from.. (<= K) have both F(i,k) and F(j,k)
// final (waiting until at least one has); the block gets the new bound.
__device__ __forceinline__ int ready_bound(const int* F, int nb, int i, int j, int k_from, int K, int epoch,
                                           int* sh, int* fail, int i2 = -1) {
  if (wave0()) {
    const int lane = threadIdx.x;
    long spins = 0;
    int bound = k_from;
    while (true) {
      const int k = k_from + lane;
      bool ok = true;
      if (k <= K)
        ok = __hip_atomic_load(F + i * nb + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch &&
             __hip_atomic_load(F + j * nb + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch &&
             (i2 < 0 || __hip_atomic_load(F + i2 * nb + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch);
      const unsigned long long miss = __ballot(!ok);
      const int run = miss ? __builtin_ctzll(miss) : 64;
      bound = k_from + run;
      if (run > 0 || ++spins > kFlagSpins) break;
      __builtin_amdgcn_s_sleep(1);
    }
    if (bound == k_from) {  // timed out: proceed (garbage), reported as an error
      atomicOr(fail, 4);
      bound = k_from + 1;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the invalidate completes asynchronously
    *sh = bound > K + 1 ? K + 1 : bound;  // every lane: the same value
  }
  __syncthreads();
  // readfirstlane: the bound steers a loop with barriers in it, so it must be
  // a scalar (uniform) value, never an exec-mask (per-lane) loop exit
  const int b = __builtin_amdgcn_readfirstlane(*sh);
  __syncthreads();
  return b;
}

// Schur / Cholesky overlap (DevProblem::tile_cnt): tile (i, j) of S is
// complete once k_schur_pts has counted every camera block of it in.  Its
// blocks are stored write-through and drained before each count, so wave 0
// polls the count (relaxed), then acquires as after a flag.
__device__ __forceinline__ bool tile_ready_poll(const int* cnt, int exp, int* sh) {
  if (wave0()) {
    const bool r = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= exp;
    if (r) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    sh[1] = r ? 1 : 0;
  }
  __syncthreads();
  const int r = __builtin_amdgcn_readfirstlane(sh[1]);
  __syncthreads();
  return r != 0;
}
__device__ __forceinline__ void tile_wait(const int* cnt, int exp, int* fail) {
  if (wave0()) {
    long spins = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < exp) {
      if (++spins > kFlagSpins) {
        atomicOr(fail, 4);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// The helpers' TRSM X = T W^T for U stacked tiles (T_u in LDS, W = L_jj^-1
// lower triangular in global memory, column-major: W(c, m) at m*NB + c).
// Wave w takes row block w of every tile and forms X^T (column block C) =
// sum_{M <= C} W_CM T_wM^T on MFMA: 40 MFMAs per tile instead of 64 (the
// products with W's zero upper blocks are skipped; they came last in the
// k order, so the sums are bitwise the full ones), the W operand shared by
// the U tiles.  x[u][C] reg rr holds X(16w + (lane & 15), 16C + 4rr + (lane >> 4)).
template <int U>
__device__ __forceinline__ void trsm_rows(const double* const* Tp, const double* __restrict__ Wk, f64x4 (*x)[4],
                                          int lane) {
  const int w = threadIdx.x >> 6, li = lane & 15, kk = lane >> 4;
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int C = 0; C < 4; ++C) x[u][C] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const int k = 16 * M + 4 * s4 + kk;
      double bt[U];
#pragma unroll
      for (int u = 0; u < U; ++u) bt[u] = Tp[u][k * TS + 16 * w + li];
#pragma unroll
      for (int C = M; C < 4; ++C) {
        const double a = Wk[k * NB + 16 * C + li];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u][C] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bt[u], x[u][C], 0, 0, 0);
      }
    }
}
// Write-through stores of trsm_rows' tiles to rows i0 + 64u.. of column
// block j0 (16 lanes per 128-B column run).
template <int U>
__device__ __forceinline__ void put_rows(double* __restrict__ A, int ld, int i0, int j0, const f64x4 (*x)[4], int lane) {
  const int w = threadIdx.x >> 6, li = lane & 15, kk = lane >> 4;
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int C = 0; C < 4; ++C)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        st_wt(A + size_t(j0 + 16 * C + 4 * rr + kk) * ld + i0 + NB * u + 16 * w + li, x[u][C][rr]);
}

// Helper: one tile (i, j).  Wave w owns the 32x32 quadrant (c in cb.., r in
// rb..), accumulated transposed: D[c][r] = sum_l L_jk[c][l] L_ik[r][l], so the MFMA's D
// column (lane & 15) walks the tile's rows (128-B column runs of A).
__device__ __forceinline__ void fused_helper_tile(double* __restrict__ A, int ld, int nb, const double* __restrict__ Winv,
                                  int* __restrict__ F, int* __restrict__ Pf, int epoch, int i, int j, double* T,
                                  int* sh, int* __restrict__ fail, const int* __restrict__ tile_cnt,
                                  const int* __restrict__ tile_exp) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int cb = 32 * (w >> 1), rb = 32 * (w & 1);
  const int lr = lane & 15, lk = lane >> 4;
  const int i0 = i * NB, j0 = j * NB;
  const bool diag = i == j;
  const bool skipq = diag && cb > rb;        // strictly upper quadrant: never read
  const int K = diag ? j - 2 : j - 1;        // updates k = 0..K by the helper
  // S tile (i, j): read here, or (overlapped with the Schur pass and not yet
  // complete) after the updates
  const bool early = tile_cnt == nullptr || tile_ready_poll(tile_cnt + i * nb + j, tile_exp[i * nb + j], sh);
  double cv[2][2][4];
  if (early) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int bb = 0; bb < 2; ++bb)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg)
          cv[a][bb][reg] = skipq ? 0.0 : A[size_t(j0 + cb + 16 * a + lk + 4 * reg) * ld + i0 + rb + 16 * bb + lr];
  }
  f64x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) acc[a][bb] = f64x4{0.0, 0.0, 0.0, 0.0};
  int kr = 0;  // k < kr are known final
  for (int k = 0; k <= K; ++k) {
    if (k >= kr) kr = ready_bound(F, nb, i, j, k, K, epoch, sh, fail);
    if (skipq) continue;  // wave-uniform; no barrier below in this iteration
    const int k0 = k * NB;
    double xa[2][16], yb[2][16];
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const size_t colbase = size_t(k0 + 4 * ks + lk) * ld;
#pragma unroll
      for (int a = 0; a < 2; ++a) xa[a][ks] = A[colbase + j0 + cb + 16 * a + lr];
#pragma unroll
      for (int bb = 0; bb < 2; ++bb) yb[bb][ks] = A[colbase + i0 + rb + 16 * bb + lr];
    }
#pragma unroll
    for (int ks = 0; ks < 16; ++ks)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int bb = 0; bb < 2; ++bb)
          acc[a][bb] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[a][ks], yb[bb][ks], acc[a][bb], 0, 0, 0);
  }
  if (!early) {
    tile_wait(tile_cnt + i * nb + j, tile_exp[i * nb + j], fail);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int bb = 0; bb < 2; ++bb)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg)
          cv[a][bb][reg] = skipq ? 0.0 : A[size_t(j0 + cb + 16 * a + lk + 4 * reg) * ld + i0 + rb + 16 * bb + lr];
  }
  if (i <= j + 1) {
    // partial tile for the diagonal walker (its diagonal update / TRSM)
    if (K >= 0 && !skipq) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int bb = 0; bb < 2; ++bb)
#pragma unroll
          for (int reg = 0; reg < 4; ++reg)
            st_wt(A + size_t(j0 + cb + 16 * a + lk + 4 * reg) * ld + i0 + rb + 16 * bb + lr, cv[a][bb][reg] - acc[a][bb][reg]);
    }
    block_publish_wt(Pf + i * nb + j, epoch);
    HSTAMP(i, j, 0);
    return;
  }
  // final tile: T -> LDS, then X = T W_j^T on MFMA once W_j is out
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int bb = 0; bb < 2; ++bb)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg)
        T[(cb + 16 * a + lk + 4 * reg) * TS + rb + 16 * bb + lr] = cv[a][bb][reg] - acc[a][bb][reg];
  block_wait(F + j * nb + j, epoch, fail);  // (its barrier also closes the LDS writes)
  const double* Wk = Winv + size_t(j) * NB * NB;
  const double* Tp[1] = {T};
  f64x4 x[1][4];
  trsm_rows<1>(Tp, Wk, x, lane);
  put_rows<1>(A, ld, i0, j0, x, lane);
  block_publish_wt(F + i * nb + j, epoch);
  HSTAMP(i, j, 1);
}

// Helper: the vertical pair of final tiles (i, j), (i+1, j) (i >= j + 2).
// Both share the L_jk operand of every update step, so a step loads three
// panel tiles for two tile updates (four as single tiles): at n = 12000 the
// helpers, 62% MFMA-busy, fetch 43.7 GB per factor re-reading panels.  Each
// tile's update order (k, then ks) is the single-tile form's, so the factor
// is bitwise unchanged.  A's values of the two tiles are read at the end
// (nobody else writes them before this task publishes).
__device__ __forceinline__ void fused_helper_pair(double* __restrict__ A, int ld, int nb,
                                                  const double* __restrict__ Winv, int* __restrict__ F, int epoch,
                                                  int i, int j, double* T0, double* T1, int* sh,
                                                  int* __restrict__ fail, const int* __restrict__ tile_cnt,
                                                  const int* __restrict__ tile_exp) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int cb = 32 * (w >> 1), rb = 32 * (w & 1);
  const int lr = lane & 15, lk = lane >> 4;
  const int i0 = i * NB, i1 = i0 + NB, j0 = j * NB;
  const int K = j - 1;
  f64x4 acc[2][2][2];  // [tile][a][bb]
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int bb = 0; bb < 2; ++bb) acc[u][a][bb] = f64x4{0.0, 0.0, 0.0, 0.0};
  int kr = 0;
  for (int k = 0; k <= K; ++k) {
    if (k >= kr) kr = ready_bound(F, nb, i, j, k, K, epoch, sh, fail, i + 1);
    const int k0 = k * NB;
    double xa[2][16], yb[2][2][16];
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const size_t colbase = size_t(k0 + 4 * ks + lk) * ld;
#pragma unroll
      for (int a = 0; a < 2; ++a) xa[a][ks] = A[colbase + j0 + cb + 16 * a + lr];
#pragma unroll
      for (int bb = 0; bb < 2; ++bb) {
        yb[0][bb][ks] = A[colbase + i0 + rb + 16 * bb + lr];
        yb[1][bb][ks] = A[colbase + i1 + rb + 16 * bb + lr];
      }
    }
#pragma unroll
    for (int ks = 0; ks < 16; ++ks)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int bb = 0; bb < 2; ++bb)
            acc[u][a][bb] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[a][ks], yb[u][bb][ks], acc[u][a][bb], 0, 0, 0);
  }
  if (tile_cnt) {  // overlapped with the Schur pass: both S tiles complete
    tile_wait(tile_cnt + i * nb + j, tile_exp[i * nb + j], fail);
    tile_wait(tile_cnt + (i + 1) * nb + j, tile_exp[(i + 1) * nb + j], fail);
  }
  // T_u = A - acc -> LDS
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    double* Tu = u ? T1 : T0;
    const int iu = u ? i1 : i0;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int bb = 0; bb < 2; ++bb)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const int c = cb + 16 * a + lk + 4 * reg, r = rb + 16 * bb + lr;
          Tu[c * TS + r] = A[size_t(j0 + c) * ld + iu + r] - acc[u][a][bb][reg];
        }
  }
  block_wait(F + j * nb + j, epoch, fail);  // (its barrier also closes the LDS writes)
  const double* Wk = Winv + size_t(j) * NB * NB;
  const double* Tp[2] = {T0, T1};
  f64x4 x[2][4];
  trsm_rows<2>(Tp, Wk, x, lane);
  put_rows<2>(A, ld, i0, j0, x, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (wave0()) {
    __hip_atomic_store(F + i * nb + j, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(F + (i + 1) * nb + j, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  HSTAMP(i, j, 1);
  HSTAMP(i + 1, j, 1);
}

// Helper tasks of column j: the diagonal tile, the subdiagonal tile (both
// partial, for the walker), the first final tile (j+2, j) alone (it feeds
// the walker two steps ahead, so its TRSM is on the chain), then the
// vertical pairs of final tiles (a last single tile when the count is odd).
__host__ __device__ __forceinline__ int col_tasks(int nb, int j) {
  const int m = nb - j;
  return m <= 2 ? m : 3 + (m - 3) / 2 + ((m - 3) & 1);
}
// (ncols < nb: a column panel -- the first ncols tile columns of an nb-row
// trailing matrix, finished as L; the tiles right of it are not touched)
__host__ __device__ __forceinline__ int chol_tasks(int nb, int ncols) {
  int s = 0;
  for (int j = 0; j < ncols; ++j) s += col_tasks(nb, j);
  return s;
}

// X = T W^T for one 64x64 tile (T and W in LDS, W lower triangular): wave w
// gets row block w, x[Cb] = block (w, Cb) in the mfma16 D layout.
// The four column blocks' MFMA chains are interleaved (same k order per
// block: bitwise the chained sums).
__device__ __forceinline__ void trsm_lds(const double* T, const double* Wl, f64x4 x[4], int lane) {
  const int w = threadIdx.x >> 6, li = lane & 15, kk = lane >> 4;
#pragma unroll
  for (int Cb = 0; Cb < 4; ++Cb) x[Cb] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int M = 0; M < 4; ++M) {
    // the column block's operands first, then its MFMAs (same order per x[Cb])
    double a[4], b[4][4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const int k = 16 * M + 4 * s4 + kk;
      a[s4] = T[k * TS + 16 * w + li];
#pragma unroll
      for (int Cb = M; Cb < 4; ++Cb) b[s4][Cb] = Wl[k * TS + 16 * Cb + li];
    }
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      asm volatile("" : "+v"(a[s4]));
#pragma unroll
      for (int Cb = M; Cb < 4; ++Cb) asm volatile("" : "+v"(b[s4][Cb]));
    }
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int Cb = M; Cb < 4; ++Cb) x[Cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s4], b[s4][Cb], x[Cb], 0, 0, 0);
  }
}
__device__ __forceinline__ void put_tile(double* D, const f64x4 x[4], int lane) {
  const int w = threadIdx.x >> 6, li = lane & 15, kk = lane >> 4;
#pragma unroll
  for (int Cb = 0; Cb < 4; ++Cb)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) D[(16 * Cb + li) * TS + 16 * w + 4 * rr + kk] = x[Cb][rr];
}
__device__ __forceinline__ void load_tile(double* D, const double* __restrict__ A, int ld, int i0, int j0) {
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = threadIdx.x + 256 * q, c = e >> 6, r = e & 63;
    D[c * TS + r] = A[size_t(j0 + c) * ld + i0 + r];
  }
}
__device__ __forceinline__ void store_tile(double* __restrict__ A, int ld, int i0, int j0, const double* D) {
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = threadIdx.x + 256 * q, c = e >> 6, r = e & 63;
    A[size_t(j0 + c) * ld + i0 + r] = D[c * TS + r];
  }
}

// The diagonal walker.  Step j: T_jj -= L_j,j-1 L_j,j-1^T, POTRF (L_jj, W_j),
// TRSM of the subdiagonal tile L_j+1,j (kept in LDS for the next update).
// The partial tiles the walker takes from the helpers -- (j+1, j) for the
// TRSM, (j+1, j+1) for the next step -- were stored sc1 and published behind
// a drain, so the walker reads them with sc1 loads after a relaxed poll and a
// barrier, with no agent acquire (MI355X_MICROARCH.md "Valid forms", row 1:
// the acquire's L1 invalidate + wait cost ~1.7 us on the chain).  Tile
// (j+1, j) is prefetched to registers during panel 3 of the POTRF when wave
// 2's poll in panel 2 found it out (potrf_tile); tile (j+1, j+1) is loaded
// after F(j,j)'s publication, its latency under the TRSM and the stores of
// L_j+1,j.  Those stores drain during the next step's first update, and their
// flag goes out after it.
// (Also taking L_j+2,j here, to shorten the helpers' chain W_j -> L_j+2,j ->
// last update of T_j+2,j+2, measured no better: the extra TRSM costs what
// the saved hand-off gains.)
// threadIdx.x through an opaque move: the per-lane offsets derived from it
// are computed where they are used.  (The walker's loop holds every value
// the compiler can hoist out of it in registers -- at 512 VGPR + AGPR per
// lane a hoisted set of 16-22 addresses spills to scratch, and a scratch
// reload waits vmcnt(0), i.e. for every load in flight.)
__device__ __forceinline__ int tid_local() {
  int v;
  asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "v"(int(threadIdx.x)));
  return v;
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Wave 0 polls one flag (relaxed, sc1), the block proceeds after the barrier;
// no acquire: every load of the awaited bytes is ld_sc1.
__device__ __forceinline__ void block_wait_sc1(const int* f, int epoch, int* fail) {
  if (wave0()) {
    if (!spin_until(f, epoch)) atomicOr(fail, 4);
  }
  __syncthreads();
}
// Waves 1-3 prefetch a 64x64 tile (column-major at src, leading dimension
// ld) into the LDS image D: 22 sc1 loads per lane (192 lanes, one 512-B
// column per wave instruction), then the LDS writes.
// 16-B sc1 loads of a handed-off tile (buffer_load_dwordx4 sc1: aux bit 4;
// 16-B sc1 loads of 8-B sc1-stored bytes are row 1 of the "Valid forms"
// table): half the load instructions of 8-B loads -- the walker's tile loads
// are issue-bound beside its MFMA work.
typedef double d2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const double* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ d2v ld2_sc1(__amdgpu_buffer_rsrc_t rs, uint32_t byte_off) {
  return __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, 16));
}
// Waves 1-3 prefetch a 64x64 tile (column-major at src, leading dimension
// ld) into the LDS image D: 11 16-B loads per lane (192 lanes; pair e =
// u + 192 q, u = t - 64, is column (u >> 5) + 6 q, rows 2 (u & 31) and + 1: two
// 512-B columns per wave instruction), the LDS writes later (store()).  The
// offsets run through an opaque register at every step: hoisted out of the
// walker's loop, the per-lane addresses held 44 registers across the whole
// walk (140 VGPRs spilled, each reload a vmcnt(0) wait).
__device__ __forceinline__ void w_st_rows012(double* dst, const double* Wl, int lane);
struct SubPrefetch {
  const double* src;
  int ld;
  double* D;
  double* wdst;  // W_j's home (its rows 0-2 go out from potrf_tile's end)
  d2v v[11];
  __device__ __forceinline__ void w_early(const double* Wl, int lane) { w_st_rows012(wdst, Wl, lane); }
  __device__ __forceinline__ void load() {
    const int u = tid_local() - 64;
    const __amdgpu_buffer_rsrc_t rs = tile_rsrc(src);
    uint32_t off = uint32_t(((u >> 5) * ld + 2 * (u & 31)) * 8);
    const uint32_t step = uint32_t(6 * ld * 8);
#pragma unroll
    for (int q = 0; q < 11; ++q) {
      asm volatile("" : "+v"(off));
      if (q < 10 || u < 128) v[q] = ld2_sc1(rs, off);
      off += step;
    }
  }
  __device__ __forceinline__ void store() {
    const int u = tid_local() - 64;
    int off = (u >> 5) * TS + 2 * (u & 31);
#pragma unroll
    for (int q = 0; q < 11; ++q) {
      asm volatile("" : "+v"(off));
      if (q < 10 || u < 128) {
        D[off] = v[q].x;
        D[off + 1] = v[q].y;
      }
      off += 6 * TS;
    }
  }
};
// The walker's whole-tile loads, 256 lanes, 8 16-B loads per lane: pair
// e = t + 256 q is column (t >> 5) + 8 q, rows 2 (t & 31) and + 1; and the
// matching LDS writes.
__device__ __forceinline__ void tile_ld2_sc1(d2v (&v)[8], const double* src, int ld) {
  const int t = tid_local();
  const __amdgpu_buffer_rsrc_t rs = tile_rsrc(src);
  uint32_t off = uint32_t(((t >> 5) * ld + 2 * (t & 31)) * 8);
  const uint32_t step = uint32_t(8 * ld * 8);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    asm volatile("" : "+v"(off));
    v[q] = ld2_sc1(rs, off);
    off += step;
  }
}
__device__ __forceinline__ void tile_put2(double* D, const d2v (&v)[8]) {
  const int t = tid_local();
  int off = (t >> 5) * TS + 2 * (t & 31);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    asm volatile("" : "+v"(off));
    D[off] = v[q].x;
    D[off + 1] = v[q].y;
    off += 8 * TS;
  }
}
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st2_sc1(__amdgpu_buffer_rsrc_t rs, uint32_t byte_off, d2v v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, byte_off, 0, 16);
}
// A 64x64 LDS image D -> the tile at dst (leading dimension ld), write-through
// 16-B sc1 stores; pair e = t + 256 q as tile_ld2_sc1.  Every LDS read is
// issued before the first store: one wait instead of one LDS round trip per
// store (the element-wise form compiled to 16 ds_read -> wait -> store
// sequences, 0.6 us per tile; the W_j publication with its lower-block mask
// 1.1 us, both on the walker's chain).  kLowerBlocks: only the 16x16 blocks
// on or below the diagonal (W_k; its upper blocks stay zero from set_problem).
template <bool kLowerBlocks>
__device__ __forceinline__ void tile_st2_wt(double* dst, int ld, const double* D) {
  const int t = tid_local();
  d2v v[8];
  int lo = (t >> 5) * TS + 2 * (t & 31);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    v[q].x = D[lo + 8 * TS * q];
    v[q].y = D[lo + 8 * TS * q + 1];
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) asm volatile("" : "+v"(v[q]));  // all reads land before the stores start
  const __amdgpu_buffer_rsrc_t rs = tile_rsrc(dst);
  uint32_t off = uint32_t(((t >> 5) * ld + 2 * (t & 31)) * 8);
  const uint32_t step = uint32_t(8 * ld * 8);
  const int r16 = (2 * (t & 31)) >> 4;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    asm volatile("" : "+v"(off));
    const int c16 = ((t >> 5) + 8 * q) >> 4;
    if (!kLowerBlocks || r16 >= c16) st2_sc1(rs, off, v[q]);
    off += step;
  }
}
// W_j = Wl (lower 16x16 blocks) -> dst (ld NB), in two parts: blocks (I, J)
// of rows 0-2 by one wavefront (pair e = lane + 64 h of block q: column
// 16 J + (e >> 3), rows 16 I + 2 (e & 7) and + 1; 128-B column runs), row 3
// by the block (pair e = t + 256 h: column e >> 3, rows 48 + 2 (e & 7)).
__device__ __forceinline__ void w_st_rows012(double* dst, const double* Wl, int lane) {
  constexpr int BI[6] = {0, 1, 2, 1, 2, 2}, BJ[6] = {0, 0, 0, 1, 1, 2};
  d2v v[12];
  const int cl = lane >> 3, rl = 2 * (lane & 7);
#pragma unroll
  for (int q = 0; q < 12; ++q) {
    const int c = 16 * BJ[q >> 1] + 8 * (q & 1) + cl, r = 16 * BI[q >> 1] + rl;
    v[q].x = Wl[c * TS + r];
    v[q].y = Wl[c * TS + r + 1];
  }
#pragma unroll
  for (int q = 0; q < 12; ++q) asm volatile("" : "+v"(v[q]));
  const __amdgpu_buffer_rsrc_t rs = tile_rsrc(dst);
  const uint32_t off0 = uint32_t((cl * NB + rl) * 8);
#pragma unroll
  for (int q = 0; q < 12; ++q) {
    uint32_t off = off0 + uint32_t(((16 * BJ[q >> 1] + 8 * (q & 1)) * NB + 16 * BI[q >> 1]) * 8);
    asm volatile("" : "+v"(off));
    st2_sc1(rs, off, v[q]);
  }
}
__device__ __forceinline__ void w_st_row3(double* dst, const double* Wl) {
  const int t = tid_local();
  d2v v[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int e = t + 256 * h, c = e >> 3, r = 48 + 2 * (e & 7);
    v[h].x = Wl[c * TS + r];
    v[h].y = Wl[c * TS + r + 1];
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) asm volatile("" : "+v"(v[h]));
  const __amdgpu_buffer_rsrc_t rs = tile_rsrc(dst);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int e = t + 256 * h;
    uint32_t off = uint32_t(((e >> 3) * NB + 48 + 2 * (e & 7)) * 8);
    asm volatile("" : "+v"(off));
    st2_sc1(rs, off, v[h]);
  }
}

template <bool kPanel>  // a column panel (ncols < nb possible) or the whole factor (ncols == nb)
__device__ __forceinline__ void fused_walker(double* __restrict__ A, int ld, int n, int nb, int ncols,
                             double* __restrict__ Winv,
                             int* __restrict__ F, const int* __restrict__ Pf, int epoch, double* T, double* Wl,
                             double* Ls, double* Tn, double (*scr)[256], int* rdy, int* __restrict__ fail) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // the next diagonal tile travels in registers (loaded one step ahead)
  d2v nx[8];
  // the last update of the next diagonal tile's column block 0 (block (w, 0)),
  // formed at the end of the previous step
  f64x4 g0acc[1];
  g0acc[0] = f64x4{0.0, 0.0, 0.0, 0.0};
  block_wait_sc1(Pf, epoch, fail);
  tile_ld2_sc1(nx, A, ld);
  for (int j = 0; j < (kPanel ? ncols : nb); ++j) {
    const int j0 = j * NB;
    WSTAMP(j, 0);
    tile_put2(T, nx);
    if (t == 0) rdy[0] = rdy[1] = 0;
    __syncthreads();
    if (j > 0) {
      // T -= L_j,j-1 L_j,j-1^T on column block 0 (wave w: block (w, 0); its
      // products were formed at the end of the last step); the blocks right
      // of it are updated inside potrf_tile, during panel 0
      const int Ib[1] = {w}, Jb[1] = {0};
      last_update_apply<1>(T, Ib, Jb, 1, lane, g0acc);
      // L_j,j-1 (stored at the end of the last step) has drained: its flag
      block_publish_wt(F + j * nb + j - 1, epoch);
    }
    WSTAMP(j, 1);
    const double* dl = j > 0 ? Ls : nullptr;  // the rest of the last update
    const bool more = j + 1 < nb;      // a tile below the diagonal
    const bool next = kPanel ? j + 1 < ncols : more;  // ... and the walker's next diagonal tile (a panel ends before it)
    const int i0 = j0 + NB;
    const int* fsub = more ? Pf + (j + 1) * nb + j : nullptr;
    // the subdiagonal partial tile, prefetched into Tn during panel 3
    SubPrefetch pre{A + size_t(j0) * ld + i0, ld, Tn, Winv + size_t(j) * NB * NB};
    const int* fdiag = next ? Pf + (j + 1) * nb + j + 1 : nullptr;
    const bool bad = (j0 + NB <= n) ? potrf_tile<true>(T, Wl, scr, j0, n, dl, fsub, fdiag, epoch, rdy, pre)
                                    : potrf_tile<false>(T, Wl, scr, j0, n, dl, fsub, fdiag, epoch, rdy, pre);
    if (bad) atomicOr(fail, 1);
    const bool early = more && (__builtin_amdgcn_readfirstlane(rdy[0]) != 0 || __builtin_amdgcn_readfirstlane(rdy[3]) == 14);
    const bool diag_out = next && __builtin_amdgcn_readfirstlane(rdy[1]) != 0;
    // the prefetched subdiagonal tile into Tn (waves 1-3)
    if (early && w >= 1) pre.store();
    WSTAMPV(j, 15, early ? 1ull : 0ull);
    // W_j: lower 16x16 blocks only (the upper blocks of every W_k stay zero
    // from set_problem, one memset: 37% fewer bytes on the chain); rows 0-2
    // went out from the POTRF's last phase (wave 0), row 3 here
    w_st_row3(Winv + size_t(j) * NB * NB, Wl);
    WSTAMP(j, 10);
    WSTAMP(j, 11);
    if (!more) {
      block_publish_wt(F + j * nb + j, epoch);
      // L_jj is read by nobody (the helpers' TRSMs and the back substitution
      // use W_j; the next Schur pass rewrites the lower triangle) except in
      // the tile that holds the augmented row n -- the last one: its z
      // entries feed k_backsolve (the kernel's end drains the stores).
      if (j0 <= n && n < j0 + NB) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int e = t + 256 * q, c = e >> 6, r = e & 63;
          st_wt(A + size_t(j0 + c) * ld + j0 + r, T[c * TS + r]);
        }
      }
      break;
    }
    if (!early) {
      // the poll missed: wait for the subdiagonal partial tile here
      block_wait_sc1(fsub, epoch, fail);
      d2v sv[8];
      tile_ld2_sc1(sv, A + size_t(j0) * ld + i0, ld);
      tile_put2(Tn, sv);
    }
    if (next) {
      // the next diagonal partial tile (out long before; wave 3 saw its flag
      // in panel 3): its loads run under the TRSM and the L_j+1,j stores
      if (!diag_out) block_wait_sc1(fdiag, epoch, fail);
      tile_ld2_sc1(nx, A + size_t(i0) * ld + i0, ld);
    }
    if (!early || !diag_out) __syncthreads();  // (the Tn writes above: before the TRSM reads them)
    WSTAMP(j, 12);
    // subdiagonal tile: L_j+1,j = Tn W^T, kept in Ls for the next update
    f64x4 x[4];
    trsm_lds(Tn, Wl, x, lane);
    put_tile(Ls, x, lane);
    // W_j's flag: its stores drained under the TRSM (the helpers' TRSMs of
    // column j feed the diagonal tiles two steps ahead, which have the slack:
    // P(j+1,j) lands ~4.5 us before the walker needs it)
    block_publish_wt(F + j * nb + j, epoch);
    WSTAMP(j, 13);
    if (next) {
      // the next step's column-block-0 update products (its MFMAs run while
      // the stores below drain)
      const int Ib[1] = {w}, Jb[1] = {0};
      last_update_acc<1>(Ls, Ib, Jb, 1, lane, g0acc);
    }
    tile_st2_wt<false>(A + size_t(j0) * ld + i0, ld, Ls);
    WSTAMP(j, 14);
    if (kPanel && !next) {
      // a panel's last column: L_j+1,j is final (no next step publishes it)
      block_publish_wt(F + (j + 1) * nb + j, epoch);
      break;
    }
  }
}

// ncols < nb: one column panel of a distributed factor (launch_cholesky_panel);
// tepoch: the ticket epoch (the flag epoch `epoch` for a whole factor; 1 for
// a panel, whose tickets are zeroed before its launch -- its task count
// differs from panel to panel)
template <bool kPanel>
__global__ __launch_bounds__(256) void k_chol_fused(double* __restrict__ A, int ld, int n, int nb, int ncols,
                                                    double* __restrict__ Winv, int* __restrict__ F,
                                                    int* __restrict__ Pf, unsigned long long* __restrict__ ticket,
                                                    int epoch, int tepoch, int nhelp, int* __restrict__ fail,
                                                    const int* __restrict__ gate, const int* __restrict__ tile_cnt,
                                                    const int* __restrict__ tile_exp) {
  __shared__ double T[NB * TS];
  __shared__ double Wl[NB * TS];
  __shared__ double Ls[NB * TS];
  __shared__ double Tn[NB * TS];  // the walker's subdiagonal tile (helpers: unused)
  __shared__ double scr[4][256];
  __shared__ int sh[4];
  if (gate && *gate == 0) {
    // device LM loop, phase skipped: the launch still takes its ntask + nhelp
    // tickets and its 1 + nhelp role tickets, so the next epoch's bases stay
    // (epoch - 1) (ntask + nhelp) and (epoch - 1) (1 + nhelp)
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      atomicAdd(ticket, (unsigned long long)(chol_tasks(nb, kPanel ? ncols : nb) + nhelp));
      atomicAdd(ticket + 1, (unsigned long long)(1 + nhelp));
    }
    return;
  }
  // role by start order: the first workgroup to run walks the diagonal, so
  // every tile the walker awaits is owned by a running helper whatever the
  // residency (a grid only partly resident beside other streams' kernels runs
  // slower but finishes)
  if (wave0()) {
    const unsigned long long v = atomicAdd(ticket + 1, threadIdx.x == 0 ? 1ULL : 0ULL);
    const unsigned lo = __builtin_amdgcn_readfirstlane(unsigned(v));
    const unsigned hi = __builtin_amdgcn_readfirstlane(unsigned(v >> 32));
    const unsigned long long te = kPanel ? tepoch : epoch;
    sh[1] = int(((unsigned long long)hi << 32 | lo) - (unsigned long long)(te - 1) * (unsigned long long)(1 + nhelp));
  }
  __syncthreads();
  const int role = __builtin_amdgcn_readfirstlane(sh[1]);
  __syncthreads();
  if (role == 0) {
    fused_walker<kPanel>(A, ld, n, nb, ncols, Winv, F, Pf, epoch, T, Wl, Ls, Tn, scr, sh, fail);
    return;
  }
  const int ntask = chol_tasks(nb, kPanel ? ncols : nb);
  // every launch takes exactly ntask + nhelp tickets (one failing grab per helper)
  const unsigned long long base =
      (unsigned long long)((kPanel ? tepoch : epoch) - 1) * (unsigned long long)(ntask + nhelp);
  while (true) {
    if (wave0()) {
      // one increment per wave (lane 0 adds 1, the others 0); every lane
      // writes lane 0's ticket
      const unsigned long long v = atomicAdd(ticket, threadIdx.x == 0 ? 1ULL : 0ULL);
      const unsigned lo = __builtin_amdgcn_readfirstlane(unsigned(v));
      const unsigned hi = __builtin_amdgcn_readfirstlane(unsigned(v >> 32));
      sh[1] = int(((unsigned long long)hi << 32 | lo) - base);
    }
    __syncthreads();
    // uniform (scalar) loop exit: a per-lane exit lets the compiler split the
    // loop by lane masks around the thread-0 ticket grab (observed: lanes
    // 1..63 re-running the body on a stale ticket, i.e. a hang)
    const int tk = __builtin_amdgcn_readfirstlane(sh[1]);
    __syncthreads();
    if (tk >= ntask) break;
    int j = 0, r = tk;
    while (r >= col_tasks(nb, j)) { r -= col_tasks(nb, j); ++j; }
    if (r < 3) {
      fused_helper_tile(A, ld, nb, Winv, F, Pf, epoch, j + r, j, T, sh, fail, tile_cnt, tile_exp);
    } else {
      const int i = j + 3 + 2 * (r - 3);
      if (i + 1 < nb) fused_helper_pair(A, ld, nb, Winv, F, epoch, i, j, T, Wl, sh, fail, tile_cnt, tile_exp);
      else fused_helper_tile(A, ld, nb, Winv, F, Pf, epoch, i, j, T, sh, fail, tile_cnt, tile_exp);
    }
  }
}

// Back substitution L^T y = z (z = row n of the augmented factor, i.e.
// L^-1 rhs), ONE launch: workgroup b owns block row b (64 unknowns),
//   y_b = W_b^T (z_b - sum_{k>b} L_kb^T y_k),
// and every L_kb tile is prefetched before y_k is awaited.  The entries of
// y are their own flags: y is filled with a signalling-NaN sentinel before
// the launch (arithmetic never yields one), the producer stores each entry
// once, write-through, and a consumer's wave 0 polls the 64 entries of y_k
// (agent-scope loads) until none is the sentinel, then passes them through
// LDS.  Against a flag after the data this drops the producer's drain and
// the consumer's invalidate + reload: one memory round trip per hand-off
// instead of three (127 -> 98 us at n = 3000 for LDS staging alone, see
// DESIGN.md).  Chunked consumption or several blocks per workgroup measured
// slower: whatever runs after the awaited block arrives is on the chain.
// Rows go by start order (the chain's first row to the first workgroup to
// run), so every awaited row belongs to a running workgroup whatever the
// residency; every wait is bounded and a timeout sets bit 1 of *fail (an
// error, never a hang).

__global__ __launch_bounds__(256) void k_backsolve(const double* __restrict__ A, int ld, int n, int nb,
                                                   const double* __restrict__ Winv, double* __restrict__ y,
                                                   int* __restrict__ fail, const int* __restrict__ gate,
                                                   unsigned long long* __restrict__ rticket, int epoch) {
  if (gate && *gate == 0) {  // device LM loop: phase skipped (its row tickets still taken)
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(rticket, (unsigned long long)nb);
    return;
  }
  __shared__ double v[NB];
  __shared__ double yl[2][NB];
  __shared__ int timed_out;
  __shared__ int row;
  // block row by start order: the chain's first row goes to the first
  // workgroup to run, so every row a workgroup awaits belongs to one that
  // is already running (any residency, any dispatch order)
  if (threadIdx.x == 0) row = int(atomicAdd(rticket, 1ULL) - (unsigned long long)(epoch - 1) * (unsigned long long)nb);
  __syncthreads();
  const int b = nb - 1 - __builtin_amdgcn_readfirstlane(row);
  const int k0 = b * NB;
  const int nreal = (n - k0) < NB ? (n - k0) : NB;
  const int t = threadIdx.x, col = t >> 2, seg = t & 3;
  if (t == 0) timed_out = 0;
  // off the chain: z entry and the W_b column segment W(16 seg + i, col)
  const double zc = (seg == 0 && col < nreal) ? A[size_t(k0 + col) * ld + n] : 0.0;
  double wr[16];
  {
    const double* Wr = Winv + size_t(b) * NB * NB + size_t(col) * NB + 16 * seg;
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      const double2 q = *reinterpret_cast<const double2*>(Wr + i);
      wr[i] = q.x;
      wr[i + 1] = q.y;
    }
  }
  __syncthreads();
  double acc = 0.0;
  // column k0 + col, rows 64 k + 16 seg .. +16 of tile (k, b)
  const double* colp = A + size_t(k0 + col) * ld + 16 * seg;
  for (int k = nb - 1; k > b; --k) {
    double lv[16];
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      const double2 q = *reinterpret_cast<const double2*>(colp + size_t(k) * NB + i);
      lv[i] = q.x;
      lv[i + 1] = q.y;
    }
    double* yb = yl[k & 1];  // double-buffered: one barrier per block
    if (wave0()) {  // scalar branch (see block_wait)
      const int lane = threadIdx.x & 63;
      const double* p = y + size_t(k) * NB + lane;
      double yv = 0.0;
      for (long spins = 0;; ++spins) {
        yv = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__builtin_amdgcn_ballot_w64(__builtin_bit_cast(uint64_t, yv) == kYSentinel) == 0) break;
        if (spins > kFlagSpins) {
          timed_out = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      yb[lane] = yv;
      if (k == b + 1) BSTAMP(b, 0);
    }
    __syncthreads();
    if (k == b + 1) BSTAMP(b, 1);
    if (__builtin_amdgcn_readfirstlane(timed_out)) break;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc = fma(lv[i], yb[16 * seg + i], acc);
  }
  // the four row segments of a column sit in adjacent lanes
  acc += __shfl_xor(acc, 1);
  acc += __shfl_xor(acc, 2);
  if (seg == 0) v[col] = (col < nreal) ? zc - acc : 0.0;
  BSTAMP(b, 2);
  __syncthreads();
  BSTAMP(b, 3);
  // y_b[col] = sum_c W(c, col) v[c]: 16 terms per lane in four chains, then
  // the four segments
  double p4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int i = 0; i < 16; ++i) p4[i & 3] = fma(wr[i], v[16 * seg + i], p4[i & 3]);
  double sum = (p4[0] + p4[1]) + (p4[2] + p4[3]);
  sum += __shfl_xor(sum, 1);
  sum += __shfl_xor(sum, 2);
  // write-through (sc1) relaxed store of the final value: the consumers'
  // polls see it when it lands, with nothing to order after it
  if (seg == 0) __hip_atomic_store(y + size_t(k0) + col, col < nreal ? sum : 0.0, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
  BSTAMP(b, 4);
  if (wave0() && timed_out) atomicOr(fail, 2);
}

// Small systems (nblk <= 2: n <= 127, keyframe-sized BAs of up to 21
// cameras): the factorisation AND the back substitution in ONE workgroup,
// no flags, tickets or global round trips.  At nblk <= 2 the persistent
// launch is two walker steps plus its start-up and the back substitution a
// second launch (C1: 37.6 + 4.7 us per step solve, each a few us of work).
// The tile operations and their order are k_chol_fused's walker (the
// helpers' partial tiles are the input tiles: no earlier column exists) and
// k_backsolve's arithmetic: bitwise the same L, W and y.
// With cam != nullptr it also takes k_cam_update's step (C <= 256: that
// launch's single workgroup, the same arithmetic and reductions).
__global__ __launch_bounds__(256) void k_chol_small(const double* __restrict__ A, int ld, int n, int nb,
                                                    double* __restrict__ y, int* __restrict__ fail,
                                                    const int* __restrict__ gate, int C,
                                                    const double* __restrict__ cam,
                                                    const double* __restrict__ scale_c, double* __restrict__ cam_new,
                                                    double* __restrict__ camRn, double* __restrict__ part_step,
                                                    double* __restrict__ part_bad) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  __shared__ double T[NB * TS];    // diagonal tile being factored, then L_jj
  __shared__ double Wl[NB * TS];   // W_j of the current step
  __shared__ double Ls[NB * TS];   // L_10
  __shared__ double W0[NB * TS];   // W_0 (kept for the back substitution)
  __shared__ double scr[4][256];
  __shared__ double v[NB];
  __shared__ double yl[NB];        // y_1
  __shared__ int rdy[4];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // ---- step 0: POTRF of tile (0, 0) ----
  load_tile(T, A, ld, 0, 0);
  __syncthreads();
  NoPrefetch nopre;
  const bool bad0 = (NB <= n) ? potrf_tile<true>(T, Wl, scr, 0, n, nullptr, nullptr, nullptr, 0, rdy, nopre)
                              : potrf_tile<false>(T, Wl, scr, 0, n, nullptr, nullptr, nullptr, 0, rdy, nopre);
  bool bad = bad0;
  if (nb > 1) {
    // W_0 kept; L_10 = A_10 W_0^T (the walker's TRSM of the subdiagonal tile)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = t + 256 * q, c = e >> 6, r = e & 63;
      W0[c * TS + r] = Wl[c * TS + r];
      T[c * TS + r] = A[size_t(c) * ld + NB + r];
    }
    __syncthreads();
    f64x4 x[4];
    trsm_lds(T, Wl, x, lane);
    put_tile(Ls, x, lane);
    __syncthreads();
    // ---- step 1: T_11 -= L_10 L_10^T (column block 0 here, the rest inside
    // the POTRF's panel 0, as the walker), POTRF of tile (1, 1) ----
    load_tile(T, A, ld, NB, NB);
    __syncthreads();
    {
      const int Ib[1] = {w}, Jb[1] = {0};
      last_update<1>(T, Ls, Ib, Jb, 1, lane);
    }
    __syncthreads();
    bad |= (2 * NB <= n) ? potrf_tile<true>(T, Wl, scr, NB, n, Ls, nullptr, nullptr, 0, rdy, nopre)
                         : potrf_tile<false>(T, Wl, scr, NB, n, Ls, nullptr, nullptr, 0, rdy, nopre);
  }
  if (bad && t == 0) atomicOr(fail, 1);
  // ---- back substitution L^T y = z, z = row n of the factor (k_backsolve's
  // arithmetic, block rows nb_real - 1 .. 0) ----
  const int nb_real = (n + NB - 1) / NB;
  const int col = t >> 2, seg = t & 3, rn = n & (NB - 1);
  // tile (n / 64, b) of the factor holding row n: L_00 (T, nb == 1), L_10
  // (Ls) and L_11 (T) (nb == 2)
  for (int b = nb_real - 1; b >= 0; --b) {
    const int k0 = b * NB;
    const int nreal = (n - k0) < NB ? (n - k0) : NB;
    const double* Zt = (nb == 1 || b == 1) ? T : Ls;
    const double* Wb = (nb == 1 || b == 1) ? Wl : W0;
    const double zc = (seg == 0 && col < nreal) ? Zt[col * TS + rn] : 0.0;
    double acc = 0.0;
    if (b == 0 && nb_real == 2) {
      // k = 1: L_10^T y_1 (column col of L_10, rows 16 seg .. +16)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc = fma(Ls[col * TS + 16 * seg + i], yl[16 * seg + i], acc);
    }
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    if (seg == 0) v[col] = (col < nreal) ? zc - acc : 0.0;
    __syncthreads();
    double p4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int i = 0; i < 16; ++i) p4[i & 3] = fma(Wb[col * TS + 16 * seg + i], v[16 * seg + i], p4[i & 3]);
    double sum = (p4[0] + p4[1]) + (p4[2] + p4[3]);
    sum += __shfl_xor(sum, 1);
    sum += __shfl_xor(sum, 2);
    if (seg == 0) {
      const double yv = col < nreal ? sum : 0.0;
      y[k0 + col] = yv;
      if (b == 1) yl[col] = yv;
    }
    __syncthreads();
  }
  if (cam) {  // the camera step (y written above, by this workgroup)
    double st = 0.0, bd = 0.0;
    if (t < C) cam_update_one(t, cam, y, scale_c, cam_new, camRn, st, bd);
    const double rs = block_reduce(st, v, false);
    if (t == 0 && part_step) part_step[0] = rs;
    const double rb = block_reduce(bd, v, true);
    if (t == 0) part_bad[0] = rb;
  }
}

// ---------------------------------------------------------------------------
// Distributed factor (1-D block-cyclic column panels over the ranks; see
// DESIGN.md §7).  Panel J = tile columns [pt J, pt J + pt); rank J % N owns
// it.  Per panel k: its owner factors it (k_chol_fused with ncols = pt on
// the trailing matrix), every rank receives it by broadcast and applies it
// to its own later panels (k_panel_update), so at the end every rank holds
// the whole L (and every W_k) and the back substitution runs replicated.

// Own tile columns of panels j in [j0, j1], in order (j % nranks == rank),
// tile columns [pt j, min(pt j + pt, nblk)); column jt holds the nblk - jt
// tiles (jt .. nblk-1, jt).
__device__ __forceinline__ bool panel_task(int task, int nblk, int pt, int j0, int j1, int nranks, int rank, int* it,
                                           int* jt) {
  int j = j0 + ((rank - j0) % nranks + nranks) % nranks;
  for (; j <= j1 && j * pt < nblk; j += nranks) {
    for (int c = j * pt; c < min(j * pt + pt, nblk); ++c) {
      const int cnt = nblk - c;
      if (task < cnt) {
        *jt = c;
        *it = c + task;
        return true;
      }
      task -= cnt;
    }
  }
  return false;
}

// S tile (it, jt) -= L_it,k L_jt,k^T over panel k's columns [kc0, kc0 + kw):
// one tile per workgroup, wave w the 32x32 quadrant (c in cb.., r in rb..)
// accumulated transposed as in fused_helper_tile (the strictly upper
// quadrant of a diagonal tile is skipped: never read).  Every tile keeps its
// k order (the panel's columns ascending), the order the single-GPU factor
// applies them in.
__global__ __launch_bounds__(256) void k_panel_update(double* __restrict__ A, int ld, int nblk, int pt, int pj0,
                                                      int pj1, int kc0, int kw, int nranks, int rank) {
  int it = 0, jt = 0;
  if (!panel_task(blockIdx.x, nblk, pt, pj0, pj1, nranks, rank, &it, &jt)) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cb = 32 * (w >> 1), rb = 32 * (w & 1);
  const int lr = lane & 15, lk = lane >> 4;
  const int i0 = it * NB, j0 = jt * NB;
  if (it == jt && cb > rb) return;  // wave-uniform; no barrier in this kernel
  f64x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) acc[a][bb] = f64x4{0.0, 0.0, 0.0, 0.0};
  for (int k0 = kc0; k0 < kc0 + kw; k0 += NB) {
    double xa[2][16], yb[2][16];
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const size_t colbase = size_t(k0 + 4 * ks + lk) * ld;
#pragma unroll
      for (int a = 0; a < 2; ++a) xa[a][ks] = A[colbase + j0 + cb + 16 * a + lr];
#pragma unroll
      for (int bb = 0; bb < 2; ++bb) yb[bb][ks] = A[colbase + i0 + rb + 16 * bb + lr];
    }
#pragma unroll
    for (int ks = 0; ks < 16; ++ks)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int bb = 0; bb < 2; ++bb)
          acc[a][bb] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[a][ks], yb[bb][ks], acc[a][bb], 0, 0, 0);
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int bb = 0; bb < 2; ++bb)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        double* q = A + size_t(j0 + cb + 16 * a + lk + 4 * reg) * ld + i0 + rb + 16 * bb + lr;
        *q -= acc[a][bb][reg];
      }
}

// Panel rectangles <-> a contiguous buffer: column c (c0_J <= c < c1_J of
// panel J, c <= n) rows [c0_J, n] at buf + off[J] + (c - c0_J)(n + 1 - c0_J)
// (off[J] < 0: panel J skipped).  One workgroup per column.  Rows beyond n
// (identity padding, zero in every real column) and columns beyond n never
// travel: every rank writes them itself (k_schur_diag_sum).
// kMode: 0 pack (S -> buf), 1 unpack (buf -> S), 2 accumulate (S += buf).
template <int kMode>
__global__ __launch_bounds__(256) void k_panel_copy(double* __restrict__ A, int ld, int n, int pcols, int col0,
                                                    const int64_t* __restrict__ off, int64_t off1,
                                                    double* __restrict__ buf) {
  const int c = col0 + blockIdx.x;
  const int J = c / pcols, c0 = J * pcols;
  const int64_t o = off ? off[J] : off1;
  if (o < 0) return;
  const int rows = n + 1 - c0;
  double* b = buf + o + int64_t(c - c0) * rows;
  double* col = A + size_t(c) * ld + c0;
  for (int r = threadIdx.x; r < rows; r += 256) {
    if (kMode == 0) b[r] = col[r];
    else if (kMode == 1) col[r] = b[r];
    else col[r] += b[r];
  }
}

// A broadcast panel's tail: its failure bits (one double slot) OR-ed into
// this rank's flag.
__global__ void k_fail_or(const double* __restrict__ slot, int* __restrict__ fail) {
  const int v = int(__builtin_bit_cast(uint64_t, *slot) & 0x7fffffffu);
  if (v) atomicOr(fail, v);
}
__global__ void k_fail_put(const int* __restrict__ fail, double* __restrict__ slot) {
  *slot = __builtin_bit_cast(double, uint64_t(uint32_t(*fail)));
}

// A diagonally dominant (so SPD) augmented system made on the device, for
// the distributed factor's component timing (sfm_dist_factor_profile): the
// timings do not depend on the values, a 12000^2 host matrix would cost
// seconds to make and upload.
__global__ void k_spd_fill(double* __restrict__ A, int ld, int n, unsigned seed) {
  const int j = blockIdx.x;
  for (int i = threadIdx.x; i < ld; i += blockDim.x) {
    uint64_t z = (uint64_t(seed) << 40) ^ (uint64_t(j) * 0x9E3779B97F4A7C15ull) ^ (uint64_t(i) * 0xBF58476D1CE4E5B9ull);
    z ^= z >> 31; z *= 0x94D049BB133111EBull; z ^= z >> 29;
    const double u = double(z >> 11) * (1.0 / 9007199254740992.0) - 0.5;
    double v = 0.0;
    if (j < n) v = i < j ? 0.0 : (i == j ? 1.0 + 0.5 * n : (i <= n ? u : 0.0));
    else v = i == j ? 1.0 : 0.0;
    A[size_t(j) * ld + i] = v;
  }
}

}  // namespace

bool launch_cholesky(const DevProblem& d, int epoch, hipStream_t s, bool clear_fail, int cam_step, int overlap) {
  if (clear_fail) (void)hipMemsetAsync(d.fail, 0, sizeof(int), s);
  // (SFM_CHOL_NO_SMALL=1: the persistent pair at every size, for the
  // bitwise comparison in tests/test_gpu_parity.py)
  static const bool no_small = [] {
    const char* e = std::getenv("SFM_CHOL_NO_SMALL");
    return e && e[0] == '1';
  }();
  if (d.nblk <= 2 && !no_small) {  // factor + back substitution in one workgroup
    const bool fold = cam_step >= 0 && d.C <= 256;
    double* part = d.partials;
    k_chol_small<<<1, 256, 0, s>>>(d.S, d.ld, d.n, d.nblk, d.ysol, d.fail, d.gate, d.C, fold ? d.cam : nullptr,
                                   d.scale_c, d.cam_new, d.camRn,
                                   fold && cam_step > 0 ? part + size_t(kPStepCam) * d.max_blocks : nullptr,
                                   part + size_t(kPBadCam) * d.max_blocks);
    return fold;
  }
  const int nb = d.nblk, ntask = chol_tasks(nb, nb);
  // one persistent workgroup per CU (roles by start order: a partly resident
  // grid still finishes)
  // (SFM_CHOL_HELPERS: a smaller helper grid, for measurements)
  static const int helpers_env = [] {
    const char* e = std::getenv("SFM_CHOL_HELPERS");
    return e ? std::atoi(e) : 0;
  }();
  // (overlapped with the Schur pass: half the CUs, the other half runs
  // k_schur_pts, whose blocks the helpers await -- at n = 3000 127 helpers
  // factor as fast as 255, 63 take 1.37x)
  const int full = overlap ? d.n_cu / 2 - 1 : d.n_cu - 1;
  const int cap = helpers_env > 0 ? std::min(helpers_env, full) : full;
  const int nhelp = std::max(1, std::min(ntask, cap));
  const int* tc = overlap ? d.tile_cnt : nullptr;
  k_chol_fused<false><<<1 + nhelp, 256, 0, s>>>(d.S, d.ld, d.n, nb, nb, d.invL, d.cflags, d.cflags + size_t(nb) * nb,
                                         d.cticket, epoch, epoch, nhelp, d.fail, d.gate, tc, d.tile_exp);
  return false;
}

void launch_backsolve(const DevProblem& d, int epoch, hipStream_t s, bool sentinel_set) {
  const int nb_real = (d.n + NB - 1) / NB;
  static const bool no_small = [] {
    const char* e = std::getenv("SFM_CHOL_NO_SMALL");
    return e && e[0] == '1';
  }();
  if (nb_real <= 0 || (d.nblk <= 2 && !no_small)) return;  // (nblk <= 2: k_chol_small solved too)
  // the sentinel in every entry of y the launch produces (ld >= 64 nb_real;
  // the solve's k_pad_init writes it, saving a launch)
  if (!sentinel_set)
    (void)hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d.ysol), int(kYSentinelWord), size_t(nb_real) * NB * 2, s);
  k_backsolve<<<nb_real, 256, 0, s>>>(d.S, d.ld, d.n, nb_real, d.invL, d.ysol, d.fail, d.gate, d.cticket + 2, epoch);
}

int launch_cholesky_panel(const DevProblem& d, int k, int pt, int epoch, hipStream_t s) {
  const int t0 = k * pt, nb = d.nblk - t0, ncols = std::min(pt, nb);
  if (ncols <= 0) return 0;
  const int c0 = t0 * NB;
  const int ntask = chol_tasks(nb, ncols);
  const int nhelp = std::max(1, std::min(ntask, d.n_cu - 1));
  // the panel's own tickets (ntask differs per panel): zeroed, ticket epoch 1
  (void)hipMemsetAsync(d.cticket + 3, 0, 2 * sizeof(unsigned long long), s);
  k_chol_fused<true><<<1 + nhelp, 256, 0, s>>>(d.S + size_t(c0) * d.ld + c0, d.ld, d.n - c0, nb, ncols,
                                         d.invL + size_t(t0) * NB * NB, d.cflags, d.cflags + size_t(nb) * nb,
                                         d.cticket + 3, epoch, 1, nhelp, d.fail, nullptr, nullptr, nullptr);
  return 0;
}

int panel_update_tiles(int nblk, int pt, int j0, int j1, int nranks, int rank) {
  int n = 0;
  for (int j = j0; j <= j1 && j * pt < nblk; ++j) {
    if (j % nranks != rank) continue;
    for (int c = j * pt; c < std::min(j * pt + pt, nblk); ++c) n += nblk - c;
  }
  return n;
}

void launch_panel_update(const DevProblem& d, int k, int j0, int j1, int pt, int nranks, int rank, hipStream_t s) {
  const int tiles = panel_update_tiles(d.nblk, pt, j0, j1, nranks, rank);
  if (tiles <= 0) return;
  const int kc0 = k * pt * NB, kw = std::min(pt, d.nblk - k * pt) * NB;
  k_panel_update<<<tiles, 256, 0, s>>>(d.S, d.ld, d.nblk, pt, j0, j1, kc0, kw, nranks, rank);
}

void launch_panel_copy(const DevProblem& d, int mode, int pt, int col0, int col1, const int64_t* off, int64_t off1,
                       double* buf, hipStream_t s) {
  col1 = std::min(col1, d.n + 1);
  if (col1 <= col0) return;
  if (mode == 0) k_panel_copy<0><<<col1 - col0, 256, 0, s>>>(d.S, d.ld, d.n, pt * NB, col0, off, off1, buf);
  else if (mode == 1) k_panel_copy<1><<<col1 - col0, 256, 0, s>>>(d.S, d.ld, d.n, pt * NB, col0, off, off1, buf);
  else k_panel_copy<2><<<col1 - col0, 256, 0, s>>>(d.S, d.ld, d.n, pt * NB, col0, off, off1, buf);
}

void launch_fail_slot(const DevProblem& d, bool put, double* slot, hipStream_t s) {
  if (put) k_fail_put<<<1, 1, 0, s>>>(d.fail, slot);
  else k_fail_or<<<1, 1, 0, s>>>(slot, d.fail);
}

void launch_spd_fill(double* A, int ld, int n, unsigned seed, hipStream_t s) {
  k_spd_fill<<<ld, 256, 0, s>>>(A, ld, n, seed);
}

}  // namespace sfm

#ifdef SFM_CHOL_STAMPS
extern "C" int sfm_debug_bstamps(unsigned long long* out, int n) {
  if (n > 256 * 8) n = 256 * 8;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(sfm::g_bstamp), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -5;
}
extern "C" int sfm_debug_pstamps(unsigned long long* out, int n) {
  if (n > 256 * 4) n = 256 * 4;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(sfm::g_pstamp), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -5;
}
extern "C" int sfm_debug_stamps(unsigned long long* out, int n, unsigned long long* hout, int hn) {
  if (n > 256 * 16) n = 256 * 16;
  if (hn > 128 * 128 * 2) hn = 128 * 128 * 2;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sfm::g_wstamp), sizeof(unsigned long long) * n) != hipSuccess) return -5;
  if (hout && hn > 0 &&
      hipMemcpyFromSymbol(hout, HIP_SYMBOL(sfm::g_hstamp), sizeof(unsigned long long) * hn) != hipSuccess)
    return -5;
  return 0;
}
#endif
