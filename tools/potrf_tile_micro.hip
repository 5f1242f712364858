// Microbenchmark + check of the walker's 64x64 tile POTRF variants
// (chol_kernels.hip potrf_tile: 16-column panels, lane-per-row pivot chain;
// potrf_tile8: 8-column panels, redundant in-register diagonal factor).
// One workgroup, the tile in LDS as in k_chol_fused; each variant runs
// `reps` times back to back on fresh copies, timed with s_memtime (100 MHz).
// Output: per-variant cycles per POTRF and max |L - L_ref|, |W - W_ref|.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I sfm_amd/csrc tools/potrf_tile_micro.hip -o tools/potrf_tile_micro
#include "../sfm_amd/csrc/chol_kernels.hip"

// Measured on MI355X: potrf_tile 9.8 us per tile, potrf_tile8 17.1 us (the
// redundant 8x8 factor + inverse is ~300 dependent fp64 VALU instructions
// per panel on one wave: issue/latency bound), so the product keeps
// potrf_tile.
namespace sfm {
namespace {
// ---------------------------------------------------------------------------
// POTRF of the 64x64 tile in 8-column panels with NO cross-lane traffic on
// the pivot chain.  Per panel b (columns g0 = 8b .. g0+7), wave 0:
//   * every lane loads the panel's 8x8 diagonal block D (LDS broadcast
//     reads) and factors it REDUNDANTLY in registers: the 8 pivots are a
//     register-only chain (rsqrt + one Newton-class step + a multiply and an
//     FMA per pivot), no readlane, no LDS round trip;
//   * lane r forward-substitutes its own row, L(r, g) = (A(r, g) - sum_k
//     L(r, k) L(g, k)) / L(g, g), from its 8 panel entries -- lane-local
//     (for r inside the diagonal block this is the same recurrence, so the
//     entries agree with D's bitwise);
//   * W_bb = L_bb^-1 (8x8) also redundantly in registers; lanes 0..7 store
//     its rows.
// Then all four waves apply the rank-8 trailing update on MFMA (16x16x4,
// two k steps; the B operand is masked to the columns right of the panel),
// and for odd b wave 0 closes the 16x16 diagonal block of W:
//   W_ba = -W_b L_ba W_a.
// The off-diagonal 16x16 blocks of W are formed by waves 1-3 (w_offdiag)
// while wave 0 factors the next panel, as in potrf_tile.  Rows above the
// panel (strictly upper part of the tile) are written as zeros.
__device__ __forceinline__ constexpr int tri8(int r, int c) { return r * (r + 1) / 2 + c; }

template <bool kFull>
__device__ __forceinline__ bool potrf_tile8(double* T, double* Wl, double (*scr)[256], int k0, int n) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = t + 256 * q, c = e >> 6, r = e & 63;
    Wl[c * TS + r] = 0.0;
  }
  __syncthreads();
  bool bad = false;
  for (int b = 0; b < 8; ++b) {
    const int g0 = 8 * b;
    if (w == 0) {
      double D[36], p[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        p[c] = T[(g0 + c) * TS + lane];
#pragma unroll
        for (int r = c; r < 8; ++r) D[tri8(r, c)] = T[(g0 + c) * TS + g0 + r];  // same address in every lane
      }
      double iv[8];
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        double d = D[tri8(g, g)];
        if (kFull || k0 + g0 + g < n) bad |= !(d > 0.0);
        else d = 1.0;
        iv[g] = rsqrt_nr(d);
        D[tri8(g, g)] = d * iv[g];
#pragma unroll
        for (int r = g + 1; r < 8; ++r) D[tri8(r, g)] *= iv[g];
#pragma unroll
        for (int c = g + 1; c < 8; ++c)
#pragma unroll
          for (int r = c; r < 8; ++r) D[tri8(r, c)] = fma(-D[tri8(r, g)], D[tri8(c, g)], D[tri8(r, c)]);
      }
      // own row (lane = row; rows above the panel are the don't-care upper part)
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        double acc = p[g];
#pragma unroll
        for (int k = 0; k < g; ++k) acc = fma(-p[k], D[tri8(g, k)], acc);
        p[g] = acc * iv[g];
      }
      const bool above = lane < g0;
#pragma unroll
      for (int c = 0; c < 8; ++c) T[(g0 + c) * TS + lane] = above ? 0.0 : p[c];
      // W_bb = L_bb^-1, column by column
      double Wb[36];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        Wb[tri8(j, j)] = iv[j];
#pragma unroll
        for (int r = j + 1; r < 8; ++r) {
          double s = 0.0;
#pragma unroll
          for (int k = j; k < r; ++k) s = fma(D[tri8(r, k)], Wb[tri8(k, j)], s);
          Wb[tri8(r, j)] = -s * iv[r];
        }
      }
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (lane == r)
#pragma unroll
          for (int c = 0; c <= r; ++c) Wl[(g0 + c) * TS + g0 + r] = Wb[tri8(r, c)];
    } else if (!(b & 1) && b >= 4 && w - 1 < (b >> 1) - 1) {
      w_offdiag(T, Wl, scr[w], (b >> 1) - 1, w - 1, lane);  // row B-1 of W, B = b/2 (its diagonal block is done)
    }
    __syncthreads();
    // ---- trailing update of columns >= g0 + 8 (rank 8, MFMA) ----
    if (b < 7) {
      const int cmin = g0 + 8, J0 = cmin >> 4, nJ = 4 - J0, nq = nJ * (nJ + 1) / 2;
      const int li = lane & 15, kk = lane >> 4;
      for (int q = w; q < nq; q += 4) {
        int J = J0, qq = q;
        while (qq >= 4 - J) { qq -= 4 - J; ++J; }
        const int I = J + qq;
        f64x4 acc = {0.0, 0.0, 0.0, 0.0};
        const bool live = 16 * J + li >= cmin;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int k = g0 + 4 * s + kk;
          const double a = T[k * TS + 16 * I + li];
          const double bv = live ? T[k * TS + 16 * J + li] : 0.0;
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bv, acc, 0, 0, 0);
        }
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) T[(16 * J + li) * TS + 16 * I + 4 * rr + kk] -= acc[rr];
      }
    }
    if ((b & 1) && w == 0) {
      // 16x16 diagonal block I of W: W_ba = -W_b L_ba W_a (8x8 blocks;
      // lane i*8 + j owns entry (i, j))
      const int I16 = 16 * (b >> 1), i = lane >> 3, j = lane & 7;
      double x = 0.0;  // X = L_ba W_a
#pragma unroll
      for (int m = 0; m < 8; ++m)
        if (m >= j) x = fma(T[(I16 + m) * TS + I16 + 8 + i], Wl[(I16 + j) * TS + I16 + m], x);
      scr[0][lane] = x;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      double y = 0.0;
#pragma unroll
      for (int m = 0; m < 8; ++m)
        if (m <= i) y = fma(Wl[(I16 + 8 + m) * TS + I16 + 8 + i], scr[0][8 * m + j], y);
      Wl[(I16 + j) * TS + I16 + 8 + i] = -y;
    }
    __syncthreads();
  }
  // ---- W row 3 off the diagonal (its diagonal block closes with panel 7) ----
  if (w < 3) w_offdiag(T, Wl, scr[w], 3, w, lane);
  __syncthreads();
  return bad;
}

}  // namespace
}  // namespace sfm
#include <cstdio>
#include <vector>
#include <cmath>

namespace sfm {
namespace {
template <int V>
__global__ __launch_bounds__(256) void k_bench(const double* __restrict__ A, double* __restrict__ L,
                                               double* __restrict__ W, unsigned long long* st, int reps, int n) {
  __shared__ double T[NB * TS];
  __shared__ double Wl[NB * TS];
  __shared__ double scr[4][256];
  const int t = threadIdx.x;
  unsigned long long tot = 0;
  bool bad = false;
  for (int rep = 0; rep < reps; ++rep) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = t + 256 * q, c = e >> 6, r = e & 63;
      T[c * TS + r] = A[c * 64 + r];
    }
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (V == 16) bad |= potrf_tile<true>(T, Wl, scr, 0, n);
    else bad |= potrf_tile8<true>(T, Wl, scr, 0, n);
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    tot += t1 - t0;
    __syncthreads();
  }
  if (t == 0) { st[0] = tot; st[1] = bad; }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = t + 256 * q, c = e >> 6, r = e & 63;
    L[c * 64 + r] = T[c * TS + r];
    W[c * 64 + r] = Wl[c * TS + r];
  }
}
}  // namespace
}  // namespace sfm

int main() {
  const int n = 64, reps = 50;
  std::vector<double> A(n * n);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (s >> 8) / double(1 << 24) - 0.5; };
  std::vector<double> B(n * n);
  for (auto& v : B) v = rnd();
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double acc = 0;
      for (int k = 0; k < n; ++k) acc += B[i * n + k] * B[j * n + k];
      A[j * n + i] = acc + (i == j ? 4.0 : 0.0);  // column-major, SPD
    }
  // reference L (lower) and W = L^-1
  std::vector<double> Lr(n * n, 0.0), Wr(n * n, 0.0);
  for (int j = 0; j < n; ++j) {
    double d = A[j * n + j];
    for (int k = 0; k < j; ++k) d -= Lr[k * n + j] * Lr[k * n + j];
    Lr[j * n + j] = std::sqrt(d);
    for (int i = j + 1; i < n; ++i) {
      double v = A[j * n + i];
      for (int k = 0; k < j; ++k) v -= Lr[k * n + i] * Lr[k * n + j];
      Lr[j * n + i] = v / Lr[j * n + j];
    }
  }
  for (int j = 0; j < n; ++j) {
    Wr[j * n + j] = 1.0 / Lr[j * n + j];
    for (int i = j + 1; i < n; ++i) {
      double sacc = 0;
      for (int k = j; k < i; ++k) sacc += Lr[k * n + i] * Wr[j * n + k];
      Wr[j * n + i] = -sacc / Lr[i * n + i];
    }
  }
  double *dA, *dL, *dW;
  unsigned long long* dst;
  hipMalloc(&dA, n * n * 8); hipMalloc(&dL, n * n * 8); hipMalloc(&dW, n * n * 8); hipMalloc(&dst, 16);
  hipMemcpy(dA, A.data(), n * n * 8, hipMemcpyHostToDevice);
  for (int v : {16, 8, 16, 8}) {
    if (v == 16) sfm::k_bench<16><<<1, 256>>>(dA, dL, dW, dst, reps, n);
    else sfm::k_bench<8><<<1, 256>>>(dA, dL, dW, dst, reps, n);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
    unsigned long long st[2];
    std::vector<double> L(n * n), W(n * n);
    hipMemcpy(st, dst, 16, hipMemcpyDeviceToHost);
    hipMemcpy(L.data(), dL, n * n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(W.data(), dW, n * n * 8, hipMemcpyDeviceToHost);
    double eL = 0, eW = 0;
    for (int j = 0; j < n; ++j)
      for (int i = j; i < n; ++i) {
        eL = std::max(eL, std::fabs(L[j * n + i] - Lr[j * n + i]) / std::fabs(Lr[j * n + j]));
        eW = std::max(eW, std::fabs(W[j * n + i] - Wr[j * n + i]) * std::fabs(Lr[i * n + i]));
      }
    // W upper part of each 16x16 diagonal block must be zero (MFMA operand)
    double up = 0;
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < j; ++i)
        if (i / 16 == j / 16) up = std::max(up, std::fabs(W[j * n + i]));
    printf("potrf_tile%-2d  %.2f us per tile (s_memtime 100 MHz)  max rel |L-Lref| %.2e  |W-Wref| %.2e  W-upper %.1e  bad %llu\n",
           v, st[0] / 100.0 / reps, eL, eW, up, st[1]);
  }
  return 0;
}
