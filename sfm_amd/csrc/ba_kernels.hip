// Bundle-adjustment LM-iteration kernels for gfx950 (MI355X), fp64.
//
// Restates on the GPU the per-iteration work Ceres performs inside
// ceres::Solve for CTracker::bundleAdjustmentStructAndPose
// (/root/reference/CTracker.cpp:670-702):
//   * residual + 2x9 Jacobian of BAStructAndPoseFunctor (CTracker.cpp:585-604)
//     with ceres::AngleAxisRotatePoint (CTracker.cpp:588), Jacobi-scaled;
//   * the DENSE_SCHUR normal-equation assembly: per-point 3x3 blocks V_p,
//     per-camera 6x6 blocks U_c, reduced camera matrix S = U + D^2 - W V^-1 W^T
//     and its right-hand side;
//   * point back-substitution, the LM model-cost change and the candidate
//     residual evaluation.
// Every reduction is a fixed-order tree (per-block partials, then one
// ordered pass), so cost / gradient / step norms are bitwise reproducible.
// (No atomics in any sum: whole solves are bitwise reproducible.)
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include "ba_device.h"
#include "ba_common.h"

namespace sfm {

namespace {

// ---------------------------------------------------------------------------
// With cam_src (the device LM loop's accepted step, k_lm_accept folded in)
// the cameras are read from cam_src and stored to cam, and the grid also
// copies X_src -> X_dst (n_x doubles); only the first ceil(C / kThreads)
// workgroups hold cameras and write |x|^2 partials.
__global__ __launch_bounds__(kThreads) void k_cam_prep(int C, double* __restrict__ cam,
                                                       double* __restrict__ camR, double* __restrict__ part_xn, const int* __restrict__ gate,
                                                       const double* __restrict__ cam_src, const double* __restrict__ X_src,
                                                       double* __restrict__ X_dst, int64_t n_x) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  __shared__ double sh[4];
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n_x; i += int64_t(gridDim.x) * blockDim.x)
    X_dst[i] = X_src[i];
  if (int64_t(blockIdx.x) * blockDim.x >= C) return;  // workgroup-uniform: no camera in this one
  double xn = 0.0;
  if (c < C) {
    const double* cs = cam_src ? cam_src : cam;
    double x6[6];
    for (int k = 0; k < 6; ++k) x6[k] = cs[6 * c + k];
    if (cam_src)
      for (int k = 0; k < 6; ++k) cam[6 * c + k] = x6[k];
    const double w[3] = {x6[0], x6[1], x6[2]};
    double R[9], dR[27];
    rotation(w, R, dR);
    double* o = camR + size_t(kCamR) * c;
    for (int i = 0; i < 9; ++i) o[i] = R[i];
    for (int i = 0; i < 27; ++i) o[9 + i] = dR[i];
    for (int k = 0; k < 6; ++k) xn += x6[k] * x6[k];
  }
  const double r = block_reduce(xn, sh, false);
  if (threadIdx.x == 0 && part_xn) part_xn[blockIdx.x] = r;
}

// ---------------------------------------------------------------------------
// Residual + Jacobian in CAMERA-major order.
// Work unit = one wavefront chunk: up to 64 consecutive observations of ONE
// camera (device-built table, 63 chunks per camera at C3).  The camera is
// wave-uniform, so its 44 doubles (R, dR/dw, t, K, Jacobi scale) are scalar
// loads; per lane the pass moves the point index (4 B), uv (16 B) and the
// point X (24 B, a 4.8-MB L2/MALL-resident gather).  In the solve the pass
// writes no per-observation record: the cost and the chunk's 27 U_c / b_c
// partial sums (jpart) are its only outputs, and every later observation
// pass recomputes what it needs.  The evaluate API (write_rec) also stores
// the 160-B record at the camera-major position, through a wave-local LDS
// transpose as fully coalesced 1-KB rows.  The grid is persistent (waves
// stride over the chunk table).
__device__ __forceinline__ int wave_uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Store the wave's staged chunk (64 records from position ib; a camera's
// run is padded to whole chunks) as ten coalesced 1-KB rows.
__device__ __forceinline__ void jac_flush(const double* wst, double* __restrict__ jrec, int64_t ib, int l) {
  double* dst = jrec + ib * kJRec;
  double2 v[kJRec / 2];
#pragma unroll
  for (int kq = 0; kq < kJRec / 2; ++kq) v[kq] = ld2(wst + 2 * (64 * kq + l));
#pragma unroll
  for (int kq = 0; kq < kJRec / 2; ++kq) st2_nt(dst + 2 * (64 * kq + l), v[kq].x, v[kq].y);
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One observation's residual and 2x9 Jacobian record (layout kJX|kRes|kJC).
__device__ __forceinline__ double jac_record(const double* cr, double tc0, double tc1, double tc2, double fx, double sk,
                                             double cx, double fy, double cy, const double* sc, const double* sp,
                                             const double Xp[3], double2 uvo, double rec[kJRec]) {
  const double pc0 = cr[0] * Xp[0] + cr[1] * Xp[1] + cr[2] * Xp[2] + tc0;
  const double pc1 = cr[3] * Xp[0] + cr[4] * Xp[1] + cr[5] * Xp[2] + tc1;
  const double pc2 = cr[6] * Xp[0] + cr[7] * Xp[1] + cr[8] * Xp[2] + tc2;
  // pc0 / pc2, pc1 / pc2, 1 / pc2 bitwise the divisions, one reciprocal
  const SharedDiv dz = shared_div(pc2);
  const double xp = sdiv(dz, pc0), yp = sdiv(dz, pc1);
  const double r0 = fx * xp + sk * yp + cx - uvo.x;
  const double r1 = fy * yp + cy - uvo.y;
  const double iz = srcp(dz);
  // d r / d pc
  const double a0 = fx * iz, a1 = sk * iz, a2 = -(fx * xp + sk * yp) * iz;
  const double b1 = fy * iz, b2 = -fy * yp * iz;
  // J_X = dr/dpc * R
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    rec[kJX + j] = (a0 * cr[j] + a1 * cr[3 + j] + a2 * cr[6 + j]) * sp[j];
    rec[kJX + 3 + j] = (b1 * cr[3 + j] + b2 * cr[6 + j]) * sp[j];
  }
  rec[kRes] = r0;
  rec[kRes + 1] = r1;
  // J_w[:,k] = dr/dpc * (dR_k X);  J_t = dr/dpc
#pragma unroll
  for (int kk = 0; kk < 3; ++kk) {
    const double* D = cr + 9 + 9 * kk;
    const double q0 = D[0] * Xp[0] + D[1] * Xp[1] + D[2] * Xp[2];
    const double q1 = D[3] * Xp[0] + D[4] * Xp[1] + D[5] * Xp[2];
    const double q2 = D[6] * Xp[0] + D[7] * Xp[1] + D[8] * Xp[2];
    rec[kJC + kk] = (a0 * q0 + a1 * q1 + a2 * q2) * sc[kk];
    rec[kJC + 6 + kk] = (b1 * q1 + b2 * q2) * sc[kk];
  }
  rec[kJC + 3] = a0 * sc[3]; rec[kJC + 4] = a1 * sc[4]; rec[kJC + 5] = a2 * sc[5];
  rec[kJC + 9] = 0.0;        rec[kJC + 10] = b1 * sc[4]; rec[kJC + 11] = b2 * sc[5];
  return 0.5 * (r0 * r0 + r1 * r1);
}

// Pipeline per wave, chunk t (vmcnt is one in-order counter for loads AND
// stores on CDNA, so a wait on a load also covers every older store):
//   [X_t, uv_t in flight] issue p_{t+1}, uv_{t+1} -> wait X_t -> compute t
//   -> stage t in LDS -> issue X_{t+1} -> store chunk t.
// kRec: the record-writing variant of the evaluate API (k_jacobian<true>);
// the solve runs the record-free k_jacobian<false> (no staging LDS, so the
// two show up apart in kernel traces and counter passes).
template <bool kRec>
__global__ __launch_bounds__(kThreads) void k_jacobian(const int32_t* __restrict__ grp_off,
                                                       const int4* __restrict__ chunks,
                                                       const int32_t* __restrict__ cm_p,
                                                       const double* __restrict__ uv_cm,
                                                       const double* __restrict__ Kc, const double* __restrict__ cam,
                                                       const double* __restrict__ camR, const double* __restrict__ X,
                                                       const double* __restrict__ scale_c,
                                                       const double* __restrict__ scale_p, int scaled,
                                                       double* __restrict__ jrec, double* __restrict__ part_cost,
                                                       double* __restrict__ jpart, const int* __restrict__ gate) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  __shared__ double sh[4];
  __shared__ __attribute__((aligned(16))) double stage[kRec ? kThreads * kJRec : 2];  // 10 KB per wave
  const int l = threadIdx.x & 63;
  const int wv = wave_uniform(threadIdx.x >> 6);
  double* wst = stage + wv * 64 * kJRec;
  // XCD-aware split: the chunk table is grouped into 8 slices of the point
  // range (a camera's list is sorted by point, so each chunk covers a narrow
  // slice); workgroup b serves slice b % 8 -- the round-robin workgroup ->
  // XCD dispatch puts each slice on one XCD, whose 4-MB L2 then holds that
  // slice's X (0.6 MB at C3) instead of every XCD gathering all 4.8 MB.
  // (Placement is a speed assumption only; any mapping is correct.)
  // Within a slice the chunks are camera-major, and each wave takes one
  // contiguous run of them, so it reduces the U_c / b_c partials once per
  // camera it meets instead of once per chunk.
  const int grp = blockIdx.x & 7;
  const int nbg = (int(gridDim.x) - 1 - grp) / 8 + 1;
  const int nw = nbg * (kThreads / 64);
  const int wi = (blockIdx.x >> 3) * (kThreads / 64) + wv;
  const int g0 = grp_off[grp], glen = grp_off[grp + 1] - g0;
  int t = g0 + int(int64_t(glen) * wi / nw);
  const int n_chunks = g0 + int(int64_t(glen) * (wi + 1) / nw);  // end of this wave's run
  double cost = 0.0;
  // Lanes past the real observations of a camera's last chunk compute the
  // padding slots (copies of its last observation): every load and store is
  // unpredicated, so nothing forces an early wait; padding records are never
  // read back and their cost is masked.
  // Prefetch depths: point index 2 chunks ahead, uv and X one chunk ahead,
  // so the only load a wave ever waits for right after issuing stores is
  // one issued a whole chunk earlier (vmcnt counts loads and stores in issue
  // order: waiting on a young load would also wait on the stores before it).
  auto chunk_at = [&](int tt) { return chunks[tt < n_chunks ? tt : t]; };
  int p_nxt = 0;                              // point index of chunk t + 1
  double2 uv_cur = make_double2(0.0, 0.0);    // chunk t
  double Xc[3] = {0.0, 0.0, 1.0}, spc[3] = {1.0, 1.0, 1.0};
  if (t < n_chunks) {
    const int64_t i = int64_t(chunks[t].y) + l;
    const int p0 = cm_p[i];
    uv_cur = ld2(uv_cm + 2 * i);
    p_nxt = cm_p[int64_t(chunk_at(t + 1).y) + l];
#pragma unroll
    for (int j = 0; j < 3; ++j) Xc[j] = X[3 * size_t(p0) + j];
    if (scaled)
#pragma unroll
      for (int j = 0; j < 3; ++j) spc[j] = scale_p[3 * size_t(p0) + j];
  }
  // materialise the prologue loads here, so the loop entry carries no
  // outstanding loads from this path (the compiler's wait counting merges
  // the prologue and back-edge states conservatively)
  asm volatile("" : "+v"(Xc[0]), "+v"(Xc[1]), "+v"(Xc[2]), "+v"(spc[0]), "+v"(spc[1]), "+v"(spc[2]), "+v"(uv_cur.x),
               "+v"(uv_cur.y), "+v"(p_nxt));
  double acc[32];  // this lane's share of the current camera's U_c (21) and b_c (6)
#pragma unroll
  for (int e = 0; e < 32; ++e) acc[e] = 0.0;
  for (; t < n_chunks; ++t) {
    const int4 ch = chunks[t];
    const int c = ch.x, cnt = ch.z;
    const int64_t ib = ch.y;
    // ---- issue: X / scale of chunk t+1 (its index is already here), uv of
    // chunk t+1, index of chunk t+2 ----
    double Xn[3], spn[3] = {1.0, 1.0, 1.0};
#pragma unroll
    for (int j = 0; j < 3; ++j) Xn[j] = X[3 * size_t(p_nxt) + j];
    if (scaled)
#pragma unroll
      for (int j = 0; j < 3; ++j) spn[j] = scale_p[3 * size_t(p_nxt) + j];
    const int4 ch_n = chunk_at(t + 1);
    const double2 uv_nxt = ld2(uv_cm + 2 * (int64_t(ch_n.y) + l));
    const int p_nn = cm_p[int64_t(chunk_at(t + 2).y) + l];
    // ---- chunk t ----
    const double* cr = camR + size_t(kCamR) * c;  // camera data: wave-uniform -> scalar loads
    const double* k = Kc + 5 * size_t(c);
    double sc[6];
#pragma unroll
    for (int a = 0; a < 6; ++a) sc[a] = scaled ? scale_c[6 * size_t(c) + a] : 1.0;
    {
      double rec[kJRec];
      const double cl = jac_record(cr, cam[6 * c + 3], cam[6 * c + 4], cam[6 * c + 5], k[0], k[1], k[2], k[3], k[4],
                                   sc, spc, Xc, uv_cur, rec);
      cost += (l < cnt) ? cl : 0.0;
      if (kRec) {  // staged for jac_flush
        double* mine = wst + l * kJRec;
#pragma unroll
        for (int f = 0; f < kJRec; f += 2) st2(mine + f, rec[f], rec[f + 1]);
      }
      if (jpart) {
        // the chunk's share of U_c = sum J_c^T J_c (21, packed upper) and
        // b_c = sum J_c^T r (6), accumulated per lane; at the end of the
        // camera's run one reduce-scatter over the wave, lane 2e stores entry
        // e into the run's last chunk slot, the run's other slots get zeros
        // (k_cam_sum adds a camera's slots in order) -- no second pass over
        // the records
        // padding lanes: their 12 J_c entries and 2 residuals zeroed once,
        // so each product sum adds an exact 0 (bitwise the masked sum, 14
        // selects instead of 27)
        // (only a camera's last chunk has padding lanes: the masks sit behind
        // a wave-uniform branch, 28 selects off the full chunks' path)
        double j0[6], j1[6], r0 = rec[kRes], r1 = rec[kRes + 1];
#pragma unroll
        for (int a = 0; a < 6; ++a) {
          j0[a] = rec[kJC + a];
          j1[a] = rec[kJC + 6 + a];
        }
        if (cnt < 64) {
          const bool real = l < cnt;
#pragma unroll
          for (int a = 0; a < 6; ++a) {
            j0[a] = real ? j0[a] : 0.0;
            j1[a] = real ? j1[a] : 0.0;
          }
          r0 = real ? r0 : 0.0;
          r1 = real ? r1 : 0.0;
        }
        int q = 0;
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
          for (int b = a; b < 6; ++b, ++q) acc[q] += j0[a] * j0[b] + j1[a] * j1[b];
#pragma unroll
        for (int a = 0; a < 6; ++a) acc[21 + a] += j0[a] * r0 + j1[a] * r1;
        double tot = 0.0;
        if (t + 1 >= n_chunks || ch_n.x != c) {  // wave-uniform
          tot = wave_sum32(acc, l);
#pragma unroll
          for (int e = 0; e < 32; ++e) acc[e] = 0.0;
        }
        if (!(l & 1) && (l >> 1) < 27) jpart[size_t(ib / 64) * 27 + (l >> 1)] = tot;
      }
    }
    if (kRec) {  // no record consumer left in the record-free solve path
      wave_lds_sync();
      jac_flush(wst, jrec, ib, l);
      wave_lds_sync();
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) { Xc[j] = Xn[j]; spc[j] = spn[j]; }
    uv_cur = uv_nxt;
    p_nxt = p_nn;
  }
  const double r = block_reduce(cost, sh, false);
  if (threadIdx.x == 0) part_cost[blockIdx.x] = r;
}

// mode 0: Jacobi scale from the unscaled column norms (diagonal of U).
// mode 1: LM diagonal (unless reused) and camera gradient max-norm.
// U_c and b_c from k_jacobian's per-chunk partials (jpart): lane t sums
// chunks w0 + t, w0 + t + 64, ..., then one reduce-scatter over the wave.
__global__ __launch_bounds__(64) void k_cam_sum(const int32_t* __restrict__ cam_rng,
                                                const double* __restrict__ jpart, double* __restrict__ Ucam, const int* __restrict__ gate) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  const int c = blockIdx.x, t = threadIdx.x;
  const int w0 = cam_rng[2 * c] / 64, w1 = (cam_rng[2 * c + 1] + 63) / 64;
  double v[32];
#pragma unroll
  for (int e = 0; e < 32; ++e) v[e] = 0.0;
  for (int w = w0 + t; w < w1; w += 64) {
    const double* src = jpart + size_t(w) * 27;
#pragma unroll
    for (int e = 0; e < 27; ++e) v[e] += src[e];
  }
  const double sum = wave_sum32(v, t);
  if (!(t & 1) && (t >> 1) < 27) Ucam[size_t(kUcam) * c + (t >> 1)] = sum;
}

// k_cam_sum + k_cam_finalize in one launch (no cross-rank U_c sum between
// them): the wave's reduce-scatter leaves entry e in lane 2e, lanes 0..5
// take their column's diagonal and gradient entries by shuffle, and the
// camera's gradient max-norm goes to partial slot c (the max over cameras
// is order-free: the same result as k_cam_finalize's per-block partials).
// Camera c's U_c / b_c sums and their finalisation (64 lanes t of one wave,
// no barrier): k_cam_sum_finalize's body, also run by k_point_eval_lds<64>'s
// trailing workgroups for small systems (CamFold: one launch fewer).
struct CamFold {
  const int32_t* cam_rng;
  const double* jpart;
  double* Ucam;
  double* scale_c;
  double* diag_c;
  double min_diag, max_diag;
  int mode, C;
  double* part_grad;
};
__device__ __forceinline__ void cam_sum_body(int c, int t, const CamFold& f) {
  const int w0 = f.cam_rng[2 * c] / 64, w1 = (f.cam_rng[2 * c + 1] + 63) / 64;
  double v[32];
#pragma unroll
  for (int e = 0; e < 32; ++e) v[e] = 0.0;
  for (int w = w0 + t; w < w1; w += 64) {
    const double* src = f.jpart + size_t(w) * 27;
#pragma unroll
    for (int e = 0; e < 27; ++e) v[e] += src[e];
  }
  const double sum = wave_sum32(v, t);
  if (!(t & 1) && (t >> 1) < 27) f.Ucam[size_t(kUcam) * c + (t >> 1)] = sum;
  const int a = t < 6 ? t : 0;
  const double cn = __shfl(sum, 2 * up6(a, a)), ga = __shfl(sum, 2 * (21 + a));
  double g = 0.0;
  if (t < 6) {
    if (f.mode == 0) {
      f.scale_c[6 * c + a] = 1.0 / (1.0 + sqrt(cn));
    } else {
      f.diag_c[6 * c + a] = fmin(fmax(cn, f.min_diag), f.max_diag);
      g = fabs(ga / f.scale_c[6 * c + a]);
    }
  }
#pragma unroll
  for (int off = 4; off > 0; off >>= 1) g = fmax(g, __shfl_xor(g, off));
  if (t == 0 && f.part_grad) f.part_grad[c] = g;
}

__global__ __launch_bounds__(64) void k_cam_sum_finalize(const CamFold f, const int* __restrict__ gate) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  cam_sum_body(blockIdx.x, threadIdx.x, f);
}

__global__ __launch_bounds__(kThreads) void k_cam_finalize(int C, const double* __restrict__ Ucam,
                                                           double* __restrict__ scale_c, double* __restrict__ diag_c,
                                                           double min_diag, double max_diag, int mode, int reuse,
                                                           double* __restrict__ part_grad, const int* __restrict__ gate) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  __shared__ double sh[4];
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  double g = 0.0;
  if (c < C) {
    const double* U = Ucam + size_t(kUcam) * c;
    for (int a = 0; a < 6; ++a) {
      const double cn = U[up6(a, a)];
      if (mode == 0) {
        scale_c[6 * c + a] = 1.0 / (1.0 + sqrt(cn));
      } else {
        if (!reuse) diag_c[6 * c + a] = fmin(fmax(cn, min_diag), max_diag);
        g = fmax(g, fabs(U[21 + a] / scale_c[6 * c + a]));
      }
    }
  }
  const double r = block_reduce(g, sh, true);
  if (threadIdx.x == 0 && part_grad) part_grad[blockIdx.x] = r;
}

// Point pass after a Jacobian evaluation (one lane per point), with the
// point's residuals and J_X recomputed (jac_record's arithmetic) from
// point-major uv (16 B per observation, streamed per lane), the camera index
// and the camera's R, t, K (L2-resident):
// mode 0: Jacobi scale of the point columns; mode 1: V_p, b_p, LM diagonal,
// gradient max-norm and |X|^2.
// Camera constants of the point-major passes, by base pointer and stride per
// camera: R (9), t (3) and K (fx sk cx fy cy), from the global arrays or from
// an LDS copy (k_point_eval_lds).
struct CamView {
  const double* R; const double* t; const double* K;
  int sR, sT, sK;
};

__device__ __forceinline__ void point_eval_body(int p, const int32_t* __restrict__ pt_off,
                                                const int32_t* __restrict__ cam_pm,
                                                const double* __restrict__ uv_pm, const CamView cv,
                                                const double* __restrict__ X, double* __restrict__ scale_p,
                                                double* __restrict__ diag_p, double* __restrict__ ptV,
                                                double min_diag, double max_diag, int mode, int reuse, double& g,
                                                double& xn) {
  double V[6] = {0, 0, 0, 0, 0, 0}, b[3] = {0, 0, 0};
  const double Xp[3] = {X[3 * size_t(p)], X[3 * size_t(p) + 1], X[3 * size_t(p) + 2]};
  double sp[3] = {1.0, 1.0, 1.0};
  if (mode == 1)
    for (int k = 0; k < 3; ++k) sp[k] = scale_p[3 * size_t(p) + k];
  const int q0 = pt_off[p], q1 = pt_off[p + 1];
  // the next observation's camera index and uv are loaded one step ahead
  int c_n = q0 < q1 ? cam_pm[q0] : 0;
  double2 uv_n = q0 < q1 ? ld2(uv_pm + 2 * size_t(q0)) : make_double2(0.0, 0.0);
  for (int q = q0; q < q1; ++q) {
    const int c = c_n;
    const double2 uvo = uv_n;
    if (q + 1 < q1) {
      c_n = cam_pm[q + 1];
      uv_n = ld2(uv_pm + 2 * size_t(q + 1));
    }
    const double* cr = cv.R + size_t(cv.sR) * c;
    const double* k5 = cv.K + size_t(cv.sK) * c;
    const double* tc = cv.t + size_t(cv.sT) * c;
    const double fx = k5[0], sk = k5[1], cx = k5[2], fy = k5[3], cy = k5[4];
    const double pc0 = cr[0] * Xp[0] + cr[1] * Xp[1] + cr[2] * Xp[2] + tc[0];
    const double pc1 = cr[3] * Xp[0] + cr[4] * Xp[1] + cr[5] * Xp[2] + tc[1];
    const double pc2 = cr[6] * Xp[0] + cr[7] * Xp[1] + cr[8] * Xp[2] + tc[2];
    const SharedDiv dz = shared_div(pc2);  // (bitwise the three divisions)
    const double xp = sdiv(dz, pc0), yp = sdiv(dz, pc1);
    const double r0 = fx * xp + sk * yp + cx - uvo.x;
    const double r1 = fy * yp + cy - uvo.y;
    const double iz = srcp(dz);
    const double a0 = fx * iz, a1 = sk * iz, a2 = -(fx * xp + sk * yp) * iz;
    const double b1 = fy * iz, b2 = -fy * yp * iz;
    double u[3], v[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      u[j] = (a0 * cr[j] + a1 * cr[3 + j] + a2 * cr[6 + j]) * sp[j];
      v[j] = (b1 * cr[3 + j] + b2 * cr[6 + j]) * sp[j];
    }
    V[0] += u[0] * u[0] + v[0] * v[0];
    V[1] += u[1] * u[0] + v[1] * v[0]; V[2] += u[1] * u[1] + v[1] * v[1];
    V[3] += u[2] * u[0] + v[2] * v[0]; V[4] += u[2] * u[1] + v[2] * v[1]; V[5] += u[2] * u[2] + v[2] * v[2];
    b[0] += u[0] * r0 + v[0] * r1; b[1] += u[1] * r0 + v[1] * r1; b[2] += u[2] * r0 + v[2] * r1;
  }
  const double cn[3] = {V[0], V[2], V[5]};
  if (mode == 0) {
    for (int k = 0; k < 3; ++k) scale_p[3 * size_t(p) + k] = 1.0 / (1.0 + sqrt(cn[k]));
  } else {
    for (int k = 0; k < 3; ++k) {
      if (!reuse) diag_p[3 * size_t(p) + k] = fmin(fmax(cn[k], min_diag), max_diag);
      g = fmax(g, fabs(b[k] / scale_p[3 * size_t(p) + k]));
      xn += X[3 * size_t(p) + k] * X[3 * size_t(p) + k];
    }
    double* o = ptV + size_t(kPtV) * p;
    st2(o, V[0], V[1]); st2(o + 2, V[2], V[3]); st2(o + 4, V[4], V[5]); st2(o + 6, b[0], b[1]); st2(o + 8, b[2], 0.0);
  }
}

__global__ __launch_bounds__(kThreads) void k_point_eval_rc(int P, const int32_t* __restrict__ pt_off,
                                                            const int32_t* __restrict__ cam_pm,
                                                            const double* __restrict__ uv_pm,
                                                            const double* __restrict__ camR,
                                                            const double* __restrict__ cam,
                                                            const double* __restrict__ Kc,
                                                            const double* __restrict__ X,
                                                            double* __restrict__ scale_p, double* __restrict__ diag_p,
                                                            double* __restrict__ ptV, double min_diag, double max_diag,
                                                            int mode, int reuse, double* __restrict__ part_grad,
                                                            double* __restrict__ part_xn, const int* __restrict__ gate) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  __shared__ double sh[4];
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  double g = 0.0, xn = 0.0;
  if (p < P)
    point_eval_body(p, pt_off, cam_pm, uv_pm, CamView{camR, cam + 3, Kc, kCamR, 6, 5}, X, scale_p, diag_p, ptV,
                    min_diag, max_diag, mode, reuse, g, xn);
  if (mode == 1) {
    const double rg = block_reduce(g, sh, true);
    if (threadIdx.x == 0) part_grad[blockIdx.x] = rg;
    const double rx = block_reduce(xn, sh, false);
    if (threadIdx.x == 0) part_xn[blockIdx.x] = rx;
  }
}

// The same pass with every camera's R, t, K (17 doubles) staged in LDS first
// (C <= kMaxC).  One lane per point gathers ~10 different cameras, so the
// global-memory form issues ~13 camera loads per observation that each touch
// up to 64 cache lines: the texture-address path, not latency, bounds it
// (index/constant prefetching measured no change).  From LDS the same values,
// in the same arithmetic, are bitwise identical.
// kGroups > 1 (C3-sized camera sets, whose 68-KB copy caps a 256-thread
// workgroup at 2 waves per SIMD): one workgroup of kGroups x 256 threads
// shares one copy, group g running the 256 points of virtual block
// blockIdx.x * kGroups + g exactly as a 256-thread workgroup would (same
// points, same per-block partials, reduced over its own four waves in
// order), i.e. twice the waves per LDS copy and half the copies.
constexpr int kCamE = 17;
template <int kMaxC, int kGroups = 1>
__global__ __launch_bounds__(kThreads * kGroups) void k_point_eval_lds(int P, int C, const int32_t* __restrict__ pt_off,
                                                             const int32_t* __restrict__ cam_pm,
                                                             const double* __restrict__ uv_pm,
                                                             const double* __restrict__ camR,
                                                             const double* __restrict__ cam,
                                                             const double* __restrict__ Kc,
                                                             const double* __restrict__ X,
                                                             double* __restrict__ scale_p, double* __restrict__ diag_p,
                                                             double* __restrict__ ptV, double min_diag, double max_diag,
                                                             int mode, int reuse, double* __restrict__ part_grad,
                                                             double* __restrict__ part_xn, const int* __restrict__ gate,
                                                             const CamFold cf) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  static_assert(kGroups == 1 || kMaxC > 64, "the camera fold runs with one group per workgroup");
  const int nbp = (P + kThreads - 1) / kThreads;
  if (kGroups == 1 && int(blockIdx.x) >= nbp) {  // (cf.C > 0) the camera sums: one camera per wave, no barrier
    const int c = (int(blockIdx.x) - nbp) * (kThreads / 64) + int(threadIdx.x >> 6);
    if (c < cf.C) cam_sum_body(c, threadIdx.x & 63, cf);
    return;
  }
  __shared__ double sh[4 * kGroups];
  __shared__ double cst[kMaxC * kCamE];
  for (int i = threadIdx.x; i < C * kCamE; i += blockDim.x) {
    const int c = i / kCamE, j = i - c * kCamE;
    cst[i] = j < 9 ? camR[size_t(kCamR) * c + j] : j < 12 ? cam[6 * size_t(c) + 3 + (j - 9)] : Kc[5 * size_t(c) + (j - 12)];
  }
  __syncthreads();
  const int grp = int(threadIdx.x) / kThreads, tg = int(threadIdx.x) % kThreads;
  const int vb = int(blockIdx.x) * kGroups + grp;  // the 256-thread block this group stands for
  const int p = vb * kThreads + tg;
  double g = 0.0, xn = 0.0;
  if (p < P)
    point_eval_body(p, pt_off, cam_pm, uv_pm, CamView{cst, cst + 9, cst + 12, kCamE, kCamE, kCamE}, X, scale_p,
                    diag_p, ptV, min_diag, max_diag, mode, reuse, g, xn);
  if (mode == 1) {
    // block_reduce per group: its four waves' values combined in wave order
    const int w = int(threadIdx.x) >> 6, l = int(threadIdx.x) & 63;
    const double wg = wave_max(g), wx = wave_sum(xn);
    if (l == 0) sh[w] = wg;
    __syncthreads();
    double rg = 0.0;
    if (tg == 0) {
      rg = sh[4 * grp];
      for (int i = 1; i < 4; ++i) rg = fmax(rg, sh[4 * grp + i]);
    }
    __syncthreads();
    if (l == 0) sh[w] = wx;
    __syncthreads();
    if (tg == 0 && vb < nbp) {
      double rx = sh[4 * grp];
      for (int i = 1; i < 4; ++i) rx = rx + sh[4 * grp + i];
      part_grad[vb] = rg;
      part_xn[vb] = rx;
    }
  }
}

// Per-iteration point factorisation (depends on the trust-region radius),
// one lane per point: V_p + D_p^2 = L L^T, z = L^-1 b_p -> ptL.
// With ptS != nullptr it also writes the point's 128-B record for the
// camera-side passes (X 3 | Jacobi scale 3 | l10 l20 l21 | 1/l_ii 3 | z 3 |
// pad): everything obs_recompute and k_schur_pts read of a point, one line.
__global__ __launch_bounds__(kThreads) void k_point_factor(int P, const double* __restrict__ ptV,
                                                           const double* __restrict__ diag_p, double radius,
                                                           double* __restrict__ ptL, double* __restrict__ part_bad,
                                                           const double* __restrict__ X,
                                                           const double* __restrict__ scale_p,
                                                           double* __restrict__ ptS, const int* __restrict__ gate, const double* __restrict__ radius_dev) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  if (radius_dev) radius = *radius_dev;  // the device LM loop's current radius
  __shared__ double sh[4];
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  double bad = 0.0;
  if (p < P) {
    const double* v = ptV + size_t(kPtV) * p;
    double D[3];
    for (int k = 0; k < 3; ++k) { const double d = sqrt(diag_p[3 * size_t(p) + k] / radius); D[k] = d * d; }
    const double V00 = v[0] + D[0], V10 = v[1], V11 = v[2] + D[1], V20 = v[3], V21 = v[4], V22 = v[5] + D[2];
    const double l00 = sqrt(V00);
    const double l10 = V10 / l00, l20 = V20 / l00;
    const double l11 = sqrt(V11 - l10 * l10);
    const double l21 = (V21 - l20 * l10) / l11;
    const double l22 = sqrt(V22 - l20 * l20 - l21 * l21);
    if (!(l00 > 0.0) || !(l11 > 0.0) || !(l22 > 0.0)) bad = 1.0;
    const double z0 = v[6] / l00, z1 = (v[7] - l10 * z0) / l11, z2 = (v[8] - l20 * z0 - l21 * z1) / l22;
    double* L = ptL + size_t(kPtL) * p;
    st2(L, l00, l10); st2(L + 2, l11, l20); st2(L + 4, l21, l22); st2(L + 6, z0, z1); st2(L + 8, z2, 0.0);
    if (ptS) {
      double* o = ptS + size_t(kPtS) * p;
      const double* x = X + 3 * size_t(p);
      const double* sp = scale_p + 3 * size_t(p);
      st2(o, x[0], x[1]); st2(o + 2, x[2], sp[0]); st2(o + 4, sp[1], sp[2]);
      st2(o + 6, l10, l20); st2(o + 8, l21, 1.0 / l00); st2(o + 10, 1.0 / l11, 1.0 / l22);
      st2(o + 12, z0, z1); st2(o + 14, z2, 0.0);
    }
  }
  const double r = block_reduce(bad, sh, true);
  if (threadIdx.x == 0) part_bad[blockIdx.x] = r;
}

// ---------------------------------------------------------------------------
// Record-free observation kernels (default): the camera-major passes after
// the Jacobian recompute an observation's residual and scaled 2x9 Jacobian
// with jac_record itself (bitwise the k_jacobian record) from the camera
// (wave-uniform: R, dR/dw, t, K, scale are scalar loads), the point (X,
// scale, L_p, z_p: L2/MALL-resident gathers) and the streamed uv, instead of
// reading the 160-B record (325 MB) and the 64-B M record (130 MB) back from
// HBM.  With every consumer recomputing, k_jacobian stops writing records.
struct ObsRC {
  double rec[kJRec];   // J_X 6 | r 2 | J_c 12 (scaled)
  double M[6];         // J_X L^-T, rows m | n
  double h0, h1;       // M z
};
__device__ __forceinline__ void obs_recompute(int c, int p, double2 uvo, const double* __restrict__ camR,
                                              const double* __restrict__ cam, const double* __restrict__ Kc,
                                              const double* __restrict__ scale_c, const double* __restrict__ ptS,
                                              ObsRC& o) {
  // camera (wave-uniform: scalar loads)
  const double* cr = camR + size_t(kCamR) * c;
  const double* k = Kc + 5 * size_t(c);
  const double* tc = cam + 6 * size_t(c) + 3;
  const double* sc = scale_c + 6 * size_t(c);
  const double fx = k[0], sk = k[1], cx = k[2], fy = k[3], cy = k[4];
  // point: one 128-B Schur record (X, scale, L's off-diagonal, 1/l_ii, z):
  // one line per observation
  const double* rp = ptS + size_t(kPtS) * p;
  double q[16];
#pragma unroll
  for (int f = 0; f < 16; f += 2) {
    const double2 x = ld2(rp + f);
    q[f] = x.x; q[f + 1] = x.y;
  }
  const double Xp[3] = {q[0], q[1], q[2]}, sp[3] = {q[3], q[4], q[5]};
  // jac_record's formulas with one reciprocal (1/z) for the projection
  const double pc0 = cr[0] * Xp[0] + cr[1] * Xp[1] + cr[2] * Xp[2] + tc[0];
  const double pc1 = cr[3] * Xp[0] + cr[4] * Xp[1] + cr[5] * Xp[2] + tc[1];
  const double pc2 = cr[6] * Xp[0] + cr[7] * Xp[1] + cr[8] * Xp[2] + tc[2];
  const double iz = srcp(shared_div(pc2)), xp = pc0 * iz, yp = pc1 * iz;  // (iz bitwise 1.0 / pc2)
  double* rec = o.rec;
  rec[kRes] = fx * xp + sk * yp + cx - uvo.x;
  rec[kRes + 1] = fy * yp + cy - uvo.y;
  const double a0 = fx * iz, a1 = sk * iz, a2 = -(fx * xp + sk * yp) * iz;
  const double b1 = fy * iz, b2 = -fy * yp * iz;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    rec[kJX + j] = (a0 * cr[j] + a1 * cr[3 + j] + a2 * cr[6 + j]) * sp[j];
    rec[kJX + 3 + j] = (b1 * cr[3 + j] + b2 * cr[6 + j]) * sp[j];
  }
#pragma unroll
  for (int kk = 0; kk < 3; ++kk) {
    const double* D = cr + 9 + 9 * kk;
    const double q0 = D[0] * Xp[0] + D[1] * Xp[1] + D[2] * Xp[2];
    const double q1 = D[3] * Xp[0] + D[4] * Xp[1] + D[5] * Xp[2];
    const double q2 = D[6] * Xp[0] + D[7] * Xp[1] + D[8] * Xp[2];
    rec[kJC + kk] = (a0 * q0 + a1 * q1 + a2 * q2) * sc[kk];
    rec[kJC + 6 + kk] = (b1 * q1 + b2 * q2) * sc[kk];
  }
  rec[kJC + 3] = a0 * sc[3]; rec[kJC + 4] = a1 * sc[4]; rec[kJC + 5] = a2 * sc[5];
  rec[kJC + 9] = 0.0;        rec[kJC + 10] = b1 * sc[4]; rec[kJC + 11] = b2 * sc[5];
  const double l10 = q[6], l20 = q[7], l21 = q[8], i00 = q[9], i11 = q[10], i22 = q[11];
  const double* e = rec + kJX;
  o.M[0] = e[0] * i00; o.M[1] = (e[1] - l10 * o.M[0]) * i11; o.M[2] = (e[2] - l20 * o.M[0] - l21 * o.M[1]) * i22;
  o.M[3] = e[3] * i00; o.M[4] = (e[4] - l10 * o.M[3]) * i11; o.M[5] = (e[5] - l20 * o.M[3] - l21 * o.M[4]) * i22;
  o.h0 = o.M[0] * q[12] + o.M[1] * q[13] + o.M[2] * q[14];
  o.h1 = o.M[3] * q[12] + o.M[4] * q[13] + o.M[5] * q[14];
}

// XCD-aware chunk order of the camera-major observation passes (as
// k_jacobian): the 64-position chunks are grouped into 8 point slices
// (grp_off), workgroup b serves slice b % 8, so the round-robin workgroup ->
// XCD dispatch keeps each slice's point records (1/8 of ptS) in one XCD's
// L2 instead of every XCD gathering all of them.  Wave wi of its slice takes
// chunks g0 + wi, g0 + wi + nw, ... (placement is a speed assumption only).
struct XcdChunks {
  int t, end, stride;
};
__device__ __forceinline__ XcdChunks xcd_chunks(const int32_t* __restrict__ grp_off, int wv) {
  const int grp = blockIdx.x & 7;
  const int nbg = (int(gridDim.x) - 1 - grp) / 8 + 1;
  const int wi = (blockIdx.x >> 3) * (kThreads / 64) + wv;
  return XcdChunks{grp_off[grp] + wi, grp_off[grp + 1], nbg * (kThreads / 64)};
}

// Per observation (camera-major, one wavefront = 64 positions of ONE camera):
// F = J_c^T M (M = J_X L_p^-T) and the wave's share of the camera's Schur
// diagonal block sum F F^T (21) and rhs sum J_c^T (r - h) (6), reduced over
// its real observations into dpart[chunk][27] (fixed tree order).  J, M, h
// are recomputed (ptS is written by k_point_factor just before).
__global__ __launch_bounds__(kThreads) void k_obs_prep_rc(const int32_t* __restrict__ grp_off,
                                                          const int4* __restrict__ chunks,
                                                          const int32_t* __restrict__ cm_p,
                                                          const double* __restrict__ uv_cm,
                                                          const int32_t* __restrict__ cam_obs,
                                                          const double* __restrict__ camR,
                                                          const double* __restrict__ cam,
                                                          const double* __restrict__ Kc,
                                                          const double* __restrict__ scale_c,
                                                          const double* __restrict__ ptS,
                                                          double* __restrict__ dpart, const int* __restrict__ gate) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // ONE chunk per wave: the grid covers the largest slice (obs_xcd_blocks).
  // (A loop over the slice's chunks took the kernel from 74 to 105 VGPRs,
  // 6 -> 4 waves per SIMD: 45.6 -> 49.5 us at C3.)
  const XcdChunks xc = xcd_chunks(grp_off, wave_uniform(wv));
  if (xc.t >= xc.end) return;  // wave-uniform, no barriers below
  const int4 ch = chunks[xc.t];
  const int64_t i0 = __builtin_amdgcn_readfirstlane(ch.y);
  const int64_t i = i0 + l;
  const int c = __builtin_amdgcn_readfirstlane(ch.x);
  ObsRC o;
  obs_recompute(c, cm_p[i], ld2(uv_cm + 2 * i), camR, cam, Kc, scale_c, ptS, o);
  const double* jc = o.rec + kJC;
  double F[18];  // 6 x 3
#pragma unroll
  for (int u = 0; u < 6; ++u) {
    F[3 * u] = jc[u] * o.M[0] + jc[6 + u] * o.M[3];
    F[3 * u + 1] = jc[u] * o.M[1] + jc[6 + u] * o.M[4];
    F[3 * u + 2] = jc[u] * o.M[2] + jc[6 + u] * o.M[5];
  }
  // padding slots (cam_obs < 0) only in a camera's last chunk (count ch.z <
  // 64): their F and r are zeroed behind a wave-uniform branch, so every
  // product sums an exact 0 (bitwise the masked sums; 24 selects off the full
  // chunks' path instead of 54 on every one)
  double r0 = o.rec[kRes] - o.h0, r1 = o.rec[kRes + 1] - o.h1;
  if (__builtin_amdgcn_readfirstlane(ch.z) < 64) {
    const bool real = cam_obs[i] >= 0;
#pragma unroll
    for (int e = 0; e < 18; ++e) F[e] = real ? F[e] : 0.0;
    r0 = real ? r0 : 0.0;
    r1 = real ? r1 : 0.0;
  }
  double v[32];
  int q = 0;
#pragma unroll
  for (int u = 0; u < 6; ++u)
#pragma unroll
    for (int w = u; w < 6; ++w, ++q)
      v[q] = F[3 * u] * F[3 * w] + F[3 * u + 1] * F[3 * w + 1] + F[3 * u + 2] * F[3 * w + 2];
#pragma unroll
  for (int u = 0; u < 6; ++u) v[21 + u] = jc[u] * r0 + jc[6 + u] * r1;
#pragma unroll
  for (int e = 27; e < 32; ++e) v[e] = 0.0;
  const double tot = wave_sum32(v, l);
  if (!(l & 1) && (l >> 1) < 27) dpart[size_t(i0 / 64) * 27 + (l >> 1)] = tot;
}

// Back substitution pass A (see k_backsub_b): e = J_c y_c, u = M^T e, and
// the observation's share of the model cost change (J, M recomputed); the
// chunks in the XCD-aware order of k_obs_prep_rc.
__global__ __launch_bounds__(kThreads) void k_backsub_a_rc(const int32_t* __restrict__ grp_off,
                                                           const int4* __restrict__ chunks,
                                                           const int32_t* __restrict__ cm_p,
                                                           const double* __restrict__ uv_cm,
                                                           const int32_t* __restrict__ cam_obs,
                                                           const double* __restrict__ camR,
                                                           const double* __restrict__ cam,
                                                           const double* __restrict__ Kc,
                                                           const double* __restrict__ scale_c,
                                                           const double* __restrict__ ptS,
                                                           const double* __restrict__ ysol, double* __restrict__ eu,
                                                           int eu_cm, double* __restrict__ part_model, const int* __restrict__ gate) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  __shared__ double sh[4];
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double model = 0.0;
  const XcdChunks xc = xcd_chunks(grp_off, wave_uniform(wv));
  for (int t = xc.t; t < xc.end; t += xc.stride) {  // wave-uniform
    const int4 ch = chunks[t];
    const int64_t i = int64_t(__builtin_amdgcn_readfirstlane(ch.y)) + l;
    const int c = __builtin_amdgcn_readfirstlane(ch.x);
    ObsRC o;
    obs_recompute(c, cm_p[i], ld2(uv_cm + 2 * i), camR, cam, Kc, scale_c, ptS, o);
    const double* y = ysol + 6 * size_t(c);
    const double* J = o.rec + kJC;
    double e0 = 0.0, e1 = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) { e0 += J[k] * y[k]; e1 += J[6 + k] * y[k]; }
    const int qo = cam_obs[i];
    if (qo >= 0) {
      model += e0 * o.rec[kRes] + e1 * o.rec[kRes + 1] - 0.5 * (e0 * e0 + e1 * e1);
      // u goes to the observation's POINT-major slot (32 B): pass B then
      // streams a point's u contiguously instead of gathering 48-B records
      const double* M = o.M;
      double* dst = eu + 4 * (eu_cm ? size_t(i) : size_t(qo));
      // (the whole 32-B slot, padding included: full-line writes, 59 -> 51 us at C3)
      st2(dst, M[0] * e0 + M[3] * e1, M[1] * e0 + M[4] * e1);
      st2(dst + 2, M[2] * e0 + M[5] * e1, 0.0);
    }
  }
  const double r = block_reduce(model, sh, false);
  if (threadIdx.x == 0) part_model[blockIdx.x] = r;
}

// ---------------------------------------------------------------------------
// Camera c's diagonal block and rhs (64 lanes t of one wave; no barrier):
// k_schur_diag_sum's body, also run by k_schur_pts<64, 4> for a small
// system's diagonal blocks (one launch fewer per LM iteration).
__device__ __forceinline__ void schur_diag_body(int c, int C, int t, const int32_t* __restrict__ cam_rng,
                                                const double* __restrict__ dpart, const double* __restrict__ Ucam,
                                                const double* __restrict__ diag_c, double radius, int add_diag,
                                                double* __restrict__ S, int ld, int n, int init,
                                                int* __restrict__ fail, unsigned long long* __restrict__ ysol,
                                                int n_y) {
  // k_pad_init folded in (one launch fewer per LM iteration): the identity
  // padding below row n of this camera's six columns and y's sentinel
  // there; the last camera also takes columns n.. (the identity block, the
  // pivot (n, n) = 1), the rest of the sentinel and the failure flag.  None
  // of these entries is written by the Schur passes.
  for (int j = 6 * c; j < 6 * c + 6; ++j) {
    for (int i = n + 1 + t; i < ld; i += 64) S[size_t(j) * ld + i] = 0.0;
    if (t == 0 && j < n_y) ysol[j] = kYSentinel;  // k_backsolve's "not yet produced"
  }
  if (c == C - 1) {
    for (int j = n; j < ld; ++j) {
      for (int i = (j > n ? j : n + 1) + t; i < ld; i += 64) S[size_t(j) * ld + i] = (i == j) ? 1.0 : 0.0;
      if (t == 0 && j < n_y) ysol[j] = kYSentinel;
    }
    if (t == 0) {
      S[size_t(n) * ld + n] = 1.0;
      *fail = 0;
    }
  }
  const int w0 = cam_rng[2 * c] / 64, w1 = (cam_rng[2 * c + 1] + 63) / 64;
  // lane t sums waves w0 + t, w0 + t + 64, ... (coalesced 216-B rows), then
  // one reduce-scatter over the wave: lane 2e ends with entry e
  double v[32];
#pragma unroll
  for (int e = 0; e < 32; ++e) v[e] = 0.0;
  for (int w = w0 + t; w < w1; w += 64) {
    const double* src = dpart + size_t(w) * 27;
#pragma unroll
    for (int e = 0; e < 27; ++e) v[e] += src[e];
  }
  const double sum = wave_sum32(v, t);
  // every lane takes part in the shuffle (a source lane must be active):
  // lanes < 36 fetch their S_cc entry, lanes 36..41 the rhs entries
  const int tu = t < 36 ? t / 6 : 0, tv = t < 36 ? t % 6 : 0;
  const int src = t < 36 ? up6(tu, tv) : (t < 42 ? 21 + (t - 36) : 0);
  const double tot = __shfl(sum, 2 * src);
  if (t < 36) {
    const int u = tu, vv = tv, q = src;
    double* sp = S + size_t(6 * c + u) * ld + 6 * size_t(c) + vv;
    double val = (init ? 0.0 : *sp) - tot;  // init: before the off-diagonal launch (k_schur_pts adds its part)
    if (add_diag) {
      val += Ucam[size_t(kUcam) * c + q];
      if (u == vv) { const double dd = sqrt(diag_c[6 * size_t(c) + u] / radius); val += dd * dd; }
    }
    *sp = val;
  } else if (t < 42) {
    S[size_t(6 * c + (t - 36)) * ld + n] = tot;
  }
}

// What k_schur_pts<64, 4> needs to run k_schur_diag_sum's body itself.
struct DiagFold {
  const int32_t* cam_rng;
  const double* dpart;
  const double* Ucam;
  const double* diag_c;
  double radius;
  const double* radius_dev;
  int add_diag, C, n, n_y;
  int* fail;
  unsigned long long* ysol;
};

// k_schur_pts: the off-diagonal Schur blocks WITHOUT the F gathers.  A pair
// (o1, o2) of block (c1, c2) shares its point p, and
//   F_o1 F_o2^T = J_c1^T M_1 M_2^T J_c2,   M_i = J_X,i L_p^-T,
// where J_X,i and J_c,i are functions of (camera c_i, X_p) alone.  So kSub
// lanes own one block: the two cameras' constants (R, dR/dw, t, K, Jacobi
// scale: 50 doubles each) sit in LDS as wave-uniform broadcasts, and each
// lane takes one pair per step, gathering only its point's 128-B record
// (X, scale, L_p, 1/l_ii, z: one line, 25.6 MB in all at C3, so L2/MALL
// resident) and recomputing both scaled Jacobians with the Jacobian pass's
// own arithmetic (jac_record).  A gathered-F formulation fetched a fresh
// 144-B F record per pair from a 293-MB array (~2.9 GB of HBM traffic per
// launch at C3); this one trades that for ~320 fp64 ops per pair.  The
// block's lanes end with a fixed-order recursive-halving reduction, so S is
// bitwise reproducible run to run.
constexpr int kCamS = 50;  // R 9 | dR/dw 27 | t 3 | K 5 | scale 6

__device__ __forceinline__ void stage_cam(double* cs, int c, const double* __restrict__ camR,
                                          const double* __restrict__ cam, const double* __restrict__ Kc,
                                          const double* __restrict__ scale_c, int l) {
  if (l < 36) cs[l] = camR[size_t(kCamR) * c + l];
  else if (l < 39) cs[l] = cam[6 * size_t(c) + 3 + (l - 36)];
  else if (l < 44) cs[l] = Kc[5 * size_t(c) + (l - 39)];
  else if (l < 50) cs[l] = scale_c[6 * size_t(c) + (l - 44)];
}

// One side of a pair: M = J_X L^-T (2x3, rows m | n) and the projection
// coefficients (a0 a1 a2 | b1 b2) its scaled J_c columns are made of
// (jac_record's Jacobian, with one reciprocal 1/z instead of three divisions).
__device__ __forceinline__ void pair_side_m(const double* cs, const double Xp[3], const double sp[3],
                                            const double Lp[6], double M[6], double ab[5]) {
  const double* cr = cs;
  const double fx = cs[39], sk = cs[40], fy = cs[42];
  const double pc0 = cr[0] * Xp[0] + cr[1] * Xp[1] + cr[2] * Xp[2] + cs[36];
  const double pc1 = cr[3] * Xp[0] + cr[4] * Xp[1] + cr[5] * Xp[2] + cs[37];
  const double pc2 = cr[6] * Xp[0] + cr[7] * Xp[1] + cr[8] * Xp[2] + cs[38];
  const double iz = srcp(shared_div(pc2)), xp = pc0 * iz, yp = pc1 * iz;  // (iz bitwise 1.0 / pc2)
  const double a0 = fx * iz, a1 = sk * iz, a2 = -(fx * xp + sk * yp) * iz;
  const double b1 = fy * iz, b2 = -fy * yp * iz;
  ab[0] = a0; ab[1] = a1; ab[2] = a2; ab[3] = b1; ab[4] = b2;
  double e[6];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    e[j] = (a0 * cr[j] + a1 * cr[3 + j] + a2 * cr[6 + j]) * sp[j];
    e[3 + j] = (b1 * cr[3 + j] + b2 * cr[6 + j]) * sp[j];
  }
  const double l10 = Lp[0], l20 = Lp[1], l21 = Lp[2], i00 = Lp[3], i11 = Lp[4], i22 = Lp[5];
  M[0] = e[0] * i00; M[1] = (e[1] - l10 * M[0]) * i11; M[2] = (e[2] - l20 * M[0] - l21 * M[1]) * i22;
  M[3] = e[3] * i00; M[4] = (e[4] - l10 * M[3]) * i11; M[5] = (e[5] - l20 * M[3] - l21 * M[4]) * i22;
}
// Sums of 32 values over the kSub lanes of a segment by recursive halving
// (see wave_sum32): afterwards lane l holds in v[0 .. kR) the sums of values
// kR * (l % kSub) + r (kSub <= 32, kR = 32 / kSub), or of value l >> 1
// (kSub = 64, kR = 1).
template <int kSub>
__device__ __forceinline__ void seg_reduce32(double (&v)[32], int l) {
#pragma unroll
  for (int d = (kSub >= 64 ? 32 : kSub / 2), n = 32; d >= 1 && n > 1; d >>= 1, n >>= 1) {
    const int h = n / 2;
    const uint64_t m = (l & d) ? ~0ull : 0ull;
#pragma unroll
    for (int j = 0; j < h; ++j) {
      const uint64_t a = __builtin_bit_cast(uint64_t, v[j]), b = __builtin_bit_cast(uint64_t, v[h + j]);
      const double keep = __builtin_bit_cast(double, (b & m) | (a & ~m));
      const double send = __builtin_bit_cast(double, (a & m) | (b & ~m));
      v[j] = keep + __shfl_xor(send, d);
    }
  }
  if (kSub == 64) v[0] += __shfl_xor(v[0], 1);
}
template <int kSub>
__device__ __forceinline__ double seg_sum(double v) {
#pragma unroll
  for (int off = kSub / 2; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// kWpb = 4: one block per workgroup, its pairs dealt over the 4 waves (64
// lanes each, kSub = 64) and the 4 partial blocks added in LDS in wave
// order -- for small reduced systems (few blocks, long pair lists), where
// one wave per block leaves most CUs idle.
template <int kSub, int kWpb = 1>
__global__ __launch_bounds__(kThreads, 3) void k_schur_pts(int64_t n_slots, const int2* __restrict__ blk,
                                                        const int32_t* __restrict__ seg,
                                                        const int32_t* __restrict__ bpts,
                                                        const double* __restrict__ ptS,
                                                        const double* __restrict__ camR,
                                                        const double* __restrict__ cam, const double* __restrict__ Kc,
                                                        const double* __restrict__ scale_c, double* __restrict__ S,
                                                        int ld,
                                                        const int32_t* __restrict__ bperm, const int* __restrict__ gate,
                                                        int* __restrict__ tile_cnt, int nbt, const DiagFold df) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  static_assert(kWpb == 1 || (kWpb == kThreads / 64 && kSub == 64), "4 waves per block take 64 lanes each");
  constexpr int kPer = 64 / kSub;  // blocks per wave
  __shared__ __attribute__((aligned(16))) double cst[kThreads / 64][kPer][2 * kCamS];
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6, g = l / kSub, sl = l % kSub;
  const int64_t wb = kWpb == 1 ? (int64_t(blockIdx.x) * (kThreads / 64) + wv) * kPer : int64_t(blockIdx.x);
  constexpr int kStride = kSub * kWpb;          // pair stride of a lane
  const int lane0 = kWpb == 1 ? sl : 64 * wv + sl;  // this lane's first pair of the block
  // (no early exit: a wave past the end runs empty lists, so every wave
  // reaches the publishing barrier)
  // bperm: the XCD-aware work order of set_problem (nullptr: the plain
  // block order of a small system) -- blocks of one row group
  // in the workgroups one XCD is dealt, descending pair count within a row,
  // so the kPer segments of a wave run lists of nearly equal length); -1 is
  // an empty slot
  auto slot_blk = [&](int64_t k) -> int32_t { return k < n_slots ? (bperm ? bperm[k] : int32_t(k)) : -1; };
  const int32_t bs = slot_blk(wb + g);
  const bool own = bs >= 0;
  const int64_t b = own ? bs : 0;
  const int2 cc = blk[b];
  double* cs1 = cst[wv][g];
  double* cs2 = cs1 + kCamS;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int32_t bq = slot_blk(wb + q);
    const int2 cq = blk[bq >= 0 ? bq : 0];
    stage_cam(cst[wv][q], cq.x, camR, cam, Kc, scale_c, l);
    stage_cam(cst[wv][q] + kCamS, cq.y, camR, cam, Kc, scale_c, l);
  }
  wave_lds_sync();
  if (kWpb > 1 && df.C > 0 && own && cc.x == cc.y && wv == 0) {
    // small system, k_schur_diag_sum folded in (df.C > 0): camera cc.x's
    // diagonal block and rhs first, by the wave that later adds this block's
    // duplicate pairs to it (its stores drained before those loads)
    const double radius = df.radius_dev ? *df.radius_dev : df.radius;
    schur_diag_body(cc.x, df.C, l, df.cam_rng, df.dpart, df.Ucam, df.diag_c, radius, df.add_diag, S, ld, df.n, 1,
                    df.fail, df.ysol, df.n_y);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  const int kb = seg[b], ke = own ? seg[b + 1] : kb;
  double acc[36];
#pragma unroll
  for (int e = 0; e < 36; ++e) acc[e] = 0.0;
  // the segments of a wave run as many steps as the longest list
  int len = ke - kb;
#pragma unroll
  for (int off = kSub; off < 64; off <<= 1) len = max(len, __shfl_xor(len, off));
  // unconditional loads of clamped indices (a past-the-end step reads a real
  // point, masked by w = 0): a predicated load becomes a branch whose join
  // drains vmcnt.  The next step's index is loaded one step ahead, so each
  // step's record gather waits on one dependent load instead of two
  // (263 -> 251 us per C3 launch, S bitwise unchanged).
  int p_nx = bpts[kb + lane0 < ke ? kb + lane0 : 0];
  for (int k0 = 0; k0 < len; k0 += kStride) {
    // the camera constants are re-read from LDS each step (hoisted, they
    // would hold 200 VGPRs)
    asm volatile("" ::: "memory");
    const int k = kb + k0 + lane0;
    const bool valid = k < ke;
    const int p = p_nx;
    p_nx = bpts[k + kStride < ke ? k + kStride : 0];
    const double* r = ptS + size_t(kPtS) * p;
    double q[12];  // X, scale, l10 l20 l21, 1/l_ii (z, the last 32 B, unused here)
#pragma unroll
    for (int f = 0; f < 12; f += 2) {
      const double2 x = ld2(r + f);
      q[f] = x.x; q[f + 1] = x.y;
    }
    const double Xp[3] = {q[0], q[1], q[2]}, sp[3] = {q[3], q[4], q[5]};
    const double Lp[6] = {q[6], q[7], q[8], q[9], q[10], q[11]};
    double M1[6], ab1[5], M2[6], ab2[5];
    pair_side_m(cs1, Xp, sp, Lp, M1, ab1);
    pair_side_m(cs2, Xp, sp, Lp, M2, ab2);
    // (a scheduling fence: without it the LDS reads of both cameras' dR/dw
    // hoist above and the VGPRs spill)
    asm volatile("" ::: "memory");
    const double w = valid ? 1.0 : 0.0;
    const double g00 = (M1[0] * M2[0] + M1[1] * M2[1] + M1[2] * M2[2]) * w;
    const double g01 = (M1[0] * M2[3] + M1[1] * M2[4] + M1[2] * M2[5]) * w;
    const double g10 = (M1[3] * M2[0] + M1[4] * M2[1] + M1[5] * M2[2]) * w;
    const double g11 = (M1[3] * M2[3] + M1[4] * M2[4] + M1[5] * M2[5]) * w;
    // J_c,i = A_i [Q_i | I] diag(sc_i), A_i = dr/dpc = [a0 a1 a2; 0 b1 b2],
    // Q_i = [dR_0 X | dR_1 X | dR_2 X]; so the pair adds
    //   [Q_1 | I]^T H [Q_2 | I],  H = A_1^T G A_2 (3x3),
    // and the Jacobi scales are applied once per block, at the store.
    double H[3][3];
    {
      const double t00 = g00 * ab2[0], t01 = g00 * ab2[1] + g01 * ab2[3], t02 = g00 * ab2[2] + g01 * ab2[4];
      const double t10 = g10 * ab2[0], t11 = g10 * ab2[1] + g11 * ab2[3], t12 = g10 * ab2[2] + g11 * ab2[4];
      H[0][0] = ab1[0] * t00; H[0][1] = ab1[0] * t01; H[0][2] = ab1[0] * t02;
      H[1][0] = ab1[1] * t00 + ab1[3] * t10; H[1][1] = ab1[1] * t01 + ab1[3] * t11; H[1][2] = ab1[1] * t02 + ab1[3] * t12;
      H[2][0] = ab1[2] * t00 + ab1[4] * t10; H[2][1] = ab1[2] * t01 + ab1[4] * t11; H[2][2] = ab1[2] * t02 + ab1[4] * t12;
    }
    double HQ[3][3];  // H Q_2
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double* D = cs2 + 9 + 9 * k;
      const double q0 = D[0] * Xp[0] + D[1] * Xp[1] + D[2] * Xp[2];
      const double q1 = D[3] * Xp[0] + D[4] * Xp[1] + D[5] * Xp[2];
      const double q2 = D[6] * Xp[0] + D[7] * Xp[1] + D[8] * Xp[2];
#pragma unroll
      for (int i = 0; i < 3; ++i) HQ[i][k] = H[i][0] * q0 + H[i][1] * q1 + H[i][2] * q2;
    }
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const double* D = cs1 + 9 + 9 * u;
      const double q0 = D[0] * Xp[0] + D[1] * Xp[1] + D[2] * Xp[2];
      const double q1 = D[3] * Xp[0] + D[4] * Xp[1] + D[5] * Xp[2];
      const double q2 = D[6] * Xp[0] + D[7] * Xp[1] + D[8] * Xp[2];
#pragma unroll
      for (int v = 0; v < 3; ++v) {
        acc[6 * u + v] += q0 * HQ[0][v] + q1 * HQ[1][v] + q2 * HQ[2][v];
        acc[6 * u + 3 + v] += q0 * H[0][v] + q1 * H[1][v] + q2 * H[2][v];
      }
    }
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int v = 0; v < 3; ++v) {
        acc[6 * (3 + u) + v] += HQ[u][v];
        acc[6 * (3 + u) + 3 + v] += H[u][v];
      }
  }
  double v32[32];
#pragma unroll
  for (int e = 0; e < 32; ++e) v32[e] = acc[e];
  seg_reduce32<kSub>(v32, l);
  double t32 = seg_sum<kSub>(acc[32]), t33 = seg_sum<kSub>(acc[33]), t34 = seg_sum<kSub>(acc[34]),
         t35 = seg_sum<kSub>(acc[35]);
  if (kWpb > 1) {
    // the waves' partial blocks, added in wave order by wave 0
    __shared__ double red[kWpb][36];
    if (!(sl & 1)) red[wv][sl >> 1] = v32[0];
    if (sl == 0) { red[wv][32] = t32; red[wv][33] = t33; red[wv][34] = t34; red[wv][35] = t35; }
    __syncthreads();
    if (wv != 0) return;
    if (!(sl & 1)) {
      double a = red[0][sl >> 1];
#pragma unroll
      for (int q = 1; q < kWpb; ++q) a += red[q][sl >> 1];
      v32[0] = a;
    }
    if (sl < 4) {
      double a = red[0][32 + sl];
#pragma unroll
      for (int q = 1; q < kWpb; ++q) a += red[q][32 + sl];
      if (sl == 0) t32 = a; else if (sl == 1) t33 = a; else if (sl == 2) t34 = a; else t35 = a;
    }
  }
  if (own) {
    // a diagonal block (same-camera duplicate pairs only) is added to what
    // k_schur_diag_sum wrote before this launch, else stored
    double* Sb = S + size_t(6 * cc.x) * ld + 6 * size_t(cc.y);
    const bool add = cc.x == cc.y;
    // the Jacobi scales of both cameras (staged in LDS by this segment)
    const double* sc1 = cst[wv][g] + 44;
    const double* sc2 = sc1 + kCamS;
    auto put = [&](int e, double v) {
      double* q = Sb + size_t(e / 6) * ld + e % 6;
      v = v * sc1[e / 6] * sc2[e % 6];
      v = add ? *q - v : -v;
      // overlapped with the factorisation: write-through, counted per tile
      if (tile_cnt) __hip_atomic_store(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else *q = v;
    };
    constexpr int kR = kSub >= 32 ? 1 : 32 / kSub;
    if (kSub == 64) {
      if (!(sl & 1)) put(sl >> 1, v32[0]);
    } else {
#pragma unroll
      for (int r = 0; r < kR; ++r) put(kR * sl + r, v32[r]);
    }
    if (sl < 4) put(32 + sl, sl == 0 ? t32 : sl == 1 ? t33 : sl == 2 ? t34 : t35);
  }
  if (tile_cnt) {
    // Schur/Cholesky overlap: the block's entries are out (write-through,
    // drained by this wave), then one lane per block counts it into every
    // 64x64 tile its 6x6 footprint touches; a helper of k_chol_fused reads a
    // tile once its count is complete (set_problem's tile_exp)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (own && sl == 0) {
      const int r0 = 6 * cc.y, c0 = 6 * cc.x;
      for (int I = r0 / 64; I <= (r0 + 5) / 64; ++I)
        for (int J = c0 / 64; J <= (c0 + 5) / 64; ++J)
          __hip_atomic_fetch_add(tile_cnt + I * nbt + J, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// A register-lighter form of k_schur_pts (built to be
// measured; SFM_SCHUR_HALVES=1): two passes over every pair list, pass kHalf
// accumulating only rows 3 kHalf .. 3 kHalf + 2 of the 6x6 block (18 sums
// instead of 36, 36 VGPRs fewer), at __launch_bounds__(kThreads, 4) for a
// fourth wave per SIMD.  Pass 1's rows [H Q_2 | H] need no Q_1; pass 0 does
// everything but half of the accumulation.  Every entry takes the full
// kernel's operations in its order, and the lane reduction pairs lanes in the
// same tree, so S is bitwise the one-pass kernel's.
template <int kSub, int kHalf>
__global__ __launch_bounds__(kThreads, 4) void k_schur_pts_half(int64_t n_slots, const int2* __restrict__ blk,
                                                             const int32_t* __restrict__ seg,
                                                             const int32_t* __restrict__ bpts,
                                                             const double* __restrict__ ptS,
                                                             const double* __restrict__ camR,
                                                             const double* __restrict__ cam,
                                                             const double* __restrict__ Kc,
                                                             const double* __restrict__ scale_c, double* __restrict__ S,
                                                             int ld, const int32_t* __restrict__ bperm,
                                                             const int* __restrict__ gate) {
  if (gate && *gate == 0) return;
  constexpr int kPer = 64 / kSub;
  __shared__ __attribute__((aligned(16))) double cst[kThreads / 64][kPer][2 * kCamS];
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6, g = l / kSub, sl = l % kSub;
  const int64_t wb = (int64_t(blockIdx.x) * (kThreads / 64) + wv) * kPer;
  auto slot_blk = [&](int64_t k) -> int32_t { return k < n_slots ? (bperm ? bperm[k] : int32_t(k)) : -1; };
  const int32_t bs = slot_blk(wb + g);
  const bool own = bs >= 0;
  const int64_t b = own ? bs : 0;
  const int2 cc = blk[b];
  double* cs1 = cst[wv][g];
  double* cs2 = cs1 + kCamS;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int32_t bq = slot_blk(wb + q);
    const int2 cq = blk[bq >= 0 ? bq : 0];
    stage_cam(cst[wv][q], cq.x, camR, cam, Kc, scale_c, l);
    stage_cam(cst[wv][q] + kCamS, cq.y, camR, cam, Kc, scale_c, l);
  }
  wave_lds_sync();
  const int kb = seg[b], ke = own ? seg[b + 1] : kb;
  double acc[18];
#pragma unroll
  for (int e = 0; e < 18; ++e) acc[e] = 0.0;
  int len = ke - kb;
#pragma unroll
  for (int off = kSub; off < 64; off <<= 1) len = max(len, __shfl_xor(len, off));
  int p_nx = bpts[kb + sl < ke ? kb + sl : 0];
  for (int k0 = 0; k0 < len; k0 += kSub) {
    asm volatile("" ::: "memory");
    const int k = kb + k0 + sl;
    const bool valid = k < ke;
    const int p = p_nx;
    p_nx = bpts[k + kSub < ke ? k + kSub : 0];
    const double* r = ptS + size_t(kPtS) * p;
    double q[12];
#pragma unroll
    for (int f = 0; f < 12; f += 2) {
      const double2 x = ld2(r + f);
      q[f] = x.x; q[f + 1] = x.y;
    }
    const double Xp[3] = {q[0], q[1], q[2]}, sp[3] = {q[3], q[4], q[5]};
    const double Lp[6] = {q[6], q[7], q[8], q[9], q[10], q[11]};
    double M1[6], ab1[5], M2[6], ab2[5];
    pair_side_m(cs1, Xp, sp, Lp, M1, ab1);
    pair_side_m(cs2, Xp, sp, Lp, M2, ab2);
    asm volatile("" ::: "memory");
    const double w = valid ? 1.0 : 0.0;
    const double g00 = (M1[0] * M2[0] + M1[1] * M2[1] + M1[2] * M2[2]) * w;
    const double g01 = (M1[0] * M2[3] + M1[1] * M2[4] + M1[2] * M2[5]) * w;
    const double g10 = (M1[3] * M2[0] + M1[4] * M2[1] + M1[5] * M2[2]) * w;
    const double g11 = (M1[3] * M2[3] + M1[4] * M2[4] + M1[5] * M2[5]) * w;
    double H[3][3];
    {
      const double t00 = g00 * ab2[0], t01 = g00 * ab2[1] + g01 * ab2[3], t02 = g00 * ab2[2] + g01 * ab2[4];
      const double t10 = g10 * ab2[0], t11 = g10 * ab2[1] + g11 * ab2[3], t12 = g10 * ab2[2] + g11 * ab2[4];
      H[0][0] = ab1[0] * t00; H[0][1] = ab1[0] * t01; H[0][2] = ab1[0] * t02;
      H[1][0] = ab1[1] * t00 + ab1[3] * t10; H[1][1] = ab1[1] * t01 + ab1[3] * t11; H[1][2] = ab1[1] * t02 + ab1[3] * t12;
      H[2][0] = ab1[2] * t00 + ab1[4] * t10; H[2][1] = ab1[2] * t01 + ab1[4] * t11; H[2][2] = ab1[2] * t02 + ab1[4] * t12;
    }
    double HQ[3][3];
#pragma unroll
    for (int kq = 0; kq < 3; ++kq) {
      const double* D = cs2 + 9 + 9 * kq;
      const double q0 = D[0] * Xp[0] + D[1] * Xp[1] + D[2] * Xp[2];
      const double q1 = D[3] * Xp[0] + D[4] * Xp[1] + D[5] * Xp[2];
      const double q2 = D[6] * Xp[0] + D[7] * Xp[1] + D[8] * Xp[2];
#pragma unroll
      for (int i = 0; i < 3; ++i) HQ[i][kq] = H[i][0] * q0 + H[i][1] * q1 + H[i][2] * q2;
    }
    if (kHalf == 0) {
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const double* D = cs1 + 9 + 9 * u;
        const double q0 = D[0] * Xp[0] + D[1] * Xp[1] + D[2] * Xp[2];
        const double q1 = D[3] * Xp[0] + D[4] * Xp[1] + D[5] * Xp[2];
        const double q2 = D[6] * Xp[0] + D[7] * Xp[1] + D[8] * Xp[2];
#pragma unroll
        for (int v = 0; v < 3; ++v) {
          acc[6 * u + v] += q0 * HQ[0][v] + q1 * HQ[1][v] + q2 * HQ[2][v];
          acc[6 * u + 3 + v] += q0 * H[0][v] + q1 * H[1][v] + q2 * H[2][v];
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < 3; ++u)
#pragma unroll
        for (int v = 0; v < 3; ++v) {
          acc[6 * u + v] += HQ[u][v];
          acc[6 * u + 3 + v] += H[u][v];
        }
    }
  }
  double v32[32];
#pragma unroll
  for (int e = 0; e < 32; ++e) v32[e] = e < 18 ? acc[e] : 0.0;
  seg_reduce32<kSub>(v32, l);
  if (own) {
    double* Sb = S + size_t(6 * cc.x) * ld + 6 * size_t(cc.y);
    const bool add = cc.x == cc.y;
    const double* sc1 = cst[wv][g] + 44;
    const double* sc2 = sc1 + kCamS;
    auto put = [&](int e, double v) {
      double* q = Sb + size_t(e / 6) * ld + e % 6;
      v = v * sc1[e / 6] * sc2[e % 6];
      *q = add ? *q - v : -v;
    };
    constexpr int kR = kSub >= 32 ? 1 : 32 / kSub;
    if (kSub == 64) {
      if (!(sl & 1) && (sl >> 1) < 18) put(18 * kHalf + (sl >> 1), v32[0]);
    } else {
#pragma unroll
      for (int r = 0; r < kR; ++r)
        if (kR * sl + r < 18) put(18 * kHalf + kR * sl + r, v32[r]);
    }
  }
}

// Diagonal blocks and rhs from k_obs_prep_rc's per-wave partials: camera c's
// waves are positions cam_rng[2c]/64 .. (run end)/64, summed in order.
//   S_cc += [rank 0] (U_c + D_c^2) - sum F F^T,   S[c][n] = sum J_c^T (r - h)
__global__ __launch_bounds__(64) void k_schur_diag_sum(const int32_t* __restrict__ cam_rng,
                                                       const double* __restrict__ dpart,
                                                       const double* __restrict__ Ucam,
                                                       const double* __restrict__ diag_c, double radius,
                                                       int add_diag, double* __restrict__ S, int ld, int n,
                                                       int init, const int* __restrict__ gate, const double* __restrict__ radius_dev,
                                                       int* __restrict__ fail, unsigned long long* __restrict__ ysol, int n_y) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  if (radius_dev) radius = *radius_dev;  // the device LM loop's current radius
  schur_diag_body(blockIdx.x, gridDim.x, threadIdx.x, cam_rng, dpart, Ucam, diag_c, radius, add_diag, S, ld, n, init,
                  fail, ysol, n_y);
}

// Packed form of the reduced system for the cross-rank all-reduce: row i
// of the row-major upper triangle, columns i..n (the rhs column n
// included), at offset i(n+1) - i(i-1)/2.  Half the bytes of the full ld^2
// image, and none of the stale factor entries outside the triangle.
__device__ __forceinline__ size_t packed_row(int i, int n) { return size_t(i) * (n + 1) - size_t(i) * (i - 1) / 2; }

__global__ void k_pack_upper(const double* __restrict__ S, int ld, int n, double* __restrict__ P, const int* __restrict__ gate) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  const int i = blockIdx.x;
  const double* row = S + size_t(i) * ld;
  double* dst = P + packed_row(i, n) - i;
  for (int j = i + threadIdx.x; j <= n; j += blockDim.x) dst[j] = row[j];
}

__global__ void k_unpack_upper(const double* __restrict__ P, int ld, int n, double* __restrict__ S, const int* __restrict__ gate) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  const int i = blockIdx.x;
  double* row = S + size_t(i) * ld;
  const double* src = P + packed_row(i, n) - i;
  for (int j = i + threadIdx.x; j <= n; j += blockDim.x) row[j] = src[j];
}

// dst = scale * src, skipped with its phase (the device LM loop's
// out-of-place collectives copy their result back through this; scale is
// the emulated rank count of the tests, a power of two: exact).
__global__ void k_gated_copy(const double* src, double* dst, int64_t n, double scale, const int* __restrict__ gate) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    dst[i] = src[i] * scale;
}

// Identity padding beyond the augmented row n (column-major lower view).
// Identity padding of the augmented system, and the Cholesky failure flag
// cleared (saves the separate memset dispatch before k_chol_fused).
__global__ void k_pad_init(double* __restrict__ S, int ld, int n, int* __restrict__ fail,
                           unsigned long long* __restrict__ ysol, int n_y, const int* __restrict__ gate) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  const int j = blockIdx.x;
  if (j == 0 && threadIdx.x == 0) *fail = 0;
  if (threadIdx.x == 0 && j < n_y) ysol[j] = kYSentinel;  // k_backsolve's "not yet produced"
  for (int i = (j > n ? j : n + 1) + threadIdx.x; i < ld; i += blockDim.x) S[size_t(j) * ld + i] = (i == j) ? 1.0 : 0.0;
  if (j == n && threadIdx.x == 0) S[size_t(n) * ld + n] = 1.0;
}

// ---------------------------------------------------------------------------
// Camera candidate: delta = -y (scaled space), dx = s * delta.
__global__ __launch_bounds__(kThreads) void k_cam_update(int C, const double* __restrict__ cam,
                                                         const double* __restrict__ ysol,
                                                         const double* __restrict__ scale_c,
                                                         double* __restrict__ cam_new, double* __restrict__ camRn,
                                                         double* __restrict__ part_step, double* __restrict__ part_bad, const int* __restrict__ gate) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  __shared__ double sh[4];
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  double st = 0.0, bad = 0.0;
  if (c < C) cam_update_one(c, cam, ysol, scale_c, cam_new, camRn, st, bad);
  const double rs = block_reduce(st, sh, false);
  if (threadIdx.x == 0 && part_step) part_step[blockIdx.x] = rs;
  const double rb = block_reduce(bad, sh, true);
  if (threadIdx.x == 0) part_bad[blockIdx.x] = rb;
}

// Pose-only step (mode POSE_ONLY: BAPoseFunctor, CTracker.cpp:607-636,
// 684-687).  With the points held constant no point block is eliminated and
// the normal matrix is block diagonal: one 6x6 block U_c + D_c^2 per camera
// (R_c and t_c are coupled through their shared residuals), right-hand side
// J_c^T r.  One lane per camera, in-register Cholesky; a non-positive or
// non-finite pivot sets fail bit 0, as a failed dense LLT does.
__global__ __launch_bounds__(kThreads) void k_cam_solve(int C, const double* __restrict__ Ucam,
                                                        const double* __restrict__ diag_c, double radius,
                                                        double* __restrict__ ysol, int* __restrict__ fail, const int* __restrict__ gate, const double* __restrict__ radius_dev) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  if (radius_dev) radius = *radius_dev;  // the device LM loop's current radius
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double* U = Ucam + size_t(kUcam) * c;
  double L[21], y[6];
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    double s = U[up6(j, j)] + diag_c[6 * c + j] / radius;
#pragma unroll
    for (int k = 0; k < j; ++k) s -= L[up6(k, j)] * L[up6(k, j)];
    ok = ok && s > 0.0 && isfinite(s);
    const double ljj = sqrt(s);
    L[up6(j, j)] = ljj;
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      double a = U[up6(j, i)];
#pragma unroll
      for (int k = 0; k < j; ++k) a -= L[up6(k, i)] * L[up6(k, j)];
      L[up6(j, i)] = a / ljj;  // L(i, j) kept at the upper index (j, i)
    }
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double s = U[21 + i];
#pragma unroll
    for (int k = 0; k < i; ++k) s -= L[up6(k, i)] * y[k];
    y[i] = s / L[up6(i, i)];
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    double s = y[i];
#pragma unroll
    for (int k = i + 1; k < 6; ++k) s -= L[up6(i, k)] * y[k];
    y[i] = s / L[up6(i, i)];
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) ysol[6 * c + i] = y[i];
  if (!ok) atomicOr(fail, 1);
}

// ---------------------------------------------------------------------------
// Point back substitution, model cost change and candidate cost, in three
// passes so that only per-point quantities are gathered:
//   A (k_backsub_a_rc, camera-major, one wavefront = 64 positions of one
//       camera): e_o = J_c,o y_c,  u_o = M_o^T e_o  -> eu at the
//       observation's point-major slot (J and M recomputed)
//   B (one lane per point):  y_p = L^-T (z_p - sum_o u_o),  delta_p = -y_p,
//       X_new = X + s_p delta_p, |dX|^2, finite check  -> ypt[p], X_new
//   C (camera-major): candidate residual at (cam_new, X_new).
// The model cost change (ceres trust_region_minimizer's -q.(r + q/2) with
// q_o = -(e_o + J_X,o y_p)) is split between A and B (see below).
// Camera runs are padded to whole wavefronts, so a wavefront never spans two
// cameras (its camera comes from wcam) and padding lanes are masked.

__global__ __launch_bounds__(kThreads) void k_backsub_b(int P, const int32_t* __restrict__ pt_off,
                                                        const double* __restrict__ eu,
                                                        const int32_t* __restrict__ eu_pos,
                                                        const double* __restrict__ ptL,
                                                        const double* __restrict__ ptV,
                                                        const double* __restrict__ scale_p,
                                                        const double* __restrict__ X, double* __restrict__ X_new,
                                                        double* __restrict__ ypt, double* __restrict__ part_step,
                                                        double* __restrict__ part_bad,
                                                        double* __restrict__ part_model, const int* __restrict__ gate) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  __shared__ double sh[4];
  // XCD point-slice order (pt_xcd_blocks): workgroups go round-robin to the
  // 8 XCDs, so workgroup b takes points of slice b % 8, the slice whose
  // observations k_backsub_a_rc ran (and wrote u) on that XCD; X_new / y_p
  // land in the L2 that k_backsub_c's same-slice chunks read them from
  const int x = blockIdx.x & 7;
  const int pb = int((int64_t(x) * P + 7) / 8), pe = int((int64_t(x + 1) * P + 7) / 8);
  const int p = pb + (blockIdx.x >> 3) * blockDim.x + threadIdx.x;
  double st = 0.0, bad = 0.0, model = 0.0;
  if (p < pe) {
    const double* L = ptL + size_t(kPtL) * p;
    const double l00 = L[0], l10 = L[1], l11 = L[2], l20 = L[3], l21 = L[4], l22 = L[5];
    double w0 = L[6], w1 = L[7], w2 = L[8];
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;  // sum of u = L^-1 J_X^T e
    const int q0 = pt_off[p], q1 = pt_off[p + 1];
    // pass A's u: at the point-major slot, or (eu_pos) at the camera-major
    // position.  Four observations' positions, then their u, are loaded
    // before any is summed (two memory round trips per four instead of two
    // per observation: what bounds keyframe-sized problems); the sums still
    // run in observation order.
    int q = q0;
    for (; q + 4 <= q1; q += 4) {
      int ps[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) ps[j] = eu_pos ? eu_pos[q + j] : q + j;
      double2 a[4];
      double b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double* u = eu + 4 * size_t(ps[j]);
        a[j] = ld2(u);
        b[j] = u[2];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        w0 -= a[j].x;
        w1 -= a[j].y;
        w2 -= b[j];
        s0 += a[j].x; s1 += a[j].y; s2 += b[j];
      }
    }
    for (; q < q1; ++q) {
      const double* u = eu + 4 * (eu_pos ? size_t(eu_pos[q]) : size_t(q));
      const double2 u01 = ld2(u);
      const double u2 = u[2];
      w0 -= u01.x;
      w1 -= u01.y;
      w2 -= u2;
      s0 += u01.x; s1 += u01.y; s2 += u2;
    }
    const double y2 = w2 / l22;
    const double y1 = (w1 - l21 * y2) / l11;
    const double y0 = (w0 - l10 * y1 - l20 * y2) / l00;
    if (!isfinite(y0) || !isfinite(y1) || !isfinite(y2)) bad = 1.0;
    // Model cost change, ceres' -sum_o m_o.(r_o + m_o/2) with m_o = -(e_o +
    // J_X,o y_p), split by observation and point:
    //   sum_o (e.r - |e|^2/2)                      (k_backsub_a_rc)
    //   + y.g_p - y.h_p - y^T V0_p y / 2           (here, per point)
    // with g_p = sum J_X^T r and V0_p = sum J_X^T J_X (ptV, k_point_eval_rc)
    // and h_p = sum J_X^T e = L_p sum u.  The candidate pass then reads no
    // Jacobian record at all.
    {
      const double* v = ptV + size_t(kPtV) * p;
      const double h0 = l00 * s0, h1 = l10 * s0 + l11 * s1, h2 = l20 * s0 + l21 * s1 + l22 * s2;
      const double yVy = v[0] * y0 * y0 + v[2] * y1 * y1 + v[5] * y2 * y2 +
                         2.0 * (v[1] * y0 * y1 + v[3] * y0 * y2 + v[4] * y1 * y2);
      model = y0 * (v[6] - h0) + y1 * (v[7] - h1) + y2 * (v[8] - h2) - 0.5 * yVy;
    }
    const double yp[3] = {y0, y1, y2};
    for (int k = 0; k < 3; ++k) {
      const double x = X[3 * size_t(p) + k];
      const double xn = x + scale_p[3 * size_t(p) + k] * (-yp[k]);
      const double d = x - xn;
      st += d * d;
      X_new[3 * size_t(p) + k] = xn;
      ypt[3 * size_t(p) + k] = yp[k];
    }
  }
  double r = block_reduce(st, sh, false);
  if (threadIdx.x == 0) part_step[blockIdx.x] = r;
  r = block_reduce(bad, sh, true);
  if (threadIdx.x == 0) part_bad[blockIdx.x] = r;
  r = block_reduce(model, sh, false);
  if (threadIdx.x == 0) part_model[blockIdx.x] = r;
}

// (chunks in the XCD point-slice order of k_obs_prep_rc, one per wave: the
// X_new gathers stay in the slice k_backsub_b wrote on this XCD)
__global__ __launch_bounds__(kThreads) void k_backsub_c(const int32_t* __restrict__ grp_off,
                                                        const int4* __restrict__ chunks,
                                                        const int32_t* __restrict__ cam_obs,
                                                        const int32_t* __restrict__ cm_p,
                                                        const double* __restrict__ uv_cm,
                                                        const double* __restrict__ Kc,
                                                        const double* __restrict__ X_new,
                                                        const double* __restrict__ camRn,
                                                        double* __restrict__ part_cost, const int* __restrict__ gate) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  __shared__ double sh[4];
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const XcdChunks xc = xcd_chunks(grp_off, wave_uniform(wv));
  double ncost = 0.0;
  if (xc.t < xc.end) {  // wave-uniform
    const int4 ch = chunks[xc.t];
    const int64_t i = int64_t(__builtin_amdgcn_readfirstlane(ch.y)) + l;
    const int c = __builtin_amdgcn_readfirstlane(ch.x);  // wave-uniform: scalar camera loads
    const bool real = cam_obs[i] >= 0;
    const int p = cm_p[i];
    // candidate residual at (cam_new, X_new)
    const double* Rn = camRn + 12 * size_t(c);
    const double Xn0 = X_new[3 * size_t(p)], Xn1 = X_new[3 * size_t(p) + 1], Xn2 = X_new[3 * size_t(p) + 2];
    double pc[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) pc[k] = Rn[3 * k] * Xn0 + Rn[3 * k + 1] * Xn1 + Rn[3 * k + 2] * Xn2 + Rn[9 + k];
    const SharedDiv dz = shared_div(pc[2]);  // (bitwise the two divisions)
    const double xp = sdiv(dz, pc[0]), ypj = sdiv(dz, pc[1]);
    const double* k5 = Kc + 5 * size_t(c);
    const double2 uvo = ld2(uv_cm + 2 * i);
    const double rn0 = k5[0] * xp + k5[1] * ypj + k5[2] - uvo.x;
    const double rn1 = k5[3] * ypj + k5[4] - uvo.y;
    if (real) ncost = 0.5 * (rn0 * rn0 + rn1 * rn1);
  }
  const double r = block_reduce(ncost, sh, false);
  if (threadIdx.x == 0) part_cost[blockIdx.x] = r;
}

// Fixed-order final reduction of one partial slot.
// Several fixed-order reductions in one launch (workgroup i = job i), and
// the Cholesky failure flag copied next to the scalars (an int in the slot
// after them), so one launch and one copy end each LM phase instead of up
// to seven launches and two copies (~5-6 us of dispatch each).
__global__ __launch_bounds__(1024) void k_reduce_batch(const double* __restrict__ partials, int64_t max_blocks,
                                                       ReduceBatch b, double* __restrict__ scal,
                                                       const int* __restrict__ fail, const int* __restrict__ gate) {
  if (gate && *gate == 0) return;  // device LM loop: phase skipped
  __shared__ double sh[16];
  reduce_batch_job(partials, max_blocks, b.job[blockIdx.x], scal, blockIdx.x == 0 ? fail : nullptr, sh);
}

__global__ __launch_bounds__(1024) void k_reduce(const double* __restrict__ src, int nb, int op,
                                                 double* __restrict__ dst) {
  __shared__ double sh[16];
  double v = 0.0;
  for (int i = threadIdx.x; i < nb; i += 1024) v = op ? fmax(v, src[i]) : v + src[i];
  v = op ? wave_max(v) : wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) sh[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double r = sh[0];
    for (int i = 1; i < 16; ++i) r = op ? fmax(r, sh[i]) : r + sh[i];
    *dst = r;
  }
}

}  // namespace

int blocks_for(int64_t n, int threads) { return int((n + threads - 1) / threads); }

static inline double* slot(const DevProblem& d, int s) { return d.partials + size_t(s) * d.max_blocks; }

void launch_cam_prep(const DevProblem& d, double* cam, bool count_norm, hipStream_t s) {
  k_cam_prep<<<blocks_for(d.C, kThreads), kThreads, 0, s>>>(d.C, cam, d.camR, count_norm ? slot(d, kPXNormCam) : nullptr, d.gate,
                                                            nullptr, nullptr, nullptr, 0);
}
void launch_cam_prep_accept(const DevProblem& d, bool count_norm, int grid, hipStream_t s) {
  k_cam_prep<<<std::max(grid, blocks_for(d.C, kThreads)), kThreads, 0, s>>>(
      d.C, d.cam, d.camR, count_norm ? slot(d, kPXNormCam) : nullptr, d.gate, d.cam_new, d.X_new, d.X, 3 * int64_t(d.P));
}
void launch_jacobian(const DevProblem& d, bool scaled, hipStream_t s, bool write_records) {
  // the record-writing variant (evaluate API) runs on its own, smaller grid
  if (write_records)
    k_jacobian<true><<<d.jac_blocks_rec, kThreads, 0, s>>>(d.jgrp, d.jchunks, d.cm_p, d.uv_cm, d.Kc, d.cam, d.camR,
                                                           d.X, d.scale_c, d.scale_p, scaled ? 1 : 0, d.jrec,
                                                           slot(d, kPCost), d.jpart, d.gate);
  else
    k_jacobian<false><<<d.jac_blocks, kThreads, 0, s>>>(d.jgrp, d.jchunks, d.cm_p, d.uv_cm, d.Kc, d.cam, d.camR, d.X,
                                                        d.scale_c, d.scale_p, scaled ? 1 : 0, d.jrec, slot(d, kPCost),
                                                        d.jpart, d.gate);
}
void launch_cam_reduce(const DevProblem& d, hipStream_t s) {
  if (d.C) k_cam_sum<<<d.C, 64, 0, s>>>(d.cam_rng, d.jpart, d.Ucam, d.gate);
}
static CamFold cam_fold(const DevProblem& d, int mode, bool count_grad) {
  return CamFold{d.cam_rng, d.jpart, d.Ucam, d.scale_c, d.diag_c, d.min_diag, d.max_diag, mode, d.C,
                 count_grad ? slot(d, kPGradCam) : nullptr};
}
void launch_cam_sum_finalize(const DevProblem& d, int mode, bool count_grad, hipStream_t s) {
  if (d.C) k_cam_sum_finalize<<<d.C, 64, 0, s>>>(cam_fold(d, mode, count_grad), d.gate);
}
bool launch_point_eval_with_cams(const DevProblem& d, int mode, bool count_grad, hipStream_t s) {
  if (d.P == 0 || d.C == 0 || d.C > 64) return false;
  const int nb = blocks_for(d.P, kThreads) + (d.C + kThreads / 64 - 1) / (kThreads / 64);
  k_point_eval_lds<64><<<nb, kThreads, 0, s>>>(d.P, d.C, d.pt_off, d.cam_pm, d.uv_pm, d.camR, d.cam, d.Kc, d.X,
                                               d.scale_p, d.diag_p, d.ptV, d.min_diag, d.max_diag, mode, 0,
                                               slot(d, kPGradPt), slot(d, kPXNormPt), d.gate,
                                               cam_fold(d, mode, count_grad));
  return true;
}
void launch_cam_finalize(const DevProblem& d, int mode, bool reuse_diag, bool count_grad, hipStream_t s) {
  k_cam_finalize<<<blocks_for(d.C, kThreads), kThreads, 0, s>>>(d.C, d.Ucam, d.scale_c, d.diag_c, d.min_diag, d.max_diag, mode,
                                                               reuse_diag ? 1 : 0,
                                                               count_grad ? slot(d, kPGradCam) : nullptr, d.gate);
}
// A/B switch, read once (SFM_PE_GROUPS1=1: the 256-thread point pass).
static bool env_flag_k(const char* name) {
  const char* v = std::getenv(name);
  return v && v[0] == '1';
}
void launch_point_eval(const DevProblem& d, int mode, bool reuse_diag, hipStream_t s) {
  if (d.P == 0) return;
  const int nb = blocks_for(d.P, kThreads);
  // camera constants from LDS while they fit (C3: 500 cameras, 68 KB)
#define SFM_PE_LDS(M_)                                                                                              \
  k_point_eval_lds<M_><<<nb, kThreads, 0, s>>>(d.P, d.C, d.pt_off, d.cam_pm, d.uv_pm, d.camR, d.cam, d.Kc, d.X,      \
                                               d.scale_p, d.diag_p, d.ptV, d.min_diag, d.max_diag, mode,           \
                                               reuse_diag ? 1 : 0, slot(d, kPGradPt), slot(d, kPXNormPt), d.gate,    \
                                               CamFold{})
  if (d.C <= 64) SFM_PE_LDS(64);
  else if (d.C <= 512 && !env_flag_k("SFM_PE_GROUPS1"))
    k_point_eval_lds<512, 2><<<blocks_for(d.P, 2 * kThreads), 2 * kThreads, 0, s>>>(
        d.P, d.C, d.pt_off, d.cam_pm, d.uv_pm, d.camR, d.cam, d.Kc, d.X, d.scale_p, d.diag_p, d.ptV, d.min_diag,
        d.max_diag, mode, reuse_diag ? 1 : 0, slot(d, kPGradPt), slot(d, kPXNormPt), d.gate, CamFold{});
  else if (d.C <= 512) SFM_PE_LDS(512);
  else
    k_point_eval_rc<<<nb, kThreads, 0, s>>>(d.P, d.pt_off, d.cam_pm, d.uv_pm, d.camR, d.cam, d.Kc, d.X, d.scale_p,
                                            d.diag_p, d.ptV, d.min_diag, d.max_diag, mode, reuse_diag ? 1 : 0,
                                            slot(d, kPGradPt), slot(d, kPXNormPt), d.gate);
#undef SFM_PE_LDS
}
void launch_point_factor(const DevProblem& d, double radius, hipStream_t s) {
  if (d.P) k_point_factor<<<blocks_for(d.P, kThreads), kThreads, 0, s>>>(d.P, d.ptV, d.diag_p, radius, d.ptL,
                                                                         slot(d, kPBad), d.X, d.scale_p, d.ptS, d.gate, d.radius_dev);
}
void launch_point_prep(const DevProblem& d, double radius, hipStream_t s) {
  launch_point_factor(d, radius, s);
  if (d.N_pad)
    k_obs_prep_rc<<<obs_xcd_blocks(d), kThreads, 0, s>>>(d.jgrp, d.jchunks, d.cm_p, d.uv_cm, d.cam_obs, d.camR, d.cam,
                                                         d.Kc, d.scale_c, d.ptS, d.dpart, d.gate);
}
void launch_schur(const DevProblem& d, double radius, bool add_diag, hipStream_t s) {
  // diagonal blocks + rhs first (k_obs_prep_rc's per-wave partials), then
  // the off-diagonal blocks, which add a block's same-camera duplicate pairs;
  // a small system's block-per-workgroup pass does the first part itself
  // (DiagFold: the workgroup of each diagonal block)
  if (d.schur_wg_blocks && d.n_blk && d.C) {
    const DiagFold f{d.cam_rng, d.dpart, d.Ucam, d.diag_c, radius, d.radius_dev, add_diag ? 1 : 0, d.C, d.n,
                     (d.n + kNB - 1) / kNB * kNB, d.fail, reinterpret_cast<unsigned long long*>(d.ysol)};
    k_schur_pts<64, kThreads / 64><<<int(d.n_bslots), kThreads, 0, s>>>(d.n_bslots, d.blk, d.seg, d.bpts, d.ptS,
                                                                       d.camR, d.cam, d.Kc, d.scale_c, d.S, d.ld,
                                                                       d.bperm, d.gate, nullptr, d.nblk, f);
    return;
  }
  launch_schur_diag(d, radius, add_diag, s);
  launch_schur_offdiag(d, nullptr, s);
}
void launch_schur_diag(const DevProblem& d, double radius, bool add_diag, hipStream_t s) {
  if (d.C)
    k_schur_diag_sum<<<d.C, 64, 0, s>>>(d.cam_rng, d.dpart, d.Ucam, d.diag_c, radius, add_diag ? 1 : 0, d.S, d.ld,
                                        d.n, 1, d.gate, d.radius_dev, d.fail,
                                        reinterpret_cast<unsigned long long*>(d.ysol), (d.n + kNB - 1) / kNB * kNB);
}
// tile_cnt != nullptr: overlapped with k_chol_fused (compute_step_enqueue):
// the blocks in their plain order (camera-major: the factor's tile columns
// complete left to right) and counted per tile
void launch_schur_offdiag(const DevProblem& d, int* tile_cnt, hipStream_t s) {
  if (!d.n_blk) return;
  const int64_t n_slots = tile_cnt ? d.n_blk : d.n_bslots;
  const int32_t* bperm = tile_cnt ? nullptr : d.bperm;
  const int sub = d.schur_pts_sub, per = 64 / sub * (kThreads / 64);
  const int nb = int((n_slots + per - 1) / per);
#define SFM_PTS(S_)                                                                                           \
  k_schur_pts<S_><<<nb, kThreads, 0, s>>>(n_slots, d.blk, d.seg, d.bpts, d.ptS, d.camR, d.cam, d.Kc, d.scale_c, \
                                          d.S, d.ld, bperm, d.gate, tile_cnt, d.nblk, DiagFold{})
  if (d.schur_wg_blocks) {  // small systems: one block per workgroup
    k_schur_pts<64, kThreads / 64><<<int(n_slots), kThreads, 0, s>>>(n_slots, d.blk, d.seg, d.bpts, d.ptS,
                                                                    d.camR, d.cam, d.Kc, d.scale_c, d.S, d.ld,
                                                                    bperm, d.gate, tile_cnt, d.nblk, DiagFold{});
    return;
  }
  static const bool halves = [] {
    const char* e = std::getenv("SFM_SCHUR_HALVES");
    return e && e[0] == '1';
  }();
  if (halves && !tile_cnt) {
#define SFM_PTS_H(S_, H_)                                                                                       \
  k_schur_pts_half<S_, H_><<<nb, kThreads, 0, s>>>(n_slots, d.blk, d.seg, d.bpts, d.ptS, d.camR, d.cam, d.Kc, \
                                                   d.scale_c, d.S, d.ld, bperm, d.gate)
    if (sub == 8) { SFM_PTS_H(8, 0); SFM_PTS_H(8, 1); }
    else if (sub == 16) { SFM_PTS_H(16, 0); SFM_PTS_H(16, 1); }
    else if (sub == 32) { SFM_PTS_H(32, 0); SFM_PTS_H(32, 1); }
    else { SFM_PTS_H(64, 0); SFM_PTS_H(64, 1); }
#undef SFM_PTS_H
    return;
  }
  if (sub == 8) SFM_PTS(8);
  else if (sub == 16) SFM_PTS(16);
  else if (sub == 32) SFM_PTS(32);
  else SFM_PTS(64);
#undef SFM_PTS
}
void launch_pack_upper(const DevProblem& d, bool unpack, hipStream_t s) {
  if (d.n == 0) return;
  if (unpack) k_unpack_upper<<<d.n, 256, 0, s>>>(d.Spack, d.ld, d.n, d.S, d.gate);
  else k_pack_upper<<<d.n, 256, 0, s>>>(d.S, d.ld, d.n, d.Spack, d.gate);
}
void launch_gated_copy(const double* src, double* dst, int64_t n, double scale, const int32_t* gate, hipStream_t s) {
  if (n <= 0) return;
  const int grid = int(std::min<int64_t>(1024, (n + 255) / 256));
  k_gated_copy<<<grid, 256, 0, s>>>(src, dst, n, scale, gate);
}
void launch_pad_init(const DevProblem& d, hipStream_t s) {
  // (also the back substitution's sentinel: 64 per real block of y)
  const int n_y = (d.n + kNB - 1) / kNB * kNB;
  k_pad_init<<<d.ld, 64, 0, s>>>(d.S, d.ld, d.n, d.fail, reinterpret_cast<unsigned long long*>(d.ysol), n_y, d.gate);
}
void launch_cam_update(const DevProblem& d, bool count_norm, hipStream_t s) {
  k_cam_update<<<blocks_for(d.C, kThreads), kThreads, 0, s>>>(d.C, d.cam, d.ysol, d.scale_c, d.cam_new, d.camRn,
                                                             count_norm ? slot(d, kPStepCam) : nullptr,
                                                             slot(d, kPBadCam), d.gate);
}
void launch_cam_solve(const DevProblem& d, double radius, hipStream_t s) {
  (void)hipMemsetAsync(d.fail, 0, sizeof(int), s);
  if (d.C) k_cam_solve<<<blocks_for(d.C, kThreads), kThreads, 0, s>>>(d.C, d.Ucam, d.diag_c, radius, d.ysol, d.fail, d.gate, d.radius_dev);
}
void launch_point_backsub(const DevProblem& d, hipStream_t s, bool cams_var, bool pts_var) {
  // cameras constant (STRUCT_ONLY): e = J_c y_c = 0 and u = 0
  if (d.N_pad && cams_var)
    k_backsub_a_rc<<<obs_xcd_blocks(d), kThreads, 0, s>>>(d.jgrp, d.jchunks, d.cm_p, d.uv_cm, d.cam_obs, d.camR,
                                                          d.cam, d.Kc, d.scale_c, d.ptS, d.ysol, d.eu, d.eu_cm ? 1 : 0,
                                                          slot(d, kPModel), d.gate);
  else if (d.N_pad) {
    (void)hipMemsetAsync(d.eu, 0, sizeof(double) * 4 * size_t(d.eu_cm ? d.N_pad : d.N), s);
    (void)hipMemsetAsync(slot(d, kPModel), 0, sizeof(double) * size_t(obs_xcd_blocks(d)), s);
  }
  if (d.P && pts_var) {
    k_backsub_b<<<pt_xcd_blocks(d), kThreads, 0, s>>>(d.P, d.pt_off, d.eu, d.eu_cm ? d.pos : nullptr,
                                                               d.ptL, d.ptV, d.scale_p,
                                                               d.X, d.X_new, d.ypt, slot(d, kPStepPt),
                                                               slot(d, kPBadBack), slot(d, kPModelPt), d.gate);
  } else if (d.P) {
    // points constant (POSE_ONLY): y_p = 0, X_new = X, no step, no bad flag
    const size_t nbP = size_t(pt_xcd_blocks(d));
    (void)hipMemsetAsync(d.ypt, 0, sizeof(double) * 3 * size_t(d.P), s);
    (void)hipMemcpyAsync(d.X_new, d.X, sizeof(double) * 3 * size_t(d.P), hipMemcpyDeviceToDevice, s);
    (void)hipMemsetAsync(slot(d, kPStepPt), 0, sizeof(double) * nbP, s);
    (void)hipMemsetAsync(slot(d, kPBadBack), 0, sizeof(double) * nbP, s);
    (void)hipMemsetAsync(slot(d, kPModelPt), 0, sizeof(double) * nbP, s);
  }
  if (d.N_pad)
    k_backsub_c<<<obs_xcd_blocks(d), kThreads, 0, s>>>(d.jgrp, d.jchunks, d.cam_obs, d.cm_p, d.uv_cm, d.Kc, d.X_new,
                                                       d.camRn, slot(d, kPNewCost), d.gate);
}
void launch_reduce(const DevProblem& d, int sl, int nb, int op, int dst, hipStream_t s) {
  k_reduce<<<1, 1024, 0, s>>>(slot(d, sl), nb, op, d.scal + dst);
}
void launch_reduce_batch(const DevProblem& d, const ReduceBatch& b, bool copy_fail, hipStream_t s) {
  if (b.n > 0)
    k_reduce_batch<<<b.n, 1024, 0, s>>>(d.partials, d.max_blocks, b, d.scal, copy_fail ? d.fail : nullptr, d.gate);
}

}  // namespace sfm
