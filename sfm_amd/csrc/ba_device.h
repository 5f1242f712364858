// Device-side data layout of one bundle-adjustment problem (one rank's shard)
// and the launchers of the LM-iteration kernels.  See DESIGN.md §3 for the
// HBM layout and the per-kernel roofline arithmetic.
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>

namespace sfm {

// Per-observation Jacobian record written by the Jacobian pass (doubles):
//   [0..5]  J_X  (2 x 3, row-major)   d r / d X          (scaled)
//   [6..7]  r    (2)                   residual
//   [8..19] J_c  (2 x 6, row-major)   d r / d (rot, t)   (scaled)
constexpr int kJRec = 20;
constexpr int kJX = 0, kRes = 6, kJC = 8;
// Back-substitution pass A output per observation, at its point-major slot:
// u = M^T e (3) | pad.
constexpr int kEU = 4;
// Per-camera rotation data: R (9, row-major) and dR/dw_k (27, k-major).
constexpr int kCamR = 36;
// Per-camera reduction record: U (21, packed upper 6x6), b_c (6), pad.
constexpr int kUcam = 28;
// Per-point record: V (6 packed lower), b_p (3), pad | L (6), z (3), pad.
constexpr int kPtV = 10;
constexpr int kPtL = 10;
// Per-point Schur record (k_schur_pts): X (3), Jacobi scale (3), L (6), 1/l_ii (3), pad: 128 B.
constexpr int kPtS = 16;
// Cholesky tile size.
constexpr int kNB = 64;
// Threads per workgroup of the observation / point kernels.
constexpr int kThreads = 256;
// k_backsolve's "not yet produced" value of a y entry (both halves: a
// signalling NaN, which arithmetic never yields)
constexpr uint32_t kYSentinelWord = 0x7FF4DEADu;
constexpr uint64_t kYSentinel = (uint64_t(kYSentinelWord) << 32) | kYSentinelWord;

// Index of scalar results (device array `scal`, doubles).
enum Scalar {
  kCost = 0,        // cost at current x (Jacobian pass)
  kGradMaxCam,      // max |g| over camera params
  kGradMaxPt,       // max |g| over point params
  kXNorm2Cam,       // sum x^2 over cameras
  kXNorm2Pt,        // sum x^2 over points
  kModelChange,     // model cost change
  kNewCost,         // cost at the candidate
  kStep2Pt,         // sum dx^2 over points
  kStep2Cam,        // sum dx^2 over cameras
  kBadStep,         // > 0 if the step or candidate is non-finite / V not PD
  kCholFail,        // reserved (the Cholesky flag is an int, fetched separately)
  kBadCam,          // > 0 if the camera step is non-finite
  kBadBack,         // > 0 if the point step is non-finite
  kModelChangePt,   // point share of the model cost change (k_backsub_b; kModelChange holds the observations')
  kNumScalars
};

// Batched scalar reductions (k_reduce_batch): job i reduces partial slot
// `slot` over `nb` blocks (op 0 sum, 1 max) into scal[dst].
struct ReduceJob {
  int slot, nb, op, dst;
};
struct ReduceBatch {
  ReduceJob job[8];
  int n = 0;
  void add(int slot, int nb, int op, int dst) { job[n++] = ReduceJob{slot, nb, op, dst}; }
};

struct DevProblem {
  int32_t C = 0, P = 0;      // cameras (global), points (this shard)
  int64_t N = 0;             // observations (this shard)
  // structure (point-major observation order; within a point by camera,
  // then by the caller's order) -- built on the device by set_problem
  int32_t* pt_off = nullptr;   // [P+1]
  int32_t* order = nullptr;    // [N] caller's observation index of point-major q
  int64_t N_pad = 0;           // camera-major positions incl. per-camera padding to 64
  int32_t* cam_obs = nullptr;  // [N_pad] point-major observation id at camera-major position (-1: padding)
  int32_t* cam_rng = nullptr;  // [C][2] camera c's records: positions [begin, end)
  int32_t* cm_p = nullptr;     // [N_pad] point index at camera-major position i
  int4* jchunks = nullptr;     // [n_jchunks] (camera, first position, count, 0): k_jacobian work units
  int32_t n_jchunks = 0;
  int32_t xcd_slice_max = 0;   // chunks of the largest of the 8 point slices (host copy)
  // Schur / Cholesky overlap (compute_step_enqueue): per 64x64 tile of S the
  // camera blocks landed so far and the count that completes it
  int32_t* tile_cnt = nullptr;  // [nblk * nblk], zeroed before each Schur pass
  int32_t* tile_exp = nullptr;  // [nblk * nblk], from set_problem
  int32_t overlap = 0;          // k_chol_fused waits on tile_cnt (and leaves CUs to k_schur_pts)
  int32_t* jgrp = nullptr;     // [9] chunk-table offsets of the 8 point slices (one per XCD)
  int32_t jac_blocks = 1;      // persistent grid of k_jacobian in the solve (cost partials)
  int32_t jac_blocks_rec = 1;  // ... of the record-writing variant (evaluate API, bench roofline)
  double* uv_cm = nullptr;     // [N_pad][2] uv in camera-major order
  int32_t* pos = nullptr;      // [N] camera-major position of point-major observation q
  double* Kc = nullptr;        // [C][5] fx skew cx fy cy
  // parameters (current and candidate)
  double* cam = nullptr;      // [C][6] rot(3) t(3)
  double* cam_new = nullptr;  // [C][6]
  double* X = nullptr;        // [P][3]
  double* X_new = nullptr;    // [P][3]
  double* cam0 = nullptr;     // [C][6] initial (reset)
  double* X0 = nullptr;       // [P][3]
  // Jacobi scaling and LM diagonal
  double* scale_c = nullptr;  // [C][6]
  double* scale_p = nullptr;  // [P][3]
  double* diag_c = nullptr;   // [C][6]
  double* diag_p = nullptr;   // [P][3]
  // per-iteration work arrays
  double* camR = nullptr;     // [C][36]
  double* camRn = nullptr;    // [C][12] candidate R (9) + t (3)
  double* jrec = nullptr;     // [N_pad][20] at camera-major position (J_X 6 | r 2 | J_c 12): evaluate API only,
                              // allocated on first use (the solve writes no records)
  double* eu = nullptr;       // [N][kEU] back substitution pass A output (point-major), or
                              // [N_pad][kEU] at camera-major positions (eu_cm)
  bool eu_cm = false;
  double* ypt = nullptr;      // [P][3] point steps y_p (scaled space)
  int32_t* wcam = nullptr;    // [N_pad / 64] camera of each camera-major wavefront (runs padded to 64)
  double* ptV = nullptr;      // [P][10]
  double* ptL = nullptr;      // [P][10]
  double* Ucam = nullptr;     // [C][28]
  // reduced camera system: column-major lower (== row-major upper), ld x ld,
  // n = 6C unknowns, row n holds the reduced right-hand side (augmented).
  int32_t n = 0, ld = 0, nblk = 0;
  double* S = nullptr;
  double* Spack = nullptr;    // [n(n+1)/2 + n] packed upper triangle + rhs (cross-rank all-reduce)
  double* invL = nullptr;     // [nblk][64][64] inverses of the diagonal tiles
  double* ysol = nullptr;     // [ld] solution of S y = rhs (camera part)
  int32_t* fail = nullptr;    // [1] 1: Cholesky pivot not positive; 2: back-substitution hand-off timeout;
                              //     4: Cholesky tile hand-off timeout
  int32_t* flags = nullptr;   // [nblk] back-substitution hand-off flags (epoch-stamped)
  int32_t* cflags = nullptr;  // [2][nblk][nblk] fused Cholesky: final (F) and partial (P) tile flags
  unsigned long long* cticket = nullptr;  // [5] fused Cholesky tile ticket, its walker-role ticket, the back
                                          // substitution's row ticket (all monotone across launches); a
                                          // distributed factor panel's two (zeroed per panel)
  int32_t n_cu = 0;           // compute units (co-residency bound of the persistent grids)
  // LM diagonal clamp of the running solve (sfm_ba_options min/max_lm_diagonal)
  double min_diag = 1e-6, max_diag = 1e32;

  // Schur (k_schur_pts): every upper-triangle camera block (c1, c2), c1 <=
  // c2, in row-major order, the CSR offsets of its pair list and, per pair
  // (o1, o2) of a common point, that point; F is recomputed per pair from the
  // point and the two wave-uniform cameras
  int64_t n_blk = 0, n_pairs = 0;
  int2* blk = nullptr;        // [n_blk]
  int32_t* seg = nullptr;     // [n_blk + 1]
  int32_t* bpts = nullptr;    // [n_pairs]
  int32_t* bperm = nullptr;   // [n_bslots] k_schur_pts work order (XCD-aware row groups; -1: empty slot;
                              // nullptr: plain block order, small systems)
  int64_t n_bslots = 0;
  double* ptS = nullptr;      // [P][kPtS] X 3, scale 3, l10 l20 l21, 1/l_ii 3, z 3, pad
  int32_t schur_pts_sub = 8;  // lanes per block (8, 16, 32 or 64; C3: 1.07 / 1.09 / 1.21 / 1.49 ms per solve)
  bool schur_wg_blocks = false;  // one block per 4-wave workgroup (small systems with long pair lists)
  // per-wave diagonal-block / rhs partials from k_obs_prep_rc ([N_pad/64][27])
  double* dpart = nullptr;
  // per-chunk U_c / b_c partials from k_jacobian ([N_pad/64][27])
  double* jpart = nullptr;
  // point-major uv and camera index (k_point_eval_rc)
  double* uv_pm = nullptr;     // [N][2]
  int32_t* cam_pm = nullptr;   // [N]
  // reductions
  double* partials = nullptr; // scratch [kNumPartialSlots][max_blocks]
  int32_t max_blocks = 0;
  double* scal = nullptr;     // [kNumScalars]
  double* scal_host = nullptr;  // pinned host mirror
  // device-driven LM loop (sfm_ba_solve_resident on an unsharded problem):
  // the gate of the phase being enqueued (kernels return at once when
  // *gate == 0) and the trust-region radius the kernels read; both nullptr
  // on the host-driven path
  const int32_t* gate = nullptr;
  const double* radius_dev = nullptr;
};

// Partial-sum slots (each max_blocks doubles).
enum PartialSlot {
  kPCost = 0, kPXNormCam, kPXNormPt, kPGradCam, kPGradPt, kPModel, kPNewCost, kPStepPt, kPStepCam, kPBad,
  kPBadCam, kPBadBack, kPModelPt,
  kNumPartialSlots
};

// ---- launchers (ba_kernels.hip) ----
void launch_cam_prep(const DevProblem& d, double* cam, bool count_norm, hipStream_t s);
// the device LM loop's accept folded in: cam_new -> cam, X_new -> X (grid >= the copy's workgroups)
void launch_cam_prep_accept(const DevProblem& d, bool count_norm, int grid, hipStream_t s);
// write_records: also store the 160-B records (evaluate API, bench roofline)
void launch_jacobian(const DevProblem& d, bool scaled, hipStream_t s, bool write_records = false);
void launch_cam_reduce(const DevProblem& d, hipStream_t s);
// mode 0: unscaled pass -> compute scale_c from colnorms; mode 1: diag (if !reuse) + gradient
void launch_cam_finalize(const DevProblem& d, int mode, bool reuse_diag, bool count_grad, hipStream_t s);
// launch_cam_reduce + launch_cam_finalize (reuse_diag false) in one launch
// (unsharded: no U_c all-reduce between them); gradient partials per camera
void launch_cam_sum_finalize(const DevProblem& d, int mode, bool count_grad, hipStream_t s);
// mode 0: unscaled pass -> scale_p; mode 1: V, b, diag (if !reuse), gradient, x-norm
void launch_point_eval(const DevProblem& d, int mode, bool reuse_diag, hipStream_t s);
void launch_point_prep(const DevProblem& d, double radius, hipStream_t s);
void launch_point_factor(const DevProblem& d, double radius, hipStream_t s);
void launch_schur(const DevProblem& d, double radius, bool add_diag, hipStream_t s);
// its two parts: the diagonal blocks + rhs (k_schur_diag_sum) and the
// off-diagonal blocks (k_schur_pts; tile_cnt != nullptr: overlapped with the
// factorisation, blocks counted per 64x64 tile as they land)
void launch_schur_diag(const DevProblem& d, double radius, bool add_diag, hipStream_t s);
void launch_schur_offdiag(const DevProblem& d, int* tile_cnt, hipStream_t s);
void launch_pad_init(const DevProblem& d, hipStream_t s);
void launch_pack_upper(const DevProblem& d, bool unpack, hipStream_t s);
// dst = scale * src unless *gate == 0 (gate may be nullptr)
void launch_gated_copy(const double* src, double* dst, int64_t n, double scale, const int32_t* gate, hipStream_t s);
void launch_cam_update(const DevProblem& d, bool count_norm, hipStream_t s);
// small systems (C <= 64): the point pass and the camera sums + finalisation
// (k_cam_sum_finalize's work) in one launch; false when not applicable
bool launch_point_eval_with_cams(const DevProblem& d, int mode, bool count_grad, hipStream_t s);
void launch_point_backsub(const DevProblem& d, hipStream_t s, bool cams_var = true, bool pts_var = true);
// grid of the XCD-ordered observation passes (k_obs_prep_rc, k_backsub_a_rc):
// one workgroup per 4 chunks, a multiple of 8 (one point slice per XCD)
inline int obs_xcd_blocks(const DevProblem& d) {
  // one wave per chunk of the LARGEST slice (slices differ by ~5% at C3; a
  // grid sized by the mean left the largest slice's excess chunks to a
  // second round of waves: 45.6 -> 50.0 us for k_obs_prep_rc)
  const int64_t per = d.xcd_slice_max > 0 ? (int64_t(d.xcd_slice_max) + 3) / 4
                                          : ((d.N_pad / 64 + 3) / 4 + 7) / 8;
  return int(8 * std::max<int64_t>(1, per));
}
// grid of the XCD-ordered point pass of the back substitution (k_backsub_b):
// workgroup b serves point slice b % 8 -- the points whose observations the
// XCD-ordered passes ran on XCD b % 8 -- in blocks of kThreads points
inline int pt_xcd_blocks(const DevProblem& d) {
  const int64_t per_slice = (int64_t(d.P) + 7) / 8;
  return int(8 * std::max<int64_t>(1, (per_slice + kThreads - 1) / kThreads));
}
void launch_cam_solve(const DevProblem& d, double radius, hipStream_t s);
// sum (op 0) or max (op 1) of `nb` partials in slot into scal[dst]
void launch_reduce(const DevProblem& d, int slot, int nb, int op, int dst, hipStream_t s);
void launch_reduce_batch(const DevProblem& d, const ReduceBatch& b, bool copy_fail, hipStream_t s);
int blocks_for(int64_t n, int threads);

// ---- dense Cholesky (chol_kernels.hip) ----
// cam_step >= 0: a small system's one-workgroup factor also takes the
// camera step (k_cam_update; cam_step > 0: with its step-length partial);
// returns whether it did.  overlap: d.overlap when the factor runs beside
// k_schur_pts (its helpers then await tile_cnt and take the overlap's grid),
// 0 otherwise -- only the overlapped branch zeroes and fills tile_cnt
bool launch_cholesky(const DevProblem& d, int epoch, hipStream_t s, bool clear_fail = true, int cam_step = -1,
                     int overlap = 0);
// W_k granules back to the sentinel (k_schur_diag_sum does this in the solve)
// sentinel_set: y already holds kYSentinel (k_pad_init wrote it)
void launch_backsolve(const DevProblem& d, int epoch, hipStream_t s, bool sentinel_set = false);

// ---- distributed factor: 1-D block-cyclic column panels of pt tiles
// (panel J on rank J % nranks; chol_kernels.hip) ----
// panel k of the trailing matrix factored in place (L, W_k) by its owner
int launch_cholesky_panel(const DevProblem& d, int k, int pt, int epoch, hipStream_t s);
// this rank's panels j in [j0, j1] (j > k) updated with panel k's L
void launch_panel_update(const DevProblem& d, int k, int j0, int j1, int pt, int nranks, int rank, hipStream_t s);
int panel_update_tiles(int nblk, int pt, int j0, int j1, int nranks, int rank);
// panel rectangles (columns col0..col1-1, rows c0_J..n) and buf at off[J]
// (device array, < 0: skipped; nullptr: every panel at off1); mode 0 packs
// S into buf, 1 unpacks buf into S, 2 adds buf into S
constexpr int kPanelPack = 0, kPanelUnpack = 1, kPanelAdd = 2;
void launch_panel_copy(const DevProblem& d, int mode, int pt, int col0, int col1, const int64_t* off, int64_t off1,
                       double* buf, hipStream_t s);
// the failure flag into (put) or OR-ed from a broadcast buffer's slot
void launch_fail_slot(const DevProblem& d, bool put, double* slot, hipStream_t s);
// a diagonally dominant augmented system (timing of the distributed factor)
void launch_spd_fill(double* A, int ld, int n, unsigned seed, hipStream_t s);

}  // namespace sfm
