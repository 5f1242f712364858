// Host side of the device bundle adjuster: problem layout, the Levenberg-
// Marquardt trust-region loop and the C ABI of include/sfm_amd.h.
//
// The loop restates Ceres' TrustRegionMinimizer + LevenbergMarquardtStrategy
// (the solver behind ceres::Solve at /root/reference/CTracker.cpp:700-701,
// options CTracker.cpp:571-577) step for step; the
// per-iteration arithmetic runs in the kernels of ba_kernels.hip /
// chol_kernels.hip and only ~10 scalars cross PCIe per iteration.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <map>
#include <atomic>
#include <thread>

#include <algorithm>
#include <array>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <vector>
#include <chrono>

#include "sfm_trace.h"
#include "ba_device.h"
#include "ba_setup.h"
#include "ba_common.h"
#include "ba_host_layout.h"
#include "../../include/sfm_amd.h"

namespace {
thread_local std::string g_err;
int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
}  // namespace

void sfm_internal_set_error(const std::string& msg) { g_err = msg; }

#define HIPCHK(expr)                                                                              \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess) return fail(SFM_EIO, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define NCCLCHK(expr)                                                                             \
  do {                                                                                            \
    ncclResult_t r_ = (expr);                                                                     \
    if (r_ != ncclSuccess) return fail(SFM_EIO, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
  } while (0)

using namespace sfm;

enum Phase { kPhJac = 0, kPhCamRed, kPhPtEval, kPhPtPrep, kPhSchur, kPhChol, kPhBack, kPhBacksub, kPhOther, kNumPh };

// device LM loop state (k_lm_decide / k_lm_post; see "device-driven LM loop")
struct LmCtl {
  int32_t run_step, run_eval, done, termination, error;
  int32_t iteration, num_consecutive_invalid;
  int32_t n_succ, n_unsucc, n_invalid, n_resid, n_jac, n_lin, trace_len;
  double radius, decrease_factor, cost, grad_max, x_norm;
  sfm_ba_iteration pending;  // an accepted iteration, completed after its evaluation
  int32_t max_iter, max_invalid;
  double ftol, gtol, ptol, max_radius, min_radius, min_rel_dec;
  uint32_t red_count;  // workgroups of k_reduce_batch_lm done (reset by the last)
  double init_cost, init_grad;  // the initial evaluation (k_lm_init), for the host's summary
};

struct sfm_ba_handle {
  int device = 0;
  hipStream_t stream = nullptr;
  DevProblem d;
  int32_t mode = SFM_BA_STRUCT_AND_POSE;  // of the running solve (CTracker.h:67)
  int32_t bs_epoch = 0;          // stamp of the last back-substitution launch (k_backsolve flags)
  int32_t chol_epoch = 0;        // launches of the fused Cholesky since the last set_problem
  bool force_pack = false;       // SFM_FORCE_PACK=1: exercise the packed all-reduce path on one rank (tests)
  std::vector<std::pair<size_t, void*>> allocs;  // (bytes, buffer) of the resident problem
  std::vector<std::pair<size_t, void*>> tmps;    // set_problem's scratch (back to the pool when it returns)
  std::multimap<size_t, void*> pool;             // buffers of earlier problems, reused by size
  bool has_problem = false;
  // multi-GPU
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  // host-callback collective (sfm_ba_set_host_comm: tests run the sharded
  // path with several ranks on one GPU, where RCCL allows one rank per GPU)
  sfm_allreduce_fn host_fn = nullptr;
  void* host_user = nullptr;
  std::vector<double> host_buf, host_buf2;
  // ... with broadcast and reduce-scatter too (sfm_ba_set_host_collectives);
  // without it the distributed factor builds both from host_fn's all-reduce
  sfm_collective_fn coll_fn = nullptr;
  void* coll_user = nullptr;
  // distributed reduced-camera factor (sfm_ba_set_distributed_factor): 1-D
  // block-cyclic column panels of dist_pt 64-column tiles; 0 = every rank
  // factors the all-reduced system (replicated)
  int dist_pt = 0;
  struct DistBufs {
    int pt = 0, nblk = 0, n = 0, nranks = 0, rank = 0;  // the layout below was made for
    int64_t total = 0;                // doubles of all panel rectangles
    int64_t bcast_cap = 0;            // largest broadcast (doubles)
    std::vector<int64_t> count, poff; // per panel: rectangle doubles, offset in the panel image
    double* send = nullptr;           // [total] this rank's partial panels (own ones: zeros)
    double* recv = nullptr;           // [total] the other ranks' sums of the own panels
    double* bcast = nullptr;          // [2][bcast_cap]: panel k travels in half k % 2
    hipStream_t cstream = nullptr;    // RCCL: the collectives' own stream (look-ahead)
    hipEvent_t ev_packed = nullptr, ev_free[2] = {nullptr, nullptr}, ev_arrived[2] = {nullptr, nullptr};
    hipEvent_t ev_sent = nullptr;     // the partial panels are packed
    std::vector<hipEvent_t> ev_red;   // [np] panel k's reduce has landed (owner)
    int64_t* off_send = nullptr;      // [np] panel offset in send, -1 for own panels (device)
    int64_t* off_recv = nullptr;      // (unused)
  } dist;
  // out-of-place target of the collectives enqueued inside a gated phase of
  // the device LM loop (allreduce below); grown on demand
  double* ar_tmp = nullptr;
  size_t ar_tmp_cap = 0;
  // SFM_EMULATE_IDENTICAL_RANKS=k (tests, read by sfm_ba_set_comm): every sum
  // collective returns k times its one-rank result, i.e. the sum over k
  // ranks holding the same shard, so a one-GPU run sees the stale-buffer
  // hazards of a multi-rank one
  int emulate_ranks = 1;
  // device-driven LM loop (unsharded solves): control block, its pinned
  // mirror and the device trace buffer (grown to the iteration cap)
  LmCtl* lm_ctl = nullptr;
  LmCtl* lm_ctl_host = nullptr;
  // (pinned host memory: the deciding workgroups write the few entries
  // straight to the host, which reads them after the batch's synchronisation)
  sfm_ba_iteration* lm_trace = nullptr;
  int lm_trace_cap = 0;
  // one-shot sfm_ba_solve on a small problem: every batch's control readback
  // also brings the parameters (cam | X) into param_host, so the final
  // download needs no further round trip (param_host_valid until consumed)
  bool prefetch_params = false;
  bool param_host_valid = false;
  double* param_host = nullptr;
  size_t param_host_cap = 0;
  // pinned staging for every host <-> device transfer of set_problem,
  // get_parameters and the LM trace: a pageable copy goes through the
  // runtime's own staging (C1: the 320-KB uv upload took 131 us, the 49-KB
  // parameter download ~100 us), a pinned one is a single DMA.  Grown
  // geometrically, only while the stream is idle.
  uint8_t* stage = nullptr;
  size_t stage_cap = 0;
  // device LM loop without a collective: the phase reductions run the
  // bookkeeping in their last workgroup (k_reduce_batch_lm)
  bool fuse_lm = false;
  // device LM loop: the evaluation's k_cam_prep also makes the accepted
  // candidate current (k_lm_accept folded in; its grid covers the copy)
  int accept_grid = 0;  // < 0: done by the deciding reduction (AcceptFold)
  bool accept_fold = false;
  int n_cu = 0;  // compute units of the device (queried once)
  // Schur / Cholesky overlap (DevProblem::overlap): the factorisation's
  // stream and the two events that fork and join it
  hipStream_t stream2 = nullptr;
  hipEvent_t ov_ev[2] = {nullptr, nullptr};
  // set_problem's uploads beside the layout kernels (large problems): the
  // parameters (uev), and uv from a worker thread (uev_uv)
  hipStream_t ustream = nullptr;
  hipEvent_t uev = nullptr, uev_uv = nullptr;
  // profiling
  bool profiling = false;
  std::vector<hipEvent_t> ev;
  int ev_used = 0;
  std::vector<std::pair<int, int>> ev_marks;  // (phase, event index of start); end = start + 1
  double phase_ms[kNumPh] = {0};
  int phase_count[kNumPh] = {0};
};

namespace {

// Device buffers are taken from the handle's pool (the previous problem's
// buffers, best fit within 2x) before hipMalloc: repeated keyframe-sized
// solves (CSfM::bundleAdjustment after every keyframe) then allocate
// nothing.  Contents are never assumed: set_problem initialises every
// buffer it relies on.
template <typename T>
int dalloc(sfm_ba_handle* h, T** p, size_t count) {
  if (count == 0) count = 1;
  const size_t bytes = (count * sizeof(T) + 255) & ~size_t(255);
  auto it = h->pool.lower_bound(bytes);
  void* q = nullptr;
  size_t got = bytes;
  if (it != h->pool.end() && it->first <= 2 * bytes) {
    q = it->second;
    got = it->first;
    h->pool.erase(it);
  } else {
    hipError_t e = hipMalloc(&q, bytes);
    if (e != hipSuccess) return fail(SFM_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  }
  h->allocs.push_back({got, q});
  *p = static_cast<T*>(q);
  return 0;
}
// set_problem scratch: retired into the pool when set_problem returns after
// its synchronisation, or -- a keyframe-sized set_problem returns without one
// -- by the next set_problem's free_problem, which synchronises first.  So a
// pooled buffer is never handed out while a kernel of this stream may still
// use it: every path that moves tmps into the pool (retire_tmps) runs behind
// a hipStreamSynchronize of the handle's stream.
template <typename T>
int dalloc_tmp(sfm_ba_handle* h, T** p, size_t count) {
  const int rc = dalloc(h, p, count);
  if (rc) return rc;
  h->tmps.push_back(h->allocs.back());
  h->allocs.pop_back();
  return 0;
}
void retire_tmps(sfm_ba_handle* h) {
  for (auto& a : h->tmps) h->pool.insert(a);
  h->tmps.clear();
}

// The pinned staging buffer with room for `bytes`.  Growing it frees the old
// buffer, so nothing may still read or write it: every caller has synchronised
// the stream (set_problem, get_parameters), and a keyframe-sized set_problem,
// which returns with its uploads from the stage still in flight, is always
// followed by a synchronising call before the stage is written again.  The
// rule is checked here: a stream found busy is drained first (and counted, so
// a test can see the rule broken).
std::atomic<int> g_stage_busy_regrows{0};
int stage_reserve(sfm_ba_handle* h, size_t bytes) {
  if (bytes <= h->stage_cap) return 0;
  if (h->stage && hipStreamQuery(h->stream) == hipErrorNotReady) {
    g_stage_busy_regrows.fetch_add(1);
    if (hipStreamSynchronize(h->stream) != hipSuccess) return fail(SFM_EIO, "stream error before the stage regrows");
  }
  const size_t cap = std::max<size_t>({bytes, size_t(1) << 20, 2 * h->stage_cap});
  if (h->stage) (void)hipHostFree(h->stage);
  h->stage = nullptr;
  h->stage_cap = 0;
  if (hipHostMalloc(reinterpret_cast<void**>(&h->stage), cap) != hipSuccess) {
    h->stage = nullptr;
    return fail(SFM_ENOMEM, "hipHostMalloc failed (staging buffer)");
  }
  h->stage_cap = cap;
  return 0;
}
// Transfers above this go straight from / to the caller's pageable memory:
// the runtime pipelines its own staging copies with the DMA, where ours
// would run them one after the other (C3 one-shot 7.4 -> 9.2 ms with the
// 48-MB observation upload staged).
constexpr size_t kStageMaxBytes = size_t(1) << 20;
constexpr size_t kParamPrefetchMaxBytes = size_t(1) << 20;  // one-shot solves that prefetch their parameters

// byte offsets of a packed staging layout (256-B aligned pieces)
struct StageLayout {
  size_t bytes = 0;
  size_t add(size_t n) {
    const size_t o = bytes;
    bytes += (n + 255) & ~size_t(255);
    return o;
  }
};

void release_pool(sfm_ba_handle* h) {
  for (auto& kv : h->pool) hipFree(kv.second);
  h->pool.clear();
}

// Retires the problem's buffers into the pool (freed by release_pool).
void free_problem(sfm_ba_handle* h) {
  for (auto& a : h->allocs) h->pool.insert(a);
  h->allocs.clear();
  retire_tmps(h);
  double* keep = h->d.scal_host;  // pinned mirror: kept for the handle's life
  h->d = DevProblem();
  h->d.scal_host = keep;
  h->has_problem = false;
}

// ---- phase timing (HIP events on the solver stream; read at the per-iteration sync)
int mark_begin(sfm_ba_handle* h, int ph, hipStream_t on = nullptr) {
  if (!h->profiling) return -1;
  if (h->ev_used + 2 > int(h->ev.size())) {
    const size_t old = h->ev.size();
    h->ev.resize(old + 256);
    for (size_t i = old; i < h->ev.size(); ++i) hipEventCreate(&h->ev[i]);
  }
  h->ev_marks.push_back({ph, h->ev_used});
  hipEventRecord(h->ev[h->ev_used], on ? on : h->stream);
  h->ev_used += 2;
  return int(h->ev_marks.size()) - 1;
}
// ends mark `m` (default: the last one begun)
void mark_end(sfm_ba_handle* h, hipStream_t on = nullptr, int m = -1) {
  if (!h->profiling) return;
  const auto& mk = m < 0 ? h->ev_marks.back() : h->ev_marks[size_t(m)];
  hipEventRecord(h->ev[mk.second + 1], on ? on : h->stream);
}
void collect_marks(sfm_ba_handle* h) {
  if (!h->profiling) return;
  for (auto& m : h->ev_marks) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, h->ev[m.second], h->ev[m.second + 1]) == hipSuccess) {
      h->phase_ms[m.first] += ms;
      h->phase_count[m.first] += 1;
    }
  }
  h->ev_marks.clear();
  h->ev_used = 0;
}

bool env_flag(const char* name) {
  const char* v = std::getenv(name);
  return v && v[0] == '1';
}

// Compute units of the device: the persistent grids (fused Cholesky) size
// themselves to one workgroup per CU (they also finish when only part of the
// grid is resident: roles go by start order).
int device_cus(int device) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess || prop.multiProcessorCount < 2) return 2;
  return prop.multiProcessorCount;
}

// SFM_TIMING=1: host phase times of sfm_ba_set_problem and of the device LM
// loop's batches on stderr.
struct HostTimer {
  bool on = env_flag("SFM_TIMING");
  const char* tag = "set_problem";
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  void mark(const char* what) {
    if (!on) return;
    const auto t1 = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[%s] %-22s %8.3f ms\n", tag, what,
                 std::chrono::duration<double, std::milli>(t1 - t0).count());
    t0 = t1;
  }
};

// ---- device-driven LM loop ----
// The trust-region bookkeeping of the host loop in sfm_ba_solve_resident,
// restated on the device so that an unsharded solve enqueues several
// iterations per host synchronisation.  k_lm_decide follows compute_step's
// reductions; the accept copy (cam_new -> cam, X_new -> X: enqueued
// iterations hold fixed pointers, where the host loop swaps them) and the
// evaluation kernels run only when the step
// was accepted (gate run_eval), k_lm_post completes the accepted iteration
// after its evaluation; compute_step's kernels run only while the loop is
// not done (gate run_step).  The arithmetic is the host loop's, operation
// for operation (contraction off), so both loops take the same decisions.


__device__ void lm_push(LmCtl* c, sfm_ba_iteration* trace, int cap, const sfm_ba_iteration& it) {
  if (c->trace_len < cap) trace[c->trace_len] = it;
  ++c->trace_len;
}
__device__ void lm_finish(LmCtl* c, int term) {
  c->termination = term;
  c->done = 1;
  c->run_step = 0;
  c->run_eval = 0;
}

// after compute_step's reduction (scal: model change, candidate cost, step
// norms, bad-step flags; the Cholesky failure int after the scalars)
__device__ void lm_decide(LmCtl* c, const double* scal, sfm_ba_iteration* trace, int cap) {
#pragma clang fp contract(off)
  if (c->done) {
    c->run_eval = 0;
    return;
  }
  ++c->iteration;
  sfm_ba_iteration itr;
  itr.iteration = c->iteration;
  itr.step_is_valid = 0;
  itr.step_is_successful = 0;
  itr.reserved = 0;
  itr.cost = 0.0;
  itr.cost_change = 0.0;
  itr.gradient_max_norm = 0.0;
  itr.step_norm = 0.0;
  itr.relative_decrease = 0.0;
  itr.trust_region_radius = 0.0;
  c->n_lin++;
  const int chol_fail = *reinterpret_cast<const int*>(scal + kNumScalars);
  if (chol_fail & 6) {  // a persistent grid's hand-off timed out: the host reports it
    c->error = chol_fail & 6;
    lm_finish(c, SFM_FAILURE);
    return;
  }
  const bool solve_ok = chol_fail == 0 && !(scal[kBadStep] > 0.0) && !(scal[kBadCam] > 0.0) && !(scal[kBadBack] > 0.0);
  const double model_cost_change = scal[kModelChange] + scal[kModelChangePt];
  itr.step_is_valid = (solve_ok && model_cost_change >= 0.0) ? 1 : 0;
  if (!itr.step_is_valid) {
    ++c->num_consecutive_invalid;
    c->n_invalid++;
    if (c->num_consecutive_invalid >= c->max_invalid) {
      itr.cost = c->cost; itr.gradient_max_norm = c->grad_max; itr.trust_region_radius = c->radius;
      lm_push(c, trace, cap, itr);
      lm_finish(c, SFM_FAILURE);
      return;
    }
    itr.cost = c->cost;
    itr.gradient_max_norm = c->grad_max;
  } else {
    c->num_consecutive_invalid = 0;
    double new_cost = scal[kNewCost];
    if (!isfinite(new_cost)) new_cost = DBL_MAX;
    c->n_resid++;
    itr.step_norm = sqrt(scal[kStep2Cam] + scal[kStep2Pt]);
    const double step_size_tolerance = c->ptol * (c->x_norm + c->ptol);
    if (itr.step_norm <= step_size_tolerance) {
      itr.cost = c->cost; itr.gradient_max_norm = c->grad_max; itr.trust_region_radius = c->radius;
      lm_push(c, trace, cap, itr);
      lm_finish(c, SFM_CONVERGENCE);
      return;
    }
    itr.cost_change = c->cost - new_cost;
    if (fabs(itr.cost_change) <= c->ftol * c->cost) {
      itr.cost = c->cost; itr.gradient_max_norm = c->grad_max; itr.trust_region_radius = c->radius;
      lm_push(c, trace, cap, itr);
      lm_finish(c, SFM_CONVERGENCE);
      return;
    }
    itr.relative_decrease = itr.cost_change / model_cost_change;
    itr.step_is_successful = itr.relative_decrease > c->min_rel_dec;
  }
  if (itr.step_is_successful) {
    c->n_succ++;
    const double q = 2.0 * itr.relative_decrease - 1.0;
    double radius = c->radius / fmax(1.0 / 3.0, 1.0 - q * q * q);
    c->radius = fmin(c->max_radius, radius);
    c->decrease_factor = 2.0;
    c->pending = itr;  // cost, gradient and radius after the evaluation (k_lm_post)
    c->run_eval = 1;
    return;
  }
  c->n_unsucc++;
  c->radius = c->radius / c->decrease_factor;
  c->decrease_factor *= 2.0;
  c->run_eval = 0;
  itr.gradient_max_norm = c->grad_max;
  itr.cost = c->cost;
  itr.trust_region_radius = c->radius;
  lm_push(c, trace, cap, itr);
  if (c->radius < c->min_radius) { lm_finish(c, SFM_CONVERGENCE); return; }
  if (c->iteration >= c->max_iter) { lm_finish(c, SFM_NO_CONVERGENCE); return; }
}
__global__ void k_lm_decide(LmCtl* c, const double* __restrict__ scal, sfm_ba_iteration* trace, int cap) {
  lm_decide(c, scal, trace, cap);
}

// after the accepted step's evaluation (scal: cost, gradient max norms, |x|^2)
__device__ void lm_post(LmCtl* c, const double* scal, sfm_ba_iteration* trace, int cap) {
#pragma clang fp contract(off)
  if (!c->run_eval) return;
  c->run_eval = 0;
  c->n_jac++;
  c->n_resid++;
  const double cost = scal[kCost];
  c->cost = cost;
  if (!isfinite(cost)) { lm_finish(c, SFM_FAILURE); return; }
  c->grad_max = fmax(scal[kGradMaxCam], scal[kGradMaxPt]);
  c->x_norm = sqrt(scal[kXNorm2Cam] + scal[kXNorm2Pt]);
  sfm_ba_iteration itr = c->pending;
  itr.gradient_max_norm = c->grad_max;
  itr.cost = cost;
  itr.trust_region_radius = c->radius;
  lm_push(c, trace, cap, itr);
  if (c->grad_max <= c->gtol) { lm_finish(c, SFM_CONVERGENCE); return; }
  if (c->iteration >= c->max_iter) { lm_finish(c, SFM_NO_CONVERGENCE); return; }
}
__global__ void k_lm_post(LmCtl* c, const double* __restrict__ scal, sfm_ba_iteration* trace, int cap) {
  lm_post(c, scal, trace, cap);
}

// after the initial evaluation (scal: cost, gradient max norms, |x|^2): the
// loop state the host loop derives from its first evaluate(), so that the
// solve needs no host round trip before the first iteration.  Error bit 8:
// the initial cost is not finite (the host reports it).
__device__ void lm_init(LmCtl* c, const double* scal) {
#pragma clang fp contract(off)
  const double cost = scal[kCost];
  c->cost = cost;
  c->init_cost = cost;
  c->grad_max = fmax(scal[kGradMaxCam], scal[kGradMaxPt]);
  c->init_grad = c->grad_max;
  c->x_norm = sqrt(scal[kXNorm2Cam] + scal[kXNorm2Pt]);
  if (!isfinite(cost)) {
    c->error |= 8;
    lm_finish(c, SFM_FAILURE);
  } else if (c->grad_max <= c->gtol) {
    lm_finish(c, SFM_CONVERGENCE);
  } else if (c->max_iter <= 0) {
    lm_finish(c, SFM_NO_CONVERGENCE);
  }
}
__global__ void k_lm_init(LmCtl* c, const double* __restrict__ scal) { lm_init(c, scal); }

// A phase's batched reduction fused with the bookkeeping that follows it
// (unsharded device loop: no collective sits between them): every
// workgroup reduces its job (reduce_batch_job, as k_reduce_batch), and the
// last one to finish runs k_lm_decide's (kPost: k_lm_post's) body on the
// reduced scalars -- one launch instead of two, ~4.5 us of dispatch each.
// The hand-off is MI355X_MICROARCH.md "Valid forms" row 1 without fences:
// each workgroup's one storing lane stores its scalars sc1, waits for them
// (vmcnt(0)) and adds to the count; the workgroup whose add returns the last
// value re-reads every scalar through sc1 loads after a barrier.  (Two
// __threadfence()s stood there before -- write-back + invalidate of the XCD
// L2, ~3.5 us each, the second by all 1024 threads.)  The count lives in the
// control block, which the loop's upload zeroes, and the last workgroup
// resets it.  Gated like the reduction: with the phase skipped the
// bookkeeping is a no-op too (run_step = 0 only once done, run_eval = 0).
enum LmTail { kTailDecide = 0, kTailPost = 1, kTailInit = 2 };
// Small problems (C <= 256, few points): the accepted step's copy and camera
// preparation -- k_cam_prep with cam_src, the evaluation's first launch --
// run in the deciding workgroup right after lm_decide, when it accepted the
// step.  Same per-camera arithmetic; the |x|^2 partial is the one-workgroup
// sum (the 12 extra waves add +0.0).  C == 0: not folded.
struct AcceptFold {
  int C;
  int64_t n_x;
  double* cam;
  double* camR;
  double* part_xn;
  const double* cam_src;
  const double* X_src;
  double* X_dst;
};
constexpr int kAcceptFoldMaxCams = 256;
constexpr int64_t kAcceptFoldMaxX = 3 * 8192;
template <int kTail>
__global__ __launch_bounds__(1024) void k_reduce_batch_lm(const double* __restrict__ partials, int64_t max_blocks,
                                                          ReduceBatch b, double* __restrict__ scal,
                                                          const int* __restrict__ fail, const int* __restrict__ gate,
                                                          LmCtl* c, sfm_ba_iteration* trace, int cap,
                                                          const AcceptFold af) {
  if (gate && *gate == 0) return;
  __shared__ double sh[16];
  __shared__ double sc[kNumScalars + 1];
  __shared__ int last;
  reduce_batch_job(partials, max_blocks, b.job[blockIdx.x], scal, blockIdx.x == 0 ? fail : nullptr, sh, true);
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the storing lane's sc1 stores landed)
    last = atomicAdd(&c->red_count, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  // The bookkeeping runs on an LDS copy of the control block, loaded and
  // stored back by the whole workgroup: its branches read and write the
  // block field by field, one dependent memory round trip each in place.
  __shared__ LmCtl lc;
  static_assert(sizeof(LmCtl) % 4 == 0, "LmCtl is copied as 32-bit words");
  constexpr int kCtlWords = int(sizeof(LmCtl) / 4);
  static_assert(kCtlWords <= 1024, "one word per thread");
  if (threadIdx.x <= kNumScalars)
    sc[threadIdx.x] = __hip_atomic_load(scal + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < kCtlWords) reinterpret_cast<int*>(&lc)[threadIdx.x] = reinterpret_cast<const int*>(c)[threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) {
    lc.red_count = 0;
    if (kTail == kTailPost) lm_post(&lc, sc, trace, cap);
    else if (kTail == kTailInit) lm_init(&lc, sc);
    else lm_decide(&lc, sc, trace, cap);
  }
  __syncthreads();
  if (threadIdx.x < kCtlWords) reinterpret_cast<int*>(c)[threadIdx.x] = reinterpret_cast<const int*>(&lc)[threadIdx.x];
  if (kTail != kTailDecide || af.C == 0 || !lc.run_eval) return;
  for (int64_t i = threadIdx.x; i < af.n_x; i += blockDim.x) af.X_dst[i] = af.X_src[i];
  double xn = 0.0;
  const int cc = threadIdx.x;
  if (cc < af.C) {
    double x6[6];
    for (int k = 0; k < 6; ++k) x6[k] = af.cam_src[6 * cc + k];
    for (int k = 0; k < 6; ++k) af.cam[6 * cc + k] = x6[k];
    const double w[3] = {x6[0], x6[1], x6[2]};
    double R[9], dR[27];
    rotation(w, R, dR);
    double* o = af.camR + size_t(kCamR) * cc;
    for (int i = 0; i < 9; ++i) o[i] = R[i];
    for (int i = 0; i < 27; ++i) o[9 + i] = dR[i];
    for (int k = 0; k < 6; ++k) xn += x6[k] * x6[k];
  }
  const double r = block_reduce(xn, sh, false);
  if (threadIdx.x == 0 && af.part_xn) af.part_xn[0] = r;
}

// Reduced systems with more camera blocks than this take the XCD-aware
// k_schur_pts order (C3: 125k blocks); smaller ones the plain order.
constexpr int64_t kSchurXcdMinBlocks = 8192;


bool sharded(const sfm_ba_handle* h) { return h->comm != nullptr || h->host_fn != nullptr; }

size_t packed_size(int n) { return size_t(n) * (n + 1) / 2 + size_t(n); }

int allreduce(sfm_ba_handle* h, double* buf, size_t count, ncclRedOp_t op) {
  if (h->host_fn) {
    h->host_buf.resize(count);
    HIPCHK(hipMemcpyAsync(h->host_buf.data(), buf, count * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    if (h->host_fn(h->host_buf.data(), int64_t(count), op == ncclMax ? 1 : 0, h->host_user) != 0)
      return fail(SFM_EIO, "host all-reduce callback failed");
    HIPCHK(hipMemcpyAsync(buf, h->host_buf.data(), count * sizeof(double), hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return 0;
  }
  if (!h->comm) return 0;
  const double scale = op == ncclSum ? double(h->emulate_ranks) : 1.0;
  // Inside a gated phase of the device LM loop the phase's kernels may return
  // at once, leaving `buf` holding the previous, already reduced values: an
  // in-place collective would sum those again (U_c times the rank count after
  // every rejected step).  So the collective goes out of place and a gated
  // kernel copies the result back.  The packed S image is scratch (its pack
  // and unpack are gated themselves) and stays in place.
  const bool gated = h->d.gate != nullptr && buf != h->d.Spack;
  if (!gated) {
    NCCLCHK(ncclAllReduce(buf, buf, count, ncclDouble, op, h->comm, h->stream));
    if (scale != 1.0) launch_gated_copy(buf, buf, int64_t(count), scale, nullptr, h->stream);
    return 0;
  }
  if (h->ar_tmp_cap < count) {
    HIPCHK(hipStreamSynchronize(h->stream));
    if (h->ar_tmp) (void)hipFree(h->ar_tmp);
    h->ar_tmp = nullptr;
    h->ar_tmp_cap = 0;
    const size_t cap = std::max<size_t>(count, 4096);
    if (hipMalloc(reinterpret_cast<void**>(&h->ar_tmp), cap * sizeof(double)) != hipSuccess) {
      h->ar_tmp = nullptr;
      return fail(SFM_ENOMEM, "hipMalloc failed (collective scratch)");
    }
    h->ar_tmp_cap = cap;
  }
  NCCLCHK(ncclAllReduce(buf, h->ar_tmp, count, ncclDouble, op, h->comm, h->stream));
  launch_gated_copy(h->ar_tmp, buf, int64_t(count), scale, h->d.gate, h->stream);
  return 0;
}

// Host-callback collective of kind SFM_COLL_* on device buffers (D2H, the
// callback, H2D; synchronous).  For a plain all-reduce hook the other two
// are built from it: a broadcast is the sum of the root's buffer and the
// others' zeros (exact), a reduce-scatter the all-reduced segments' own.
int host_collective(sfm_ba_handle* h, int kind, double* buf, double* out, int64_t count, int arg) {
  const int64_t in_n = kind == SFM_COLL_REDUCE_SCATTER ? count * h->nranks : count;
  h->host_buf.resize(size_t(in_n));
  HIPCHK(hipMemcpyAsync(h->host_buf.data(), buf, sizeof(double) * size_t(in_n), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  int rc = 0;
  double* res = h->host_buf.data();
  if (h->coll_fn) {
    if (kind == SFM_COLL_REDUCE_SCATTER) {
      h->host_buf2.resize(size_t(count));
      res = h->host_buf2.data();
    }
    rc = h->coll_fn(kind, h->host_buf.data(), res, count, arg, h->coll_user);
  } else if (kind == SFM_COLL_BROADCAST) {
    if (h->rank != arg) std::fill(h->host_buf.begin(), h->host_buf.end(), 0.0);
    rc = h->host_fn(h->host_buf.data(), count, 0, h->host_user);
  } else if (kind == SFM_COLL_REDUCE_SCATTER) {
    rc = h->host_fn(h->host_buf.data(), in_n, 0, h->host_user);
    res = h->host_buf.data() + size_t(h->rank) * size_t(count);
  } else {
    rc = h->host_fn(h->host_buf.data(), count, arg, h->host_user);
  }
  if (rc != 0) return fail(SFM_EIO, "host collective callback failed");
  HIPCHK(hipMemcpyAsync(kind == SFM_COLL_REDUCE_SCATTER ? out : buf, res, sizeof(double) * size_t(count),
                        hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

int broadcast(sfm_ba_handle* h, double* buf, int64_t count, int root) {
  if (h->host_fn || h->coll_fn) return host_collective(h, SFM_COLL_BROADCAST, buf, nullptr, count, root);
  if (!h->comm) return 0;
  NCCLCHK(ncclBroadcast(buf, buf, size_t(count), ncclDouble, root, h->comm, h->stream));
  return 0;
}

int reduce_scatter(sfm_ba_handle* h, double* send, double* recv, int64_t count) {
  if (h->host_fn || h->coll_fn) return host_collective(h, SFM_COLL_REDUCE_SCATTER, send, recv, count, 0);
  if (!h->comm) return 0;
  NCCLCHK(ncclReduceScatter(send, recv, size_t(count), ncclDouble, ncclSum, h->comm, h->stream));
  return 0;
}

// Sum of count doubles at send over the ranks, into recv on rank `root`.
int reduce_to(sfm_ba_handle* h, double* send, double* recv, int64_t count, int root, hipStream_t st) {
  if (h->host_fn || h->coll_fn) {
    h->host_buf.resize(size_t(count));
    HIPCHK(hipMemcpyAsync(h->host_buf.data(), send, sizeof(double) * size_t(count), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    int rc = h->coll_fn ? h->coll_fn(SFM_COLL_REDUCE, h->host_buf.data(), h->host_buf.data(), count, root, h->coll_user)
                        : h->host_fn(h->host_buf.data(), count, 0, h->host_user);  // (an all-reduce: root keeps it)
    if (rc != 0) return fail(SFM_EIO, "host collective callback failed");
    if (h->rank == root) {
      HIPCHK(hipMemcpyAsync(recv, h->host_buf.data(), sizeof(double) * size_t(count), hipMemcpyHostToDevice, st));
      HIPCHK(hipStreamSynchronize(st));
    }
    return 0;
  }
  if (!h->comm) return 0;
  NCCLCHK(ncclReduce(send, recv, size_t(count), ncclDouble, ncclSum, root, h->comm, st));
  return 0;
}

// The panel layout of the distributed factor and its buffers (remade when
// the problem size, the panel width or the rank layout changed).
int dist_prepare(sfm_ba_handle* h) {
  DevProblem& d = h->d;
  auto& D = h->dist;
  const int pt = h->dist_pt;
  if (D.send && D.pt == pt && D.nblk == d.nblk && D.n == d.n && D.nranks == h->nranks && D.rank == h->rank) return 0;
  HIPCHK(hipStreamSynchronize(h->stream));
  for (void* p : {static_cast<void*>(D.send), static_cast<void*>(D.recv), static_cast<void*>(D.bcast),
                  static_cast<void*>(D.off_send), static_cast<void*>(D.off_recv)})
    if (p) (void)hipFree(p);
  const hipStream_t cs = D.cstream;
  const hipEvent_t evs[5] = {D.ev_packed, D.ev_free[0], D.ev_free[1], D.ev_arrived[0], D.ev_arrived[1]};
  std::vector<hipEvent_t> ev_red = std::move(D.ev_red);
  const hipEvent_t ev_sent = D.ev_sent;
  D = sfm_ba_handle::DistBufs();
  D.ev_red = std::move(ev_red);
  D.ev_sent = ev_sent;
  D.cstream = cs;  // (kept for the handle's life)
  D.ev_packed = evs[0]; D.ev_free[0] = evs[1]; D.ev_free[1] = evs[2]; D.ev_arrived[0] = evs[3]; D.ev_arrived[1] = evs[4];
  if (!D.cstream) {
    HIPCHK(hipStreamCreateWithFlags(&D.cstream, hipStreamNonBlocking));
    for (hipEvent_t* e : {&D.ev_packed, &D.ev_free[0], &D.ev_free[1], &D.ev_arrived[0], &D.ev_arrived[1]})
      HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
  const int np = (d.nblk + pt - 1) / pt, N = h->nranks;
  D.count.assign(size_t(np), 0);
  D.poff.assign(size_t(np), 0);
  for (int J = 0; J < np; ++J) {
    const int c0 = J * pt * kNB, c1 = std::min((J + 1) * pt * kNB, d.n + 1);
    D.count[J] = c1 > c0 ? int64_t(c1 - c0) * (d.n + 1 - c0) : 0;
    D.poff[J] = D.total;
    D.total += D.count[J];
    D.bcast_cap = std::max<int64_t>(D.bcast_cap, D.count[J] + int64_t(pt) * kNB * kNB + 1);
  }
  std::vector<int64_t> os(static_cast<size_t>(np));
  for (int J = 0; J < np; ++J) os[J] = J % N == h->rank ? -1 : D.poff[J];
  auto grab = [&](void** p, size_t bytes) { return hipMalloc(p, std::max<size_t>(bytes, 256)) == hipSuccess; };
  if (!grab(reinterpret_cast<void**>(&D.send), sizeof(double) * size_t(D.total)) ||
      !grab(reinterpret_cast<void**>(&D.recv), sizeof(double) * size_t(D.total)) ||
      !grab(reinterpret_cast<void**>(&D.bcast), 2 * sizeof(double) * size_t(D.bcast_cap)) ||
      !grab(reinterpret_cast<void**>(&D.off_send), sizeof(int64_t) * np))
    return fail(SFM_ENOMEM, "hipMalloc failed (distributed factor buffers)");
  HIPCHK(hipMemcpy(D.off_send, os.data(), sizeof(int64_t) * np, hipMemcpyHostToDevice));
  // the own panels' regions of send stay zero: the owner's partial is
  // updated in place and the others' sum is added just before its factor
  HIPCHK(hipMemsetAsync(D.send, 0, sizeof(double) * size_t(D.total), h->stream));
  while (int(D.ev_red.size()) < np) {
    hipEvent_t e;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    D.ev_red.push_back(e);
  }
  if (!D.ev_sent) HIPCHK(hipEventCreateWithFlags(&D.ev_sent, hipEventDisableTiming));
  D.pt = pt; D.nblk = d.nblk; D.n = d.n; D.nranks = N; D.rank = h->rank;
  return 0;
}

// The reduced camera system's factor, distributed:
// the ranks' partial systems are summed per column panel into its owner (a
// reduce per panel, not one reduce-scatter up front), per panel k its owner
// factors it and broadcasts L (+ its W_k tiles and failure bits), every rank
// applies it to its own later panels; then every rank holds the whole factor
// and back-substitutes (replicated).
// * The owner updates its OWN partial of a panel in place and adds the other
//   ranks' sum (its own region of the send buffer is zero) just before
//   factoring it: the updates are linear, so the panels' reduces can run
//   beside the factorisation instead of ahead of it.
// * Look-ahead: having panel k, the owner of k+1 first updates that panel
//   alone, adds its reduce, factors and packs it, and only then applies
//   panel k to its other panels.
// * Under RCCL the collectives run on a second stream of the handle in the
//   order reduce 0, reduce 1, then per k: broadcast k, reduce k+2 -- so the
//   reduce of a panel lands one step before its owner needs it, and the
//   broadcast of k+1 overlaps the bulk updates (two broadcast buffers,
//   events order each buffer's reuse after its last reader).
// Every panel takes its updates in panel order on every rank count.
int dist_factor_enqueue(sfm_ba_handle* h) {
  SFM_TRACE("sfm:dist_factor");
  DevProblem& d = h->d;
  hipStream_t s = h->stream;
  int rc;
  if ((rc = dist_prepare(h))) return rc;
  auto& D = h->dist;
  const int pt = D.pt, N = h->nranks, me = h->rank, np = int(D.count.size());
  // The broadcasts on a second stream of the handle (the collective stream,
  // two broadcast buffers and the events that order their reuse) only with
  // SFM_DIST_OVERLAP=1.  Its non-owner branches (the wait on ev_free, the
  // unpack, a half reused across owners) have never run with more than one
  // RCCL rank -- no second GPU was ever available to this build, and RCCL
  // takes one rank per GPU -- so the multi-GPU default is the schedule the
  // 2-4-rank host-hook tests run (tests/test_gpu_shards.py), the same order
  // of operations on one stream.  On one rank (RCCL's collectives local) the
  // flag is the one-GPU test of the look-ahead plumbing, tests/test_gpu_scale.py.
  static const bool force_overlap = env_flag("SFM_DIST_OVERLAP");
  const bool overlap = h->comm != nullptr && force_overlap;
  const bool comm = N > 1 || overlap;
  hipStream_t cs = overlap ? D.cstream : s;
  launch_panel_copy(d, kPanelPack, pt, 0, d.n + 1, D.off_send, 0, D.send, s);
  if (overlap) {
    HIPCHK(hipEventRecord(D.ev_sent, s));
    HIPCHK(hipStreamWaitEvent(cs, D.ev_sent, 0));
    // both broadcast halves free from here (the last factor's readers are before this on s)
    HIPCHK(hipEventRecord(D.ev_free[0], s));
    HIPCHK(hipEventRecord(D.ev_free[1], s));
  }
  auto reduce_panel = [&](int k) -> int {
    if (!comm || k >= np) return 0;
    if (int e = reduce_to(h, D.send + D.poff[k], D.recv + D.poff[k], D.count[k], k % N, cs)) return e;
    if (overlap && k % N == me) HIPCHK(hipEventRecord(D.ev_red[k], cs));
    return 0;
  };
  auto geom = [&](int k, int* t0, int* c0, int* c1, int64_t* nw) {
    *t0 = k * pt;
    const int ncols = std::min(pt, d.nblk - *t0);
    *c0 = *t0 * kNB;
    *c1 = *c0 + ncols * kNB;
    *nw = int64_t(ncols) * kNB * kNB;
  };
  auto half = [&](int k) { return D.bcast + size_t(k & 1) * size_t(D.bcast_cap); };
  // the owner's part: the other ranks' sum into its updated partial, factor
  // panel k, pack L + W_k tiles + failure bits
  auto factor_pack = [&](int k) -> int {
    int t0, c0, c1;
    int64_t nw;
    geom(k, &t0, &c0, &c1, &nw);
    if (comm) {
      if (overlap) HIPCHK(hipStreamWaitEvent(s, D.ev_red[k], 0));
      launch_panel_copy(d, kPanelAdd, pt, c0, c1, nullptr, D.poff[k], D.recv, s);
    }
    double* b = half(k);
    launch_cholesky_panel(d, k, pt, ++h->chol_epoch, s);
    launch_panel_copy(d, kPanelPack, pt, c0, c1, nullptr, 0, b, s);
    HIPCHK(hipMemcpyAsync(b + D.count[k], d.invL + size_t(t0) * kNB * kNB, sizeof(double) * size_t(nw),
                          hipMemcpyDeviceToDevice, s));
    launch_fail_slot(d, true, b + D.count[k] + nw, s);
    if (overlap) HIPCHK(hipEventRecord(D.ev_packed, s));
    return 0;
  };
  if ((rc = reduce_panel(0)) || (rc = reduce_panel(1))) return rc;
  if (np > 0 && me == 0 && (rc = factor_pack(0))) return rc;
  for (int k = 0; k < np; ++k) {
    const int owner = k % N;
    int t0, c0, c1;
    int64_t nw;
    geom(k, &t0, &c0, &c1, &nw);
    double* b = half(k);
    const int64_t cnt = D.count[k] + nw + 1;
    if (comm) {
      if (overlap) {
        // the half is packed (owner) / no longer read by panel k-2's unpack
        if (me == owner) HIPCHK(hipStreamWaitEvent(cs, D.ev_packed, 0));
        else HIPCHK(hipStreamWaitEvent(cs, D.ev_free[k & 1], 0));
        NCCLCHK(ncclBroadcast(b, b, size_t(cnt), ncclDouble, owner, h->comm, cs));
        HIPCHK(hipEventRecord(D.ev_arrived[k & 1], cs));
      } else if ((rc = broadcast(h, b, cnt, owner))) {
        return rc;
      }
      if ((rc = reduce_panel(k + 2))) return rc;
      if (overlap) HIPCHK(hipStreamWaitEvent(s, D.ev_arrived[k & 1], 0));
    }
    if (me != owner) {
      launch_panel_copy(d, kPanelUnpack, pt, c0, c1, nullptr, 0, b, s);
      HIPCHK(hipMemcpyAsync(d.invL + size_t(t0) * kNB * kNB, b + D.count[k], sizeof(double) * size_t(nw),
                            hipMemcpyDeviceToDevice, s));
      launch_fail_slot(d, false, b + D.count[k] + nw, s);
      if (overlap) HIPCHK(hipEventRecord(D.ev_free[k & 1], s));
    }
    if (k + 1 < np && (k + 1) % N == me) {
      launch_panel_update(d, k, k + 1, k + 1, pt, N, me, s);  // the next panel first (look-ahead)
      if ((rc = factor_pack(k + 1))) return rc;
    }
    launch_panel_update(d, k, k + 2, INT32_MAX / 2, pt, N, me, s);  // (k+1 is not ours unless updated above)
  }
  return 0;
}

// D2H of the scalar block + stream sync.
int fetch_scalars(sfm_ba_handle* h) {
  HIPCHK(hipMemcpyAsync(h->d.scal_host, h->d.scal, sizeof(double) * (kNumScalars + 1), hipMemcpyDeviceToHost,
                        h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  collect_marks(h);
  return 0;
}

// A phase's closing reduction; in the fused device loop (h->fuse_lm) with
// the bookkeeping that follows it: k_lm_decide after compute_step
// (kTailDecide), k_lm_post after an evaluation (kTailPost), k_lm_init after
// the initial one (kTailInit).
void reduce_phase(sfm_ba_handle* h, const ReduceBatch& rb, bool copy_fail, int tail) {
  DevProblem& d = h->d;
  if (h->fuse_lm && rb.n > 0) {
#define SFM_RB_LM(T_)                                                                                      \
  k_reduce_batch_lm<T_><<<rb.n, 1024, 0, h->stream>>>(d.partials, d.max_blocks, rb, d.scal,                 \
                                                      copy_fail ? d.fail : nullptr, d.gate, h->lm_ctl,      \
                                                      h->lm_trace, h->lm_trace_cap, af)
    AcceptFold af{};
    if (tail == kTailPost) SFM_RB_LM(kTailPost);
    else if (tail == kTailInit) SFM_RB_LM(kTailInit);
    else {
      if (h->accept_fold)
        af = AcceptFold{d.C, 3 * int64_t(d.P), d.cam, d.camR,
                        h->mode != SFM_BA_STRUCT_ONLY ? d.partials + size_t(kPXNormCam) * d.max_blocks : nullptr,
                        d.cam_new, d.X_new, d.X};
      SFM_RB_LM(kTailDecide);
    }
#undef SFM_RB_LM
    return;
  }
  launch_reduce_batch(d, rb, copy_fail, h->stream);
}

// Evaluate cost, Jacobian, Jacobi scale (first call), per-block normal
// equations, LM diagonal and gradient at the current parameters.
int evaluate_enqueue(sfm_ba_handle* h, bool first, bool jacobi_scaling) {
  SFM_TRACE("sfm:evaluate");
  DevProblem& d = h->d;
  hipStream_t s = h->stream;
  int rc;
  // constant blocks (STRUCT_ONLY: cameras, POSE_ONLY: points) carry a zero
  // Jacobi scale, so their scaled Jacobian columns vanish; their norms and
  // gradients are left out like Ceres leaves out constant blocks
  const bool cams_var = h->mode != SFM_BA_STRUCT_ONLY, pts_var = h->mode != SFM_BA_POSE_ONLY;
  const int nbP = std::max(1, blocks_for(d.P, 256)),
            nbC = std::max(1, blocks_for(d.C, 256));
  if (h->accept_grid > 0) launch_cam_prep_accept(d, cams_var, h->accept_grid, s);
  else if (h->accept_grid == 0) launch_cam_prep(d, d.cam, cams_var, s);
  // accept_grid < 0: done by the deciding workgroup (AcceptFold)
  mark_begin(h, kPhJac);
  launch_jacobian(d, !first || !jacobi_scaling ? true : false, s);
  mark_end(h);
  // unsharded: the U_c sums and their finalisation in one launch
  const bool fuse_cam = !sharded(h);
  // small systems (C <= 64): the camera sums ride in the point pass's launch
  const bool fold_cams = fuse_cam && cams_var && pts_var && d.P > 0 && d.C > 0 && d.C <= 64;
  if (first && jacobi_scaling) {
    if (fold_cams) {
      mark_begin(h, kPhPtEval);
      launch_point_eval_with_cams(d, 0, false, s);
      mark_end(h);
    } else {
      if (cams_var) {
        mark_begin(h, kPhCamRed);
        if (fuse_cam) {
          launch_cam_sum_finalize(d, 0, false, s);
        } else {
          launch_cam_reduce(d, s);
          if ((rc = allreduce(h, d.Ucam, size_t(kUcam) * d.C, ncclSum))) return rc;
          launch_cam_finalize(d, 0, false, false, s);
        }
        mark_end(h);
      }
      if (pts_var) launch_point_eval(d, 0, false, s);
    }
    mark_begin(h, kPhJac);
    launch_jacobian(d, true, s);
    mark_end(h);
  }
  if (fold_cams) {
    mark_begin(h, kPhPtEval);
    launch_point_eval_with_cams(d, 1, true, s);
    mark_end(h);
  } else if (cams_var) {
    mark_begin(h, kPhCamRed);
    if (fuse_cam) {
      launch_cam_sum_finalize(d, 1, true, s);
    } else {
      launch_cam_reduce(d, s);
      if ((rc = allreduce(h, d.Ucam, size_t(kUcam) * d.C, ncclSum))) return rc;
      launch_cam_finalize(d, 1, false, true, s);
    }
    mark_end(h);
  } else {
    hipMemsetAsync(d.partials + size_t(kPGradCam) * d.max_blocks, 0, sizeof(double) * nbC, s);
    hipMemsetAsync(d.partials + size_t(kPXNormCam) * d.max_blocks, 0, sizeof(double) * nbC, s);
  }
  if (fold_cams) {
    // (done above, with the camera sums)
  } else if (pts_var) {
    mark_begin(h, kPhPtEval);
    launch_point_eval(d, 1, false, s);
    mark_end(h);
  } else {
    hipMemsetAsync(d.partials + size_t(kPGradPt) * d.max_blocks, 0, sizeof(double) * nbP, s);
    hipMemsetAsync(d.partials + size_t(kPXNormPt) * d.max_blocks, 0, sizeof(double) * nbP, s);
  }
  if (d.N == 0) hipMemsetAsync(d.partials + size_t(kPCost) * d.max_blocks, 0, sizeof(double), s);
  if (d.P == 0) {
    hipMemsetAsync(d.partials + size_t(kPGradPt) * d.max_blocks, 0, sizeof(double), s);
    hipMemsetAsync(d.partials + size_t(kPXNormPt) * d.max_blocks, 0, sizeof(double), s);
  }
  ReduceBatch rb;
  rb.add(kPCost, d.jac_blocks, 0, kCost);
  rb.add(kPGradCam, cams_var && fuse_cam ? std::max(1, d.C) : nbC, 1, kGradMaxCam);
  rb.add(kPGradPt, nbP, 1, kGradMaxPt);
  rb.add(kPXNormCam, nbC, 0, kXNorm2Cam);
  rb.add(kPXNormPt, nbP, 0, kXNorm2Pt);
  reduce_phase(h, rb, false, first ? kTailInit : kTailPost);
  if (sharded(h)) {
    if ((rc = allreduce(h, d.scal + kCost, 1, ncclSum))) return rc;
    if ((rc = allreduce(h, d.scal + kGradMaxCam, 2, ncclMax))) return rc;
    if ((rc = allreduce(h, d.scal + kXNorm2Pt, 1, ncclSum))) return rc;
  }
  return 0;
}
int evaluate(sfm_ba_handle* h, bool first, bool jacobi_scaling) {
  if (int rc = evaluate_enqueue(h, first, jacobi_scaling)) return rc;
  return fetch_scalars(h);
}

// One trust-region step: factor, Schur, dense Cholesky, back substitution,
// model cost change and candidate cost.
int compute_step_enqueue(sfm_ba_handle* h, double radius) {
  SFM_TRACE("sfm:compute_step");
  DevProblem& d = h->d;
  hipStream_t s = h->stream;
  int rc;
  const int nbP = std::max(1, blocks_for(d.P, 256)), nbC = std::max(1, blocks_for(d.C, 256));
  bool cam_done = false;  // the camera step taken by the small-system factor
  if (h->mode == SFM_BA_STRUCT_AND_POSE && d.overlap && d.C && !sharded(h) && !h->force_pack) {
    // Schur / Cholesky overlap: the diagonal blocks and rhs first, then the
    // factorisation on its own stream with half the CUs while k_schur_pts
    // fills the off-diagonal blocks on the other half, in camera-major order
    // (the factor's tile columns complete left to right); a helper reads an
    // S tile once k_schur_pts has counted all its camera blocks in
    mark_begin(h, kPhPtPrep);
    launch_point_prep(d, radius, s);
    mark_end(h);
    if (!h->stream2) {
      HIPCHK(hipStreamCreateWithFlags(&h->stream2, hipStreamNonBlocking));
      HIPCHK(hipEventCreateWithFlags(&h->ov_ev[0], hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&h->ov_ev[1], hipEventDisableTiming));
    }
    const int m_schur = mark_begin(h, kPhSchur);
    HIPCHK(hipMemsetAsync(d.tile_cnt, 0, sizeof(int32_t) * size_t(d.nblk) * d.nblk, s));
    launch_schur_diag(d, radius, h->rank == 0, s);
    HIPCHK(hipEventRecord(h->ov_ev[0], s));
    HIPCHK(hipStreamWaitEvent(h->stream2, h->ov_ev[0], 0));
    mark_begin(h, kPhChol, h->stream2);
    launch_cholesky(d, ++h->chol_epoch, h->stream2, false, -1, d.overlap);
    mark_end(h, h->stream2);
    launch_schur_offdiag(d, d.tile_cnt, s);
    HIPCHK(hipEventRecord(h->ov_ev[1], h->stream2));
    HIPCHK(hipStreamWaitEvent(s, h->ov_ev[1], 0));
    mark_end(h, nullptr, m_schur);  // (after the join: the Schur phase spans the overlapped factor)
    mark_begin(h, kPhBack);
    launch_backsolve(d, ++h->bs_epoch, s, true);
    mark_end(h);
  } else if (h->mode == SFM_BA_STRUCT_AND_POSE) {
    mark_begin(h, kPhPtPrep);
    launch_point_prep(d, radius, s);
    mark_end(h);
    mark_begin(h, kPhSchur);
    launch_schur(d, radius, h->rank == 0, s);
    mark_end(h);
    // (k_schur_diag_sum also wrote the identity padding, y's sentinel and
    // the cleared failure flag; without cameras the separate launch does)
    if (!d.C) launch_pad_init(d, s);
    if (sharded(h) && h->dist_pt > 0) {
      mark_begin(h, kPhChol);
      if ((rc = dist_factor_enqueue(h))) return rc;
      mark_end(h);
    } else {
      if (sharded(h) || h->force_pack) {
        // all-reduce only the packed upper triangle + rhs (half the ld^2 image)
        launch_pack_upper(d, false, s);
        if ((rc = allreduce(h, d.Spack, packed_size(d.n), ncclSum))) return rc;
        launch_pack_upper(d, true, s);
      }
      mark_begin(h, kPhChol);
      cam_done = launch_cholesky(d, ++h->chol_epoch, s, false, h->rank == 0 ? 1 : 0);
      mark_end(h);
    }
    mark_begin(h, kPhBack);
    launch_backsolve(d, ++h->bs_epoch, s, true);
    mark_end(h);
  } else if (h->mode == SFM_BA_POSE_ONLY) {
    // block-diagonal camera system from the all-reduced U_c (same on every rank)
    launch_cam_solve(d, radius, s);
    // the back substitution reads X from the point records (their factor
    // is unused here: y_p = 0); its bad flags are cleared below
    if (d.P) launch_point_factor(d, radius, s);
    hipMemsetAsync(d.partials + size_t(kPBad) * d.max_blocks, 0, sizeof(double) * nbP, s);
  } else {
    // STRUCT_ONLY: per-point 3x3 systems only; y_c = 0
    hipMemsetAsync(d.fail, 0, sizeof(int), s);
    if (d.P) {
      mark_begin(h, kPhPtPrep);
      launch_point_factor(d, radius, s);
      mark_end(h);
    }
    hipMemsetAsync(d.ysol, 0, sizeof(double) * 6 * size_t(d.C), s);
  }
  if (!cam_done) launch_cam_update(d, h->rank == 0 && h->mode != SFM_BA_STRUCT_ONLY, s);
  mark_begin(h, kPhBacksub);
  launch_point_backsub(d, s, h->mode != SFM_BA_STRUCT_ONLY, h->mode != SFM_BA_POSE_ONLY);
  mark_end(h);
  if (d.P == 0) {
    const int slots[] = {kPModel, kPModelPt, kPNewCost, kPStepPt, kPBadBack, kPBad};
    for (int sl : slots) hipMemsetAsync(d.partials + size_t(sl) * d.max_blocks, 0, sizeof(double), s);
  }
  if (h->rank != 0 || h->mode == SFM_BA_STRUCT_ONLY)
    hipMemsetAsync(d.partials + size_t(kPStepCam) * d.max_blocks, 0, sizeof(double) * nbC, s);
  const int nbI = d.N_pad ? obs_xcd_blocks(d) : 1;  // k_backsub_a_rc / k_backsub_c grid
  const int nbB = d.P ? pt_xcd_blocks(d) : 1;       // k_backsub_b grid
  ReduceBatch rb;
  rb.add(kPModel, nbI, 0, kModelChange);
  rb.add(kPNewCost, nbI, 0, kNewCost);
  rb.add(kPStepPt, nbB, 0, kStep2Pt);
  rb.add(kPStepCam, nbC, 0, kStep2Cam);
  // bad-step flags: max over point_prep, cam_update and backsub partials
  rb.add(kPBad, nbP, 1, kBadStep);
  rb.add(kPBadCam, nbC, 1, kBadCam);
  rb.add(kPBadBack, nbB, 1, kBadBack);
  rb.add(kPModelPt, nbB, 0, kModelChangePt);
  // ... and the Cholesky failure flag (an int) into the slot after the scalars
  reduce_phase(h, rb, true, kTailDecide);
  if (sharded(h)) {
    if ((rc = allreduce(h, d.scal + kModelChange, 4, ncclSum))) return rc;  // model, new cost, step pt, step cam
    if ((rc = allreduce(h, d.scal + kBadStep, 4, ncclMax))) return rc;
    if ((rc = allreduce(h, d.scal + kModelChangePt, 1, ncclSum))) return rc;
  }
  return 0;
}
int compute_step(sfm_ba_handle* h, double radius) {
  if (int rc = compute_step_enqueue(h, radius)) return rc;
  return fetch_scalars(h);
}

// Ceres 1.12 Solver::Options::IsValid (CommonOptionsAreValid +
// TrustRegionOptionsAreValid): ceres::Solve refuses options that fail these
// (the reference only sets linear_solver_type, CTracker.cpp:571-577).
// Returns the offending rule, or nullptr.
const char* invalid_option(const sfm_ba_options& o) {
  if (!(o.max_num_iterations >= 0)) return "max_num_iterations >= 0";
  if (!(o.max_num_consecutive_invalid_steps >= 0)) return "max_num_consecutive_invalid_steps >= 0";
  if (!(o.function_tolerance >= 0)) return "function_tolerance >= 0";
  if (!(o.gradient_tolerance >= 0)) return "gradient_tolerance >= 0";
  if (!(o.parameter_tolerance >= 0)) return "parameter_tolerance >= 0";
  if (!(o.initial_trust_region_radius > 0)) return "initial_trust_region_radius > 0";
  if (!(o.min_trust_region_radius > 0)) return "min_trust_region_radius > 0";
  if (!(o.max_trust_region_radius > 0)) return "max_trust_region_radius > 0";
  if (!(o.min_trust_region_radius <= o.max_trust_region_radius)) return "min_trust_region_radius <= max";
  if (!(o.min_trust_region_radius <= o.initial_trust_region_radius)) return "min_trust_region_radius <= initial";
  if (!(o.initial_trust_region_radius <= o.max_trust_region_radius)) return "initial_trust_region_radius <= max";
  if (!(o.min_relative_decrease >= 0)) return "min_relative_decrease >= 0";
  if (!(o.min_lm_diagonal >= 0)) return "min_lm_diagonal >= 0";
  if (!(o.max_lm_diagonal >= 0)) return "max_lm_diagonal >= 0";
  if (!(o.min_lm_diagonal <= o.max_lm_diagonal)) return "min_lm_diagonal <= max_lm_diagonal";
  return nullptr;
}

// The device-driven LM loop of sfm_ba_solve_resident (all but the
// host-callback collective), initial evaluation included:
// state in LmCtl, initialised on the device from the initial evaluation
// (k_lm_init: no host round trip before the first iteration), iterations
// enqueued in batches (3, then 2; SFM_LM_BATCH fixes the size), the host
// reads the control block once per batch.  The gated kernels of iterations
// enqueued past the end return at once.  *nonfinite: the initial cost was
// not finite (the summary is then the host loop's FAILURE).
template <class Push>
int run_device_lm(sfm_ba_handle* h, const sfm_ba_options& opts, double* cost, sfm_ba_summary* sm, Push& push,
                  bool* nonfinite) {
  DevProblem& d = h->d;
  hipStream_t s = h->stream;
  HostTimer timer;
  timer.tag = "solve";
  if (!h->lm_ctl) {
    if (hipMalloc(reinterpret_cast<void**>(&h->lm_ctl), sizeof(LmCtl)) != hipSuccess) {
      h->lm_ctl = nullptr;
      return fail(SFM_ENOMEM, "hipMalloc failed (LM control)");
    }
    if (hipHostMalloc(reinterpret_cast<void**>(&h->lm_ctl_host), sizeof(LmCtl)) != hipSuccess) {
      h->lm_ctl_host = nullptr;
      return fail(SFM_ENOMEM, "hipHostMalloc failed (LM control)");
    }
  }
  const int cap = std::max(1, opts.max_num_iterations + 1);
  if (h->lm_trace_cap < cap) {
    if (h->lm_trace) {
      (void)hipStreamSynchronize(s);
      (void)hipHostFree(h->lm_trace);
    }
    h->lm_trace = nullptr;
    h->lm_trace_cap = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&h->lm_trace), sizeof(sfm_ba_iteration) * size_t(cap)) != hipSuccess) {
      h->lm_trace = nullptr;
      return fail(SFM_ENOMEM, "hipMalloc failed (LM trace)");
    }
    h->lm_trace_cap = cap;
  }
  LmCtl& c = *h->lm_ctl_host;
  std::memset(&c, 0, sizeof(c));
  c.run_step = 1;
  c.radius = opts.initial_trust_region_radius;
  c.decrease_factor = 2.0;
  c.max_iter = opts.max_num_iterations;
  c.max_invalid = opts.max_num_consecutive_invalid_steps;
  c.ftol = opts.function_tolerance;
  c.gtol = opts.gradient_tolerance;
  c.ptol = opts.parameter_tolerance;
  c.max_radius = opts.max_trust_region_radius;
  c.min_radius = opts.min_trust_region_radius;
  c.min_rel_dec = opts.min_relative_decrease;
  HIPCHK(hipMemcpyAsync(h->lm_ctl, &c, sizeof(LmCtl), hipMemcpyHostToDevice, s));
  // 3 iterations first (a keyframe or C3 solve typically ends there), then 2
  // at a time: each gated iteration past the end still costs its launches
  // (measured per C1 solve: batch 3 0.49 ms, 4 0.52, 6 0.62; host loop 0.54)
  int batch = 3, batch_next = 2;
  if (const char* b = std::getenv("SFM_LM_BATCH")) batch = batch_next = std::max(1, std::min(64, std::atoi(b)));
  if (opts.max_num_iterations <= 0) batch = 0;  // k_lm_init ends the solve (NO_CONVERGENCE unless converged)
  const bool jac_scaling = opts.jacobi_scaling != 0;
  const int acc_blocks = std::max(1, std::min(1024, blocks_for(6 * int64_t(d.C) + 3 * int64_t(d.P), 256)));
  d.radius_dev = &h->lm_ctl->radius;
  // without a collective between a phase's reduction and the bookkeeping,
  // the two are one launch (k_reduce_batch_lm)
  h->fuse_lm = !sharded(h) && !env_flag("SFM_LM_UNFUSED");
  h->accept_fold = h->fuse_lm && d.C > 0 && d.C <= kAcceptFoldMaxCams && 3 * int64_t(d.P) <= kAcceptFoldMaxX &&
                   !env_flag("SFM_NO_ACCEPT_FOLD");
  // the initial evaluation (Jacobi scaling on first use); its scalars
  // initialise the loop state on the device
  d.gate = nullptr;
  int rc = evaluate_enqueue(h, true, jac_scaling);
  if (rc == 0 && !h->fuse_lm) k_lm_init<<<1, 1, 0, s>>>(h->lm_ctl, d.scal);
  while (rc == 0) {
    for (int b = 0; b < batch && rc == 0; ++b) {
      d.gate = &h->lm_ctl->run_step;
      if ((rc = compute_step_enqueue(h, c.radius))) break;
      d.gate = nullptr;
      if (!h->fuse_lm) k_lm_decide<<<1, 1, 0, s>>>(h->lm_ctl, d.scal, h->lm_trace, h->lm_trace_cap);
      d.gate = &h->lm_ctl->run_eval;
      // k_lm_accept's copy inside the evaluation's k_cam_prep, or already
      // done in the deciding workgroup
      h->accept_grid = h->accept_fold ? -1 : acc_blocks;
      rc = evaluate_enqueue(h, false, jac_scaling);
      h->accept_grid = 0;
      if (rc) break;
      d.gate = nullptr;
      if (!h->fuse_lm) k_lm_post<<<1, 1, 0, s>>>(h->lm_ctl, d.scal, h->lm_trace, h->lm_trace_cap);
    }
    if (rc) break;
    timer.mark("batch enqueued");
    if (h->prefetch_params) {
      if (hipMemcpyAsync(h->param_host, d.cam, sizeof(double) * 6 * size_t(d.C), hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipMemcpyAsync(h->param_host + 6 * size_t(d.C), d.X, sizeof(double) * 3 * size_t(d.P), hipMemcpyDeviceToHost,
                         s) != hipSuccess) {
        rc = fail(SFM_EIO, "parameter readback failed");
        break;
      }
    }
    if (hipMemcpyAsync(&c, h->lm_ctl, sizeof(LmCtl), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      rc = fail(SFM_EIO, "LM control readback failed");
      break;
    }
    timer.mark("batch synchronised");
    collect_marks(h);
    if (c.done) break;
    batch = batch_next;
  }
  d.gate = nullptr;
  d.radius_dev = nullptr;
  h->fuse_lm = false;
  h->accept_fold = false;
  if (rc) return rc;
  if (c.error & 4) return fail(SFM_EIO, "Cholesky tile hand-off timed out (persistent grid made no progress)");
  if (c.error & 2) return fail(SFM_EIO, "back-substitution hand-off timed out (persistent grid made no progress)");
  sm->num_jacobian_evaluations++;  // the initial evaluation
  sm->num_residual_evaluations++;
  sm->initial_cost = c.init_cost;
  if (c.error & 8) {
    *nonfinite = true;
    sm->termination_type = SFM_FAILURE;
    sm->final_cost = c.init_cost;
    return fail(SFM_EIO, "initial residual evaluation is not finite");
  }
  {
    sfm_ba_iteration it0;
    std::memset(&it0, 0, sizeof(it0));
    it0.cost = c.init_cost;
    it0.gradient_max_norm = c.init_grad;
    it0.trust_region_radius = opts.initial_trust_region_radius;
    it0.step_is_valid = 1;
    it0.step_is_successful = 1;
    push(it0);
  }
  const int n_tr = std::min(c.trace_len, h->lm_trace_cap);
  // (written to pinned host memory, complete at the last batch's synchronisation)
  for (int i = 0; i < n_tr; ++i) push(h->lm_trace[i]);
  h->param_host_valid = h->prefetch_params;
  sm->termination_type = c.termination;
  sm->num_iterations = c.iteration;
  sm->num_successful_steps += c.n_succ;
  sm->num_unsuccessful_steps += c.n_unsucc;
  sm->num_invalid_steps += c.n_invalid;
  sm->num_residual_evaluations += c.n_resid;
  sm->num_jacobian_evaluations += c.n_jac;
  sm->num_linear_solves += c.n_lin;
  *cost = c.cost;
  return 0;
}

}  // namespace

extern "C" {

int32_t sfm_abi_version(void) { return SFM_ABI_VERSION; }
const char* sfm_last_error(void) { return g_err.c_str(); }

void sfm_ba_default_options(sfm_ba_options* o) {
  o->max_num_iterations = 50;
  o->max_num_consecutive_invalid_steps = 5;
  o->jacobi_scaling = 1;
  o->reserved0 = 0;
  o->function_tolerance = 1e-6;
  o->gradient_tolerance = 1e-10;
  o->parameter_tolerance = 1e-8;
  o->initial_trust_region_radius = 1e4;
  o->max_trust_region_radius = 1e16;
  o->min_trust_region_radius = 1e-32;
  o->min_lm_diagonal = 1e-6;
  o->max_lm_diagonal = 1e32;
  o->min_relative_decrease = 1e-3;
}

int32_t sfm_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int sfm_ba_create(int32_t device, sfm_ba_handle** out) {
  if (!out) return fail(SFM_EINVAL, "out is NULL");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(SFM_ENODEV, "no HIP device visible");
  if (device < 0 || device >= n) return fail(SFM_EINVAL, "device ordinal out of range");
  HIPCHK(hipSetDevice(device));
  auto* h = new sfm_ba_handle();
  h->device = device;
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return fail(SFM_EIO, "hipStreamCreate failed");
  }
  h->n_cu = device_cus(device);  // (hipGetDeviceProperties: once, not per set_problem)
  *out = h;
  return 0;
}

int sfm_ba_destroy(sfm_ba_handle* h) {
  if (!h) return 0;
  hipSetDevice(h->device);
  hipStreamSynchronize(h->stream);
  free_problem(h);
  release_pool(h);
  if (h->d.scal_host) hipHostFree(h->d.scal_host);
  if (h->lm_ctl) hipFree(h->lm_ctl);
  if (h->lm_ctl_host) hipHostFree(h->lm_ctl_host);
  if (h->lm_trace) hipHostFree(h->lm_trace);
  if (h->param_host) hipHostFree(h->param_host);
  if (h->stage) hipHostFree(h->stage);
  if (h->ar_tmp) hipFree(h->ar_tmp);
  for (void* p : {static_cast<void*>(h->dist.send), static_cast<void*>(h->dist.recv),
                  static_cast<void*>(h->dist.bcast), static_cast<void*>(h->dist.off_send),
                  static_cast<void*>(h->dist.off_recv)})
    if (p) hipFree(p);
  if (h->dist.cstream) {
    hipStreamSynchronize(h->dist.cstream);
    hipStreamDestroy(h->dist.cstream);
    for (hipEvent_t e : {h->dist.ev_packed, h->dist.ev_free[0], h->dist.ev_free[1], h->dist.ev_arrived[0],
                         h->dist.ev_arrived[1]})
      hipEventDestroy(e);
  }
  for (hipEvent_t e : h->dist.ev_red) hipEventDestroy(e);
  if (h->dist.ev_sent) hipEventDestroy(h->dist.ev_sent);
  if (h->stream2) {
    hipStreamSynchronize(h->stream2);
    hipStreamDestroy(h->stream2);
    hipEventDestroy(h->ov_ev[0]);
    hipEventDestroy(h->ov_ev[1]);
  }
  if (h->ustream) {
    hipStreamSynchronize(h->ustream);
    hipStreamDestroy(h->ustream);
    hipEventDestroy(h->uev);
    if (h->uev_uv) hipEventDestroy(h->uev_uv);
  }
  for (auto e : h->ev) hipEventDestroy(e);
  if (h->comm) ncclCommDestroy(h->comm);
  hipStreamDestroy(h->stream);
  delete h;
  return 0;
}

int sfm_comm_unique_id(uint8_t out[128]) {
  ncclUniqueId id;
  NCCLCHK(ncclGetUniqueId(&id));
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  std::memcpy(out, &id, 128);
  return 0;
}

int sfm_ba_set_comm(sfm_ba_handle* h, int32_t nranks, int32_t rank, const uint8_t id[128]) {
  if (!h || nranks < 1 || rank < 0 || rank >= nranks) return fail(SFM_EINVAL, "bad communicator arguments");
  HIPCHK(hipSetDevice(h->device));
  if (h->comm) { ncclCommDestroy(h->comm); h->comm = nullptr; }
  h->host_fn = nullptr;
  h->coll_fn = nullptr;
  h->nranks = nranks;
  h->rank = rank;
  // a one-rank communicator is created too: it runs every collective of the
  // sharded path (identities over one rank), which the one-GPU tests use
  ncclUniqueId uid;
  std::memcpy(&uid, id, 128);
  NCCLCHK(ncclCommInitRank(&h->comm, nranks, uid, rank));
  h->emulate_ranks = 1;
  if (const char* e = std::getenv("SFM_EMULATE_IDENTICAL_RANKS")) h->emulate_ranks = std::max(1, std::atoi(e));
  return 0;
}

int sfm_ba_set_host_comm(sfm_ba_handle* h, int32_t nranks, int32_t rank, sfm_allreduce_fn fn, void* user) {
  if (!h || nranks < 1 || rank < 0 || rank >= nranks || !fn) return fail(SFM_EINVAL, "bad communicator arguments");
  if (h->comm) { ncclCommDestroy(h->comm); h->comm = nullptr; }
  h->nranks = nranks;
  h->rank = rank;
  h->host_fn = fn;
  h->host_user = user;
  h->coll_fn = nullptr;
  h->coll_user = nullptr;
  return 0;
}

// An all-reduce hook built from the general one (kind SFM_COLL_ALLREDUCE).
namespace {
int coll_as_allreduce(double* buf, int64_t count, int32_t op, void* user) {
  auto* h = static_cast<sfm_ba_handle*>(user);
  return h->coll_fn(SFM_COLL_ALLREDUCE, buf, buf, count, op, h->coll_user);
}
}  // namespace

int sfm_ba_set_host_collectives(sfm_ba_handle* h, int32_t nranks, int32_t rank, sfm_collective_fn fn, void* user) {
  if (!h || nranks < 1 || rank < 0 || rank >= nranks || !fn) return fail(SFM_EINVAL, "bad communicator arguments");
  if (h->comm) { ncclCommDestroy(h->comm); h->comm = nullptr; }
  h->nranks = nranks;
  h->rank = rank;
  h->coll_fn = fn;
  h->coll_user = user;
  h->host_fn = coll_as_allreduce;  // the sharded path's all-reduces
  h->host_user = h;
  return 0;
}

int sfm_ba_set_distributed_factor(sfm_ba_handle* h, int32_t panel_tiles) {
  if (!h || panel_tiles < 0 || panel_tiles > 64) return fail(SFM_EINVAL, "panel_tiles must be in [0, 64]");
  h->dist_pt = panel_tiles;
  return 0;
}

int sfm_ba_set_problem(sfm_ba_handle* h, int64_t n_obs, const double* obs_uv, const int32_t* cam_idx,
                       const int32_t* pt_idx, int32_t n_cams, const double* K9, const double* rot, const double* t,
                       int32_t n_pts, const double* X) {
  SFM_TRACE("sfm_ba_set_problem");
  if (!h) return fail(SFM_EINVAL, "handle is NULL");
  if (n_obs < 0 || n_cams < 0 || n_pts < 0) return fail(SFM_EINVAL, "negative size");
  if (n_obs > 0 && (!obs_uv || !cam_idx || !pt_idx)) return fail(SFM_EINVAL, "observation arrays are NULL");
  if (n_cams > 0 && (!K9 || !rot || !t)) return fail(SFM_EINVAL, "camera arrays are NULL");
  if (n_pts > 0 && !X) return fail(SFM_EINVAL, "point array is NULL");
  if (n_obs > int64_t(INT32_MAX) - 64 * int64_t(n_cams))
    return fail(SFM_EINVAL, "more than 2^31-1 observations per shard");
  HostTimer timer;
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->stream));
  free_problem(h);
  DevProblem& d = h->d;
  timer.mark("sync + free");
  const int64_t N = n_obs;
  const int C = n_cams, P = n_pts;
  d.C = C; d.P = P; d.N = N;
  hipStream_t s = h->stream;
  int rc = 0;
  // large problems: uv goes up from a worker thread (below); it is joined
  // before any return (the copy writes a buffer of this call and reads the
  // caller's array)
  std::atomic<int> uv_state{0};     // 1: uv's copy and event are enqueued, 2: that failed
  std::atomic<int> param_state{0};  // the same for the parameters' copies (by that worker)
  struct Joiner {
    std::thread t;
    void join() {
      if (t.joinable()) t.join();
    }
    ~Joiner() { join(); }  // (declared after the states: joined before they go)
  } uv_worker;
  // Any failure returns through here: the buffers go back to the pool.
  auto bail = [&](int code) {
    uv_worker.join();
    free_problem(h);
    return code;
  };
// observations up to which set_problem checks and counts them on the host
constexpr int64_t kHostCheckMaxObs = 65536;
// and from which uv (16 B each) goes up from a worker thread beside the index
// layouts (4 MB: the thread's start-up is noise beside the copy)
constexpr int64_t kDeferredUvMinObs = 262144;
#define ALLOC(ptr, cnt) if ((rc = dalloc(h, &(ptr), (cnt)))) return bail(rc)
#define TMP(ptr, cnt) if ((rc = dalloc_tmp(h, &(ptr), (cnt)))) return bail(rc)
#define HCHK(expr)                                                                                \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess) return bail(fail(SFM_EIO, std::string(#expr) + ": " + hipGetErrorString(e_))); \
  } while (0)
  std::vector<int32_t> cam_cnt(size_t(C) + 4);
  // host-checked problems with few cameras: per camera, its observations per
  // point slice (the 8 XCD slices of k_small_chunks' key p * 8 / P) -- the
  // chunk table's slice sizes follow from them on the host -- and the pair
  // total's estimate (no same-camera duplicates): the small path then needs no
  // round trip before the pair lists
  std::vector<int32_t> cam_slice;
  int64_t pairs_est = 0;
  uint8_t* stg = nullptr;
  double* in_uv = nullptr;
  int32_t *in_cam = nullptr, *in_pt = nullptr, *cnt_p = nullptr;
  // ---- the caller's observation arrays go up as they are (packed into the
  // pinned stage: one DMA); the O(N) layout work runs on the device
  // (ba_setup.hip) ----
  // keyframe-sized problems: the checks and the camera / point counts on
  // the host, their point counts riding in the same upload -- no validation
  // launch and no round trip before the layout (C1: ~60 us of set_problem)
  const bool host_check = N <= kHostCheckMaxObs;
  StageLayout up;
  const size_t o_uv = up.add(sizeof(double) * 2 * size_t(N)), o_cam = up.add(sizeof(int32_t) * size_t(N)),
               o_pt = up.add(sizeof(int32_t) * size_t(N)),
               o_pc = host_check ? up.add(sizeof(int32_t) * (size_t(P) + 1)) : 0;
  const size_t in_bytes = up.bytes;
  const bool stage_in = in_bytes <= kStageMaxBytes;
  // large problems: uv uploaded beside the index layouts (SFM_SYNC_UV=1: in
  // line, as before round 6)
  const bool deferred_uv = !stage_in && N >= kDeferredUvMinObs && !env_flag("SFM_SYNC_UV");
  // (host checks: the camera-run blob below is staged AFTER the input blob,
  // which is still in flight -- no synchronisation in between -- so the
  // stage holds both from here: 2 C + chunks + ... ints, bounded)
  const size_t il_base = host_check && stage_in ? (in_bytes + 255) / 256 * 256 : 0;
  const size_t il_bound = host_check && stage_in ? hostlayout::runs_blob_bound(C, N, P) : 0;
  // intrinsics, the parameters and their reset copies: one blob, one DMA
  StageLayout pl;
  const size_t o_K = pl.add(sizeof(double) * 5 * size_t(C)), o_c = pl.add(sizeof(double) * 6 * size_t(C)),
               o_c0 = pl.add(sizeof(double) * 6 * size_t(C)), o_X = pl.add(sizeof(double) * 3 * size_t(P)),
               o_X0 = pl.add(sizeof(double) * 3 * size_t(P));
  // host-checked problems stage it behind the camera-run blob and upload it
  // before the layout round trip (its host copies overlap the layout kernels)
  const size_t pl_base = (il_base + il_bound + 255) / 256 * 256;
  const bool early_params = il_base > 0 && (C || P) && pl_base + pl.bytes <= 4 * kStageMaxBytes;
  if ((rc = stage_reserve(h, std::max({stage_in ? il_base + il_bound : 0, early_params ? pl_base + pl.bytes : 0,
                                        sizeof(int32_t) * (size_t(C) + 4)}))))
    return bail(rc);
  stg = h->stage;
  uint8_t* in_blob = nullptr;
  TMP(in_blob, in_bytes);
  in_uv = reinterpret_cast<double*>(in_blob + o_uv);
  in_cam = reinterpret_cast<int32_t*>(in_blob + o_cam);
  in_pt = reinterpret_cast<int32_t*>(in_blob + o_pt);
  std::vector<double> Kc(5 * size_t(C)), cam(6 * size_t(C));
  for (int c = 0; c < C; ++c) {
    const double* k = K9 + 9 * size_t(c);
    Kc[5 * c] = k[0]; Kc[5 * c + 1] = k[1]; Kc[5 * c + 2] = k[2]; Kc[5 * c + 3] = k[4]; Kc[5 * c + 4] = k[5];
    for (int j = 0; j < 3; ++j) { cam[6 * c + j] = rot[3 * c + j]; cam[6 * c + 3 + j] = t[3 * c + j]; }
  }
  // large problems: the parameters (above the stage's 1 MB) go up from the
  // caller's pageable arrays on a stream of their own while the layout
  // kernels run (with a deferred uv, from its worker, before uv) (the host's staging copies took ~0.5 ms at C3 after the
  // layout round trip, with the device idle); the solve stream waits for them
  // at the end of set_problem
  const bool side_params = !early_params && (C || P) && pl.bytes > kStageMaxBytes;
  if (side_params) {
    uint8_t* pb = nullptr;
    ALLOC(pb, pl.bytes);
    d.Kc = reinterpret_cast<double*>(pb + o_K);
    d.cam = reinterpret_cast<double*>(pb + o_c);
    d.cam0 = reinterpret_cast<double*>(pb + o_c0);
    d.X = reinterpret_cast<double*>(pb + o_X);
    d.X0 = reinterpret_cast<double*>(pb + o_X0);
    if (!h->ustream) {
      HCHK(hipStreamCreateWithFlags(&h->ustream, hipStreamNonBlocking));
      HCHK(hipEventCreateWithFlags(&h->uev, hipEventDisableTiming));
    }
  }
  auto params_copies = [&]() -> bool {
    hipStream_t u = h->ustream;
    return hipMemcpyAsync(d.Kc, Kc.data(), sizeof(double) * Kc.size(), hipMemcpyHostToDevice, u) == hipSuccess &&
           hipMemcpyAsync(d.cam, cam.data(), sizeof(double) * cam.size(), hipMemcpyHostToDevice, u) == hipSuccess &&
           hipMemcpyAsync(d.cam0, d.cam, sizeof(double) * cam.size(), hipMemcpyDeviceToDevice, u) == hipSuccess &&
           (!P || (hipMemcpyAsync(d.X, X, sizeof(double) * 3 * size_t(P), hipMemcpyHostToDevice, u) == hipSuccess &&
                   hipMemcpyAsync(d.X0, d.X, sizeof(double) * 3 * size_t(P), hipMemcpyDeviceToDevice, u) ==
                       hipSuccess)) &&
           hipEventRecord(h->uev, u) == hipSuccess;
  };
  auto upload_params_side = [&]() -> int { return params_copies() ? 0 : fail(SFM_EIO, "parameter upload failed"); };
  int32_t* err = nullptr;
  int32_t* cnt_c = nullptr;
  if (host_check && stage_in) {
    // k_validate's checks and counts on the host (ba_host_layout.h)
    hostlayout::check_and_count(N, obs_uv, cam_idx, pt_idx, C, P, C <= kSmallSetupMaxC, cam_cnt.data(),
                                reinterpret_cast<int32_t*>(stg + o_pc), &cam_slice, &pairs_est);
    cnt_p = reinterpret_cast<int32_t*>(in_blob + o_pc);
    timer.mark("host checks + counts");
  } else {
    TMP(err, 4 + size_t(C) + 1);  // first bad observation (4) | per-camera counts (C + 1)
    cnt_c = err + 4;
    TMP(cnt_p, size_t(P) + 1);
  }
  // (host checks: the point counts ride in this upload, so it goes up even
  // without observations -- the zero counts then reach cnt_p)
  if ((N || host_check) && stage_in) {
    if (N) {
      std::memcpy(stg + o_uv, obs_uv, sizeof(double) * 2 * size_t(N));
      std::memcpy(stg + o_cam, cam_idx, sizeof(int32_t) * size_t(N));
      std::memcpy(stg + o_pt, pt_idx, sizeof(int32_t) * size_t(N));
    }
    HCHK(hipMemcpyAsync(in_blob, stg, in_bytes, hipMemcpyHostToDevice, s));
    timer.mark("stage copy + upload");
  } else if (N) {
    HCHK(hipMemcpyAsync(in_cam, cam_idx, sizeof(int32_t) * size_t(N), hipMemcpyHostToDevice, s));
    HCHK(hipMemcpyAsync(in_pt, pt_idx, sizeof(int32_t) * size_t(N), hipMemcpyHostToDevice, s));
    if (deferred_uv) {
      // the indices are up; uv (two thirds of the bytes) goes up from a
      // worker thread on the side stream -- a pageable copy holds its thread
      // until the data has left the caller's array -- while this thread lays
      // out the indices; k_uv_layout takes it once it has landed
      if (!h->ustream) {
        HCHK(hipStreamCreateWithFlags(&h->ustream, hipStreamNonBlocking));
        HCHK(hipEventCreateWithFlags(&h->uev, hipEventDisableTiming));
      }
      if (!h->uev_uv) HCHK(hipEventCreateWithFlags(&h->uev_uv, hipEventDisableTiming));
      const int dev = h->device;
      hipStream_t u = h->ustream;
      hipEvent_t ue = h->uev_uv;
      // (the parameters first: 5 MB the solve needs only at its start, off
      // the copy engine before uv's layouts wait on it)
      auto uv_job = [dev, u, ue, in_uv, obs_uv, N, side_params, &params_copies, &uv_state, &param_state]() {
        bool ok = hipSetDevice(dev) == hipSuccess;
        if (side_params) param_state.store(ok && params_copies() ? 1 : 2, std::memory_order_release);
        ok = ok && hipMemcpyAsync(in_uv, obs_uv, sizeof(double) * 2 * size_t(N), hipMemcpyHostToDevice, u) ==
                       hipSuccess &&
             hipEventRecord(ue, u) == hipSuccess;
        uv_state.store(ok ? 1 : 2, std::memory_order_release);
      };
      // (no exception crosses the C ABI: without a thread the copies run here)
      try {
        uv_worker.t = std::thread(uv_job);
      } catch (...) {
        uv_job();
      }
    } else {
      HCHK(hipMemcpyAsync(in_uv, obs_uv, sizeof(double) * 2 * size_t(N), hipMemcpyHostToDevice, s));
    }
  }
  // the solve stream takes uv once the worker has enqueued its copy
  auto wait_uv = [&]() -> int {
    uv_worker.join();
    if (uv_state.load(std::memory_order_acquire) != 1) return fail(SFM_EIO, "observation upload failed");
    if (hipStreamWaitEvent(s, h->uev_uv, 0) != hipSuccess) return fail(SFM_EIO, "observation upload wait failed");
    return 0;
  };
  if (!(host_check && stage_in)) {
    {
      Fill32Set fs;
      fs.add(err, 4 * sizeof(int32_t), uint32_t(INT32_MAX));
      fs.add(cnt_c, sizeof(int32_t) * (size_t(C) + 1), 0);
      fs.add(cnt_p, sizeof(int32_t) * (size_t(P) + 1), 0);
      launch_fill32(fs, s);
    }
    // (deferred uv: no point counts either -- pt_off comes from the sorted keys)
    launch_validate(N, deferred_uv ? nullptr : in_uv, in_cam, in_pt, C, P, err, cnt_c, deferred_uv ? nullptr : cnt_p, s);
    // one round trip: the first bad observation and the per-camera counts
    // (the host lays out the C camera runs and the wavefront chunk table);
    // the readback lands in the stage after the upload has read it (stream order)
    HCHK(hipMemcpyAsync(stg, err, sizeof(int32_t) * (size_t(C) + 4), hipMemcpyDeviceToHost, s));
    HCHK(hipStreamSynchronize(s));
    std::memcpy(cam_cnt.data(), stg, sizeof(int32_t) * (size_t(C) + 4));
    if (deferred_uv && std::min(cam_cnt[0], cam_cnt[1]) != INT32_MAX) {
      // a bad index: the whole check once uv is up, so the error reported is
      // the first bad observation of any kind, as without the deferral
      if ((rc = wait_uv())) return bail(rc);
      launch_validate(N, in_uv, in_cam, in_pt, C, P, err, cnt_c, cnt_p, s);
      HCHK(hipMemcpyAsync(stg, err, sizeof(int32_t) * 4, hipMemcpyDeviceToHost, s));
      HCHK(hipStreamSynchronize(s));
      std::memcpy(cam_cnt.data(), stg, sizeof(int32_t) * 4);
    }
  }
  timer.mark("upload + validate");
  {
    const int32_t e0 = cam_cnt[0], e1 = cam_cnt[1], e2 = cam_cnt[2];
    const int32_t first = std::min({e0, e1, e2});
    if (first != INT32_MAX) {
      const char* what = first == e0 ? "cam_idx out of range at " : first == e1 ? "pt_idx out of range at "
                                                                                   : "non-finite observation at ";
      return bail(fail(SFM_EINVAL, what + std::to_string(first)));
    }
  }
  // ---- camera runs: camera-major, each camera's run padded to a whole
  // number of 64-wide wavefront chunks; the chunk table camera-major
  // (grouped into 8 point slices on the device, one per XCD) ----
  hostlayout::Runs runs;
  hostlayout::camera_runs(C, cam_cnt.data() + 4, &runs);
  const std::vector<int32_t>&cam_off = runs.cam_off, &cam_rng = runs.cam_rng, &wcam = runs.wcam;
  const std::vector<hostlayout::Chunk>& chunks = runs.chunks;
  const int64_t npad = runs.npad;
  d.N_pad = npad;
  d.n_jchunks = int32_t(chunks.size());
  d.jac_blocks_rec = 8 * std::max(1, std::min((d.n_jchunks / 8 + 3) / 4, 128));  // multiple of 8 (one slice per XCD)
  // the record-free pass of the solve (no 160-B stores) prefers a larger
  // grid: 256 workgroups per XCD, 0.256 -> 0.223 ms per C3 solve
  d.jac_blocks = 8 * std::max(1, std::min((d.n_jchunks / 8 + 3) / 4, 256));
  if (const char* jw = std::getenv("SFM_JAC_WG_PER_XCD")) {  // tuning knob (tools/sweep_jac.sh)
    const int v = std::atoi(jw);
    if (v > 0) d.jac_blocks = 8 * std::max(1, std::min((d.n_jchunks / 8 + 3) / 4, v));
  }
  // keyframe-sized problems: the layouts without radix sorts (ba_setup.hip
  // small path; the same arrays bit for bit), when the host has the counts
  // and the segments fit its bounds (SFM_SMALL_SETUP=0: the sorted path)
  // (C (C + 1) / 2 <= kSchurXcdMinBlocks: the plain k_schur_pts block order,
  // as the sorted path takes for these sizes)
  bool small = host_check && stage_in && N > 0 && N <= kSmallSetupMaxObs && C > 0 && C <= kSmallSetupMaxC &&
               int64_t(C) * (C + 1) / 2 <= kSchurXcdMinBlocks;
  if (small) {
    const char* ss = std::getenv("SFM_SMALL_SETUP");
    if (ss && ss[0] == '0') small = false;
  }
  if (small) {
    int64_t nch_small = 0;
    for (int c = 0; c < C; ++c) nch_small += (cam_cnt[4 + c] + 63) / 64;
    small = nch_small <= kSmallSetupMaxChunks;
  }
  if (small) {
    const int32_t* pc = reinterpret_cast<const int32_t*>(stg + o_pc);
    for (int p = 0; p < P && small; ++p) small = pc[p] <= kSmallSetupMaxPtObs;
  }
  timer.mark("camera runs (host)");
  // ---- resident arrays of the point-major and camera-major layouts ----
  int64_t n_pairs = 0;
  int32_t *pt_s = nullptr, *cm_order = nullptr;
  const int32_t* pair_order = nullptr;  // the Schur pair lists' emission order (nullptr: point-major)
  int64_t* poff = nullptr;
  void* sort_tmp = nullptr;
  size_t sort_bytes = 0;
  int32_t* small_fill = nullptr;  // small path: the scatters' slot counters (P | C), zeroed in the camera-run blob
  if (!small) ALLOC(d.pt_off, size_t(P) + 1);  // (small path: in the camera-run blob)
  ALLOC(d.order, size_t(N));
  ALLOC(d.uv_pm, 2 * size_t(N));
  ALLOC(d.cam_pm, size_t(N));
  ALLOC(d.cam_obs, size_t(npad));
  ALLOC(d.cm_p, size_t(npad));
  ALLOC(d.jchunks, size_t(std::max(1, d.n_jchunks)));
  ALLOC(d.jgrp, size_t(9));
  ALLOC(d.uv_cm, 2 * size_t(npad));
  ALLOC(d.pos, size_t(N));
  // scratch of the sorts
  uint64_t *k64a = nullptr, *k64b = nullptr;
  uint32_t *k32a = nullptr, *k32b = nullptr;
  int32_t *iota = nullptr, *d_cam_off = nullptr, *perm = nullptr;
  int4* ch_in = nullptr;
  const int64_t nch = d.n_jchunks;
  const int64_t nmax = std::max<int64_t>({N, nch, 1});
  TMP(k64a, size_t(N));
  TMP(k64b, size_t(N));
  TMP(k32a, size_t(nmax));
  TMP(k32b, size_t(nmax));
  TMP(iota, size_t(nmax));
  TMP(pt_s, size_t(N));
  TMP(cm_order, size_t(N));
  TMP(perm, size_t(std::max<int64_t>(1, nch)));
  sort_bytes = std::max({setup_sort_bytes(N, 64), setup_sort_bytes(nmax, 32), setup_sort_bytes(P + 1, 1),
                                setup_sort_bytes(N + 1, 2), size_t(256)});
  {
    uint8_t* tb = nullptr;
    TMP(tb, sort_bytes);
    sort_tmp = tb;
  }
  {
    // the host-made camera runs and chunk table in one resident blob, one
    // DMA from the stage (the validation readback was consumed above):
    // cam_rng | wcam (resident), cam_off | chunks (read by the setup only)
    StageLayout il;
    const size_t o_rng = il.add(sizeof(int32_t) * cam_rng.size()), o_w = il.add(sizeof(int32_t) * wcam.size()),
                 o_off = il.add(sizeof(int32_t) * cam_off.size()), o_ch = il.add(sizeof(hostlayout::Chunk) * chunks.size());
    // small path: pt_off (the host's scan of the point counts, resident) and
    // the zeroed slot counters of the point / camera scatters
    const size_t o_poff = small ? il.add(sizeof(int32_t) * (size_t(P) + 1)) : 0,
                 o_fill = small ? il.add(sizeof(int32_t) * (size_t(P) + size_t(C))) : 0;
    if (il_base && il.bytes > il_bound) return bail(fail(SFM_EIO, "internal: camera-run blob above its bound"));
    if ((rc = stage_reserve(h, il_base + il.bytes))) return bail(rc);  // (never regrows with il_base > 0)
    if (early_params && il_base + il.bytes > pl_base) return bail(fail(SFM_EIO, "internal: stage layout overlap"));
    stg = h->stage;
    uint8_t* ib = nullptr;
    ALLOC(ib, il.bytes);
    uint8_t* sb = stg + il_base;
    std::memcpy(sb + o_rng, cam_rng.data(), sizeof(int32_t) * cam_rng.size());
    std::memcpy(sb + o_w, wcam.data(), sizeof(int32_t) * wcam.size());
    std::memcpy(sb + o_off, cam_off.data(), sizeof(int32_t) * cam_off.size());
    if (nch) std::memcpy(sb + o_ch, chunks.data(), sizeof(hostlayout::Chunk) * chunks.size());
    if (small) {
      const int32_t* pc = reinterpret_cast<const int32_t*>(stg + o_pc);
      int32_t* po = reinterpret_cast<int32_t*>(sb + o_poff);
      po[0] = 0;
      for (int p = 0; p < P; ++p) po[p + 1] = po[p] + pc[p];
      std::memset(sb + o_fill, 0, sizeof(int32_t) * (size_t(P) + size_t(C)));
    }
    if (deferred_uv) {
      // uv's 32-MB DMA is on the copy engine now: this blob, on it, would
      // wait behind it and hold up the layouts, so a kernel reads it from
      // the pinned stage instead (il.bytes: 256-B aligned pieces)
      void* sbd = nullptr;
      HCHK(hipHostGetDevicePointer(&sbd, sb, 0));
      launch_copy_from_host(ib, sbd, (il.bytes + 15) / 16 * 16, s);
    } else {
      HCHK(hipMemcpyAsync(ib, sb, il.bytes, hipMemcpyHostToDevice, s));
    }
    if (small) {
      d.pt_off = reinterpret_cast<int32_t*>(ib + o_poff);
      small_fill = reinterpret_cast<int32_t*>(ib + o_fill);
    }
    d.cam_rng = reinterpret_cast<int32_t*>(ib + o_rng);
    d.wcam = reinterpret_cast<int32_t*>(ib + o_w);
    d_cam_off = reinterpret_cast<int32_t*>(ib + o_off);
    ch_in = reinterpret_cast<int4*>(ib + o_ch);
  }
  if (early_params) {
    uint8_t* pb = nullptr;
    ALLOC(pb, pl.bytes);
    d.Kc = reinterpret_cast<double*>(pb + o_K);
    d.cam = reinterpret_cast<double*>(pb + o_c);
    d.cam0 = reinterpret_cast<double*>(pb + o_c0);
    d.X = reinterpret_cast<double*>(pb + o_X);
    d.X0 = reinterpret_cast<double*>(pb + o_X0);
    uint8_t* ps = stg + pl_base;
    std::memcpy(ps + o_K, Kc.data(), sizeof(double) * Kc.size());
    std::memcpy(ps + o_c, cam.data(), sizeof(double) * cam.size());
    std::memcpy(ps + o_c0, cam.data(), sizeof(double) * cam.size());
    if (P) {
      std::memcpy(ps + o_X, X, sizeof(double) * 3 * size_t(P));
      std::memcpy(ps + o_X0, X, sizeof(double) * 3 * size_t(P));
    }
    HCHK(hipMemcpyAsync(pb, ps, pl.bytes, hipMemcpyHostToDevice, s));
  }
  int32_t* small_cnt = nullptr;  // small path: per-block pair counts
  if (small) {
    // the same layouts without radix sorts (ba_setup.hip small path):
    // point-major by (point, camera, caller index), camera-major by (camera,
    // point-major id), the chunk table by slice, the pair counts per block
    // (seg = their exclusive sum, seg[n_blk] = the pair total)
    d.n_blk = int64_t(C) * (C + 1) / 2;
    ALLOC(d.seg, size_t(d.n_blk) + 1);
    TMP(small_cnt, std::max<size_t>(1, size_t(d.n_blk)));
    timer.mark("allocs + camera-run blob");
    launch_small_pm(N, in_pt, in_cam, in_uv, d.pt_off, small_fill, reinterpret_cast<int32_t*>(k32a), d.order,
                    d.uv_pm, d.cam_pm, pt_s, s);
    launch_small_cm(N, C, d.cam_pm, d_cam_off, cm_order, s);
    launch_fill_cm(npad, d.wcam, d.cam_rng, d_cam_off, cm_order, pt_s, d.uv_pm, d.cm_p, d.uv_cm, d.cam_obs, d.pos, s);
    launch_small_chunks(int(nch), ch_in, cm_order, pt_s, P, d.jchunks, d.jgrp, s);
    launch_small_pairs_count(C, d.n_blk, d_cam_off, cm_order, d.cam_pm, pt_s, d.pt_off, small_cnt, d.seg, s);
    // (into the stage: stream order puts it after the upload that reads the stage)
  } else {
  timer.mark("allocs + camera-run blob");
  // point-major order: stable sort by (point, camera)
  launch_pm_keys(N, in_cam, in_pt, C, k64a, iota, s);
  HCHK(sort_pairs64(sort_tmp, sort_bytes, k64a, k64b, iota, d.order, N,
                    uint64_t(std::max(1, P)) * uint64_t(std::max(1, C)) - 1, s));
  launch_gather_pm(N, d.order, deferred_uv ? nullptr : in_uv, in_cam, in_pt, d.uv_pm, d.cam_pm, pt_s, k32a, iota, s);
  if (deferred_uv) launch_pt_off(P, k64b, N, C, d.pt_off, s);
  else HCHK(exclusive_sum32(sort_tmp, sort_bytes, cnt_p, d.pt_off, int64_t(P) + 1, s));
  // camera-major order of the point-major ids: stable sort by camera
  HCHK(sort_pairs32(sort_tmp, sort_bytes, k32a, k32b, iota, cm_order, N, uint64_t(std::max(1, C)) - 1, s));
  launch_fill_cm(npad, d.wcam, d.cam_rng, d_cam_off, cm_order, pt_s, deferred_uv ? nullptr : d.uv_pm, d.cm_p,
                 d.uv_cm, d.cam_obs, d.pos, s);
  // chunk table grouped by point slice (stable: camera-major order kept)
  launch_chunk_keys(int(nch), ch_in, cm_order, pt_s, P, k32a, iota, s);
  HCHK(sort_pairs32(sort_tmp, sort_bytes, k32a, k32b, iota, perm, nch, 7, s));
  launch_chunk_gather(int(nch), perm, ch_in, k32b, d.jchunks, d.jgrp, s);
  // Schur pair counts: the second (and last) round trip
  int64_t* pcnt = nullptr;
  TMP(pcnt, size_t(N) + 1);
  TMP(poff, size_t(N) + 1);
  // (point-major emission: the same lists; SFM_PAIRS_CM=1 emits in camera-major order)
  pair_order = env_flag("SFM_PAIRS_CM") ? cm_order : nullptr;
  launch_pair_count(N, pair_order, d.cam_pm, pt_s, d.pt_off, pcnt, s);
  HCHK(exclusive_sum64(sort_tmp, sort_bytes, pcnt, poff, N + 1, s));
  // (into the stage: stream order puts it after the upload that reads the stage)
  if (!deferred_uv) HCHK(hipMemcpyAsync(stg, poff + N, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  }
  if (small) {
    // no round trip: the pair lists go into a buffer of the pair total's
    // bound (every ordered pair of a point's observations: twice the
    // estimate), the chunk table's slice sizes come from the host's
    // per-camera slice counts (a camera's chunk k starts at its 64 k-th
    // observation in point order, whose slice the counts' running sum gives)
    n_pairs = std::max<int64_t>(1, 2 * pairs_est);
    d.xcd_slice_max = hostlayout::small_slice_max(C, cam_cnt.data() + 4, cam_slice);
    timer.mark("layout launches");
  } else {
    // and the 8 slices' chunk offsets: the observation passes size their
    // grids by the largest slice (obs_xcd_blocks)
    if (!deferred_uv) HCHK(hipMemcpyAsync(stg + 8, d.jgrp, 9 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    timer.mark("layout launches");
    if (deferred_uv) {
      // the pair total and the slice offsets read back by a kernel into the
      // pinned stage: uv's DMA holds the copy engine (uv itself is taken
      // after the pair lists are enqueued, which do not read it)
      void* stg_d = nullptr;
      HCHK(hipHostGetDevicePointer(&stg_d, stg, 0));
      uint8_t* sd = static_cast<uint8_t*>(stg_d);
      HostCopySet cs;
      cs.add(sd, poff + N, sizeof(int64_t));
      cs.add(sd + 8, d.jgrp, 9 * sizeof(int32_t));
      launch_copy_to_host(cs, s);
    }
    if (side_params && !deferred_uv) {
      if ((rc = upload_params_side())) return bail(rc);
      timer.mark("parameter upload (side stream)");
    }
    HCHK(hipStreamSynchronize(s));
    std::memcpy(&n_pairs, stg, sizeof(int64_t));
    int32_t g[9];
    std::memcpy(g, stg + 8, sizeof(g));
    d.xcd_slice_max = 0;
    for (int i = 0; i < 8; ++i) d.xcd_slice_max = std::max(d.xcd_slice_max, g[i + 1] - g[i]);
    timer.mark("layouts (device)");
  }
  if (n_pairs >= int64_t(INT32_MAX)) return bail(fail(SFM_EINVAL, "too many Schur pairs for 32-bit offsets"));
  d.n_blk = int64_t(C) * (C + 1) / 2;
  // the Schur pass's shape below follows the mean pair count: the host's
  // estimate on host-checked problems (either layout path, so both choose
  // alike), else the device's count.  The estimate counts every unordered
  // pair of a point's observations, so it undercounts when a camera sees a
  // point twice (a same-camera pair is an ordered pair of the diagonal
  // block); it picks the lanes per block only -- the pair buffer is sized by
  // twice the estimate, an upper bound of the true count either way.
  d.n_pairs = host_check && stage_in && !cam_slice.empty() ? pairs_est : n_pairs;
  // lanes per Schur block ~ a tenth of the mean pair count, 8..64 (measured
  // best: C3, 72 pairs per block -> 8; C1 / C2, ~460 -> 64)
  if (const char* ss = std::getenv("SFM_SCHUR_PTS_SUB")) {
    const int v = std::atoi(ss);
    d.schur_pts_sub = v == 64 ? 64 : v == 32 ? 32 : v == 8 ? 8 : 16;
  } else {
    const double avg = d.n_blk ? double(d.n_pairs) / double(d.n_blk) : 0.0;
    int sub = 8;
    while (sub < 64 && sub < avg / 10.0) sub *= 2;
    d.schur_pts_sub = sub;
  }
  // few blocks with long lists (keyframe-sized: C1 210 blocks of ~460
  // pairs): a workgroup per block instead of a wave (SFM_SCHUR_WG=0/1 forces)
  d.schur_wg_blocks = d.schur_pts_sub == 64 && d.n_blk <= 4 * 256 &&
                      (d.n_blk ? double(d.n_pairs) / double(d.n_blk) : 0.0) >= 256.0;
  if (const char* sw = std::getenv("SFM_SCHUR_WG")) d.schur_wg_blocks = sw[0] == '1' && d.schur_pts_sub == 64;
  if (!d.scal_host && hipHostMalloc(&d.scal_host, sizeof(double) * (kNumScalars + 1 + 17)) != hipSuccess) {
    d.scal_host = nullptr;
    return bail(fail(SFM_ENOMEM, "hipHostMalloc failed"));
  }
  // the pinned mirror's 17-slot tail: the k_schur_pts group sizes (16), then
  // the deferred uv's finite check (slot 16)
  int64_t* grp_host = reinterpret_cast<int64_t*>(d.scal_host + kNumScalars + 1);
  int32_t* uv_err_host = reinterpret_cast<int32_t*>(grp_host + 16);
  int bperm_per = 0;
  ALLOC(d.blk, std::max<size_t>(1, size_t(d.n_blk)));
  if (!small) ALLOC(d.seg, size_t(d.n_blk) + 1);
  ALLOC(d.bpts, std::max<size_t>(1, size_t(n_pairs)));
  if (small) {
    launch_small_pairs_fill(C, d.n_blk, d_cam_off, cm_order, d.cam_pm, pt_s, d.pt_off, d.seg, d.bpts, s);
    launch_blk(C, d.blk, s);
    d.bperm = nullptr;
    d.n_bslots = d.n_blk;
  } else {
    uint32_t *bk_a = nullptr, *bk_b = nullptr;
    int32_t* bv = nullptr;
    const int64_t nk = std::max<int64_t>({n_pairs, d.n_blk, 1});
    TMP(bk_a, size_t(nk));
    TMP(bk_b, size_t(nk));
    TMP(bv, size_t(nk));
    const size_t need = std::max(setup_sort_bytes(n_pairs, 32), setup_sort_bytes(d.n_blk, 32));
    if (need > sort_bytes) {
      uint8_t* tb = nullptr;
      TMP(tb, need);
      sort_tmp = tb;
      sort_bytes = need;
    }
    launch_pair_fill(N, pair_order, d.cam_pm, pt_s, d.pt_off, poff, C, bk_a, bv, s);
    HCHK(sort_pairs32(sort_tmp, sort_bytes, bk_a, bk_b, bv, d.bpts, n_pairs, uint64_t(std::max<int64_t>(1, d.n_blk)) - 1,
                      s));
    launch_seg(d.n_blk, bk_b, n_pairs, d.seg, s);
    launch_blk(C, d.blk, s);
    // ---- k_schur_pts work order: XCD-aware (ba_setup.hip k_bperm_*).
    // Block (c1, c2)'s pairs gather records of points camera c1 sees, so a
    // row c1 (its blocks c2 >= c1) reads one camera's ~N/C point records
    // (C3: ~0.5 MB).  Rows go to 8 groups of contiguous rows with equal pair
    // totals; group x's blocks, row by row (descending pair count within a
    // row, so a wave's blocks run lists of nearly equal length), fill
    // workgroups x, x + 8, x + 16, ... -- the ones dealt to one XCD
    // (round-robin placement: a speed assumption only, MI355X_MICROARCH.md),
    // so a row's records stay in that XCD's L2 while its blocks run.  Slots
    // past a group's end hold -1 (an empty list).  Small reduced systems
    // (keyframe-sized solves: everything fits one L2) keep the plain block
    // order (bperm = nullptr).  The group sizes come back with the final
    // synchronisation of set_problem.
    d.bperm = nullptr;
    d.n_bslots = d.n_blk;
    if (d.n_blk > kSchurXcdMinBlocks) {
      const int per = 64 / d.schur_pts_sub * (kThreads / 64);
      int32_t *sorted = nullptr, *row_x = nullptr;
      int64_t* grp = nullptr;
      TMP(sorted, size_t(d.n_blk));
      TMP(row_x, size_t(C));
      TMP(grp, 16);
      ALLOC(d.bperm, size_t(bperm_slots_bound(d.n_blk, per)));
      HCHK(launch_bperm(C, d.n_blk, n_pairs, d.seg, d.blk, per, bk_a, bk_b, bv, sorted, row_x, grp, sort_tmp,
                        sort_bytes, d.bperm, s));
      HCHK(hipMemcpyAsync(grp_host, grp, sizeof(int64_t) * 16, hipMemcpyDeviceToHost, s));
      bperm_per = per;
    }
  }
  // ---- parameters, per-iteration arrays, dense system ----
  d.n = 6 * C;
  d.ld = ((d.n + 1 + kNB - 1) / kNB) * kNB;
  d.nblk = d.ld / kNB;
  d.max_blocks = std::max({1, C, blocks_for(N, 256), blocks_for(P, 256), d.jac_blocks,
                           d.jac_blocks_rec, blocks_for(npad, 256), obs_xcd_blocks(d), pt_xcd_blocks(d)});
  if (!early_params && !side_params) {
    uint8_t* pb = nullptr;
    ALLOC(pb, pl.bytes);
    d.Kc = reinterpret_cast<double*>(pb + o_K);
    d.cam = reinterpret_cast<double*>(pb + o_c);
    d.cam0 = reinterpret_cast<double*>(pb + o_c0);
    d.X = reinterpret_cast<double*>(pb + o_X);
    d.X0 = reinterpret_cast<double*>(pb + o_X0);
  }
  ALLOC(d.cam_new, 6 * size_t(C));
  ALLOC(d.X_new, 3 * size_t(P));
  ALLOC(d.scale_c, 6 * size_t(C));
  ALLOC(d.scale_p, 3 * size_t(P));
  ALLOC(d.diag_c, 6 * size_t(C));
  ALLOC(d.diag_p, 3 * size_t(P));
  ALLOC(d.camR, size_t(kCamR) * C);
  ALLOC(d.camRn, 12 * size_t(C));
  // pass A stores u at the camera-major position it runs at (coalesced) and
  // pass B gathers it through pos[]: 85 + 31 -> 60 + 41 us per C3 iteration
  // against the point-major scatter (SFM_EU_CM=0), S and steps bitwise equal
  {
    const char* ec = std::getenv("SFM_EU_CM");
    d.eu_cm = !(ec && ec[0] == '0');
  }
  ALLOC(d.eu, size_t(kEU) * size_t(d.eu_cm ? npad : N));
  ALLOC(d.ypt, 3 * size_t(P));
  ALLOC(d.ptV, size_t(kPtV) * P);
  ALLOC(d.ptL, size_t(kPtL) * P);
  ALLOC(d.ptS, size_t(kPtS) * std::max(1, P));
  ALLOC(d.Ucam, size_t(kUcam) * C);
  ALLOC(d.jpart, 27 * std::max<size_t>(1, size_t(npad / 64)));
  ALLOC(d.dpart, 27 * std::max<size_t>(1, size_t(npad / 64)));
  ALLOC(d.S, size_t(d.ld) * d.ld);
  h->force_pack = env_flag("SFM_FORCE_PACK");
  if (sharded(h) || h->force_pack) ALLOC(d.Spack, packed_size(d.n));
  ALLOC(d.invL, size_t(d.nblk) * kNB * kNB);
  ALLOC(d.flags, size_t(d.nblk));
  ALLOC(d.cflags, 2 * size_t(d.nblk) * d.nblk);
  ALLOC(d.cticket, 5);  // task ticket, walker-role ticket, back-substitution role ticket, a panel's two
  // Schur / Cholesky overlap (SFM_OVERLAP=1; unsharded, more than two tiles):
  // per 64x64 tile of S the number of camera blocks (c1 <= c2, stored at
  // rows 6 c2.., columns 6 c1..) whose 6x6 footprint touches it.  (The
  // round-4 mode 2, a full helper grid placed as the Schur pass retires,
  // relied on the dispatcher starting the Schur pass's workgroups first:
  // not guaranteed, and seen to time out the factor, so removed.)
  {
    const char* ov = std::getenv("SFM_OVERLAP");
    const int v = ov ? std::atoi(ov) : 0;
    d.overlap = v > 0 && d.nblk > 2 && !sharded(h) ? 1 : 0;
  }
  if (d.overlap) {
    ALLOC(d.tile_cnt, size_t(d.nblk) * d.nblk);
    ALLOC(d.tile_exp, size_t(d.nblk) * d.nblk);
    std::vector<int32_t> te(size_t(d.nblk) * d.nblk, 0);
    for (int c1 = 0; c1 < C; ++c1)
      for (int c2 = c1; c2 < C; ++c2)
        for (int I = 6 * c2 / kNB; I <= (6 * c2 + 5) / kNB; ++I)
          for (int J = 6 * c1 / kNB; J <= (6 * c1 + 5) / kNB; ++J) ++te[size_t(I) * d.nblk + J];
    HCHK(hipMemcpy(d.tile_exp, te.data(), sizeof(int32_t) * te.size(), hipMemcpyHostToDevice));
  }
  ALLOC(d.ysol, size_t(d.ld));
  ALLOC(d.fail, size_t(1));
  ALLOC(d.partials, size_t(kNumPartialSlots) * d.max_blocks);
  ALLOC(d.scal, size_t(kNumScalars) + 1);  // + the Cholesky failure int (k_reduce_batch)
#undef ALLOC
#undef TMP
  release_pool(h);  // earlier problems' buffers this one did not reuse
  if (deferred_uv) {
    // uv (and before it the parameters) by now up or nearly: its two
    // layouts and its finite check on the side stream, behind its copy and
    // beside the pair lists (the index layouts they read are complete: the
    // host synchronised on them), the check read back by a kernel with the
    // final synchronisation
    uv_worker.join();
    if (uv_state.load(std::memory_order_acquire) != 1) return bail(fail(SFM_EIO, "observation upload failed"));
    timer.mark("uv upload (worker)");
    hipStream_t u = h->ustream;
    launch_uv_layout(N, npad, d.order, d.wcam, d.cam_rng, d_cam_off, cm_order, in_uv, d.uv_pm, d.uv_cm, err, u);
    void* ue_d = nullptr;
    HCHK(hipHostGetDevicePointer(&ue_d, uv_err_host, 0));
    HostCopySet cs;
    cs.add(ue_d, err + 2, sizeof(int32_t));
    launch_copy_to_host(cs, u);
    HCHK(hipEventRecord(h->uev_uv, u));  // (the solve stream waits for it after its own fills, below)
  }
  if (side_params) {
    if (small && (rc = upload_params_side())) return bail(rc);  // (the small path has no layout round trip)
    // (deferred uv: its worker, joined above, enqueued them)
    if (deferred_uv && param_state.load(std::memory_order_acquire) != 1)
      return bail(fail(SFM_EIO, "parameter upload failed"));
    HCHK(hipStreamWaitEvent(s, h->uev, 0));
  } else if ((C || P) && !early_params) {
    if (pl.bytes <= kStageMaxBytes) {
      // the stage is free: the n_pairs readback synchronised the stream
      if ((rc = stage_reserve(h, pl.bytes))) return bail(rc);
      uint8_t* ps = h->stage;
      std::memcpy(ps + o_K, Kc.data(), sizeof(double) * Kc.size());
      std::memcpy(ps + o_c, cam.data(), sizeof(double) * cam.size());
      std::memcpy(ps + o_c0, cam.data(), sizeof(double) * cam.size());
      if (P) {
        std::memcpy(ps + o_X, X, sizeof(double) * 3 * size_t(P));
        std::memcpy(ps + o_X0, X, sizeof(double) * 3 * size_t(P));
      }
      HCHK(hipMemcpyAsync(d.Kc, ps, pl.bytes, hipMemcpyHostToDevice, s));
    } else {
      // (the host vectors live until the synchronisation below)
      HCHK(hipMemcpyAsync(d.Kc, Kc.data(), sizeof(double) * Kc.size(), hipMemcpyHostToDevice, s));
      HCHK(hipMemcpyAsync(d.cam, cam.data(), sizeof(double) * cam.size(), hipMemcpyHostToDevice, s));
      HCHK(hipMemcpyAsync(d.cam0, d.cam, sizeof(double) * cam.size(), hipMemcpyDeviceToDevice, s));
      if (P) {
        HCHK(hipMemcpyAsync(d.X, X, sizeof(double) * 3 * size_t(P), hipMemcpyHostToDevice, s));
        HCHK(hipMemcpyAsync(d.X0, d.X, sizeof(double) * 3 * size_t(P), hipMemcpyDeviceToDevice, s));
      }
    }
  }
  {
    // the walker stores only the lower 16x16 blocks of each W_k (k_chol_fused)
    Fill32Set fs;
    fs.add(d.S, sizeof(double) * size_t(d.ld) * d.ld, 0);
    fs.add(d.invL, sizeof(double) * size_t(d.nblk) * kNB * kNB, 0);
    fs.add(d.flags, sizeof(int32_t) * size_t(d.nblk), 0);
    fs.add(d.cflags, sizeof(int32_t) * 2 * size_t(d.nblk) * d.nblk, 0);
    fs.add(d.cticket, 5 * sizeof(unsigned long long), 0);
    fs.add(d.partials, sizeof(double) * size_t(kNumPartialSlots) * d.max_blocks, 0);
    launch_fill32(fs, s);
  }
  h->chol_epoch = 0;
  h->bs_epoch = 0;
  d.n_cu = h->n_cu;
  timer.mark("pairs + params launches");
  // Small problems end without a synchronisation: every host-to-device copy
  // came from the pinned stage, nothing is read back, so the pair lists and
  // uploads run on while the caller enqueues the solve (stream order covers
  // every reader; the scratch buffers stay out of the pool until the next
  // set_problem's free_problem, after its synchronisation, and the stage is
  // next written by a call that synchronises first).  Otherwise: the
  // k_schur_pts group sizes come back, copies from pageable host memory (the
  // caller's arrays, this call's vectors) complete, and the scratch buffers
  // return to the pool.
  // (SFM_SYNC_SETUP=1: always synchronise, so that a fault in a layout kernel
  // is reported by set_problem itself, not by the next call)
  static const bool sync_setup = env_flag("SFM_SYNC_SETUP");
  if (deferred_uv) HCHK(hipStreamWaitEvent(s, h->uev_uv, 0));
  if (!(small && early_params && !bperm_per) || sync_setup) {
    HCHK(hipStreamSynchronize(s));
    if (deferred_uv && *uv_err_host != INT32_MAX)
      return bail(fail(SFM_EINVAL, "non-finite observation at " + std::to_string(*uv_err_host)));
    if (bperm_per) {
      int64_t m_max = 1;
      for (int x = 0; x < 8; ++x) m_max = std::max<int64_t>(m_max, (grp_host[8 + x] + bperm_per - 1) / bperm_per);
      d.n_bslots = m_max * 8 * bperm_per;
    }
    retire_tmps(h);
    timer.mark("pair lists + uploads (device)");
  }
#undef HCHK
  h->has_problem = true;
  return 0;
}

int sfm_ba_reset_parameters(sfm_ba_handle* h) {
  if (!h || !h->has_problem) return fail(SFM_EINVAL, "no problem set");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipMemcpyAsync(h->d.cam, h->d.cam0, sizeof(double) * 6 * size_t(h->d.C), hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->d.X, h->d.X0, sizeof(double) * 3 * size_t(h->d.P), hipMemcpyDeviceToDevice, h->stream));
  return 0;
}

int sfm_ba_get_parameters(sfm_ba_handle* h, double* rot, double* t, double* X) {
  if (!h || !h->has_problem) return fail(SFM_EINVAL, "no problem set");
  HIPCHK(hipSetDevice(h->device));
  const DevProblem& d = h->d;
  // both arrays through the pinned stage (the stream is drained first: the
  // stage may be regrown, and nothing in flight may still use it)
  HIPCHK(hipStreamSynchronize(h->stream));
  StageLayout gl;
  const size_t o_c = gl.add(sizeof(double) * 6 * size_t(d.C)), o_X = gl.add(sizeof(double) * 3 * size_t(d.P));
  const bool stage_x = gl.bytes <= kStageMaxBytes;  // (else X straight into the caller's array)
  if (int rc = stage_reserve(h, stage_x ? gl.bytes : o_X)) return rc;
  const double* cam = reinterpret_cast<const double*>(h->stage + o_c);
  if (d.C) HIPCHK(hipMemcpyAsync(h->stage + o_c, d.cam, sizeof(double) * 6 * size_t(d.C), hipMemcpyDeviceToHost, h->stream));
  if (X && d.P)
    HIPCHK(hipMemcpyAsync(stage_x ? static_cast<void*>(h->stage + o_X) : static_cast<void*>(X), d.X,
                          sizeof(double) * 3 * size_t(d.P), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (X && d.P && stage_x) std::memcpy(X, h->stage + o_X, sizeof(double) * 3 * size_t(d.P));
  for (int c = 0; c < d.C; ++c)
    for (int j = 0; j < 3; ++j) {
      if (rot) rot[3 * c + j] = cam[6 * c + j];
      if (t) t[3 * c + j] = cam[6 * c + 3 + j];
    }
  return 0;
}

int sfm_ba_set_profiling(sfm_ba_handle* h, int32_t on) {
  if (!h) return fail(SFM_EINVAL, "handle is NULL");
  h->profiling = on != 0;
  for (int i = 0; i < kNumPh; ++i) { h->phase_ms[i] = 0; h->phase_count[i] = 0; }
  return 0;
}

int sfm_ba_phase_times(sfm_ba_handle* h, double* ms) {
  if (!h || !ms) return fail(SFM_EINVAL, "bad arguments");
  for (int i = 0; i < kNumPh; ++i) ms[i] = h->phase_ms[i];
  for (int i = 0; i < kNumPh; ++i) ms[kNumPh + i] = h->phase_count[i];
  return 0;
}

int sfm_ba_sync(sfm_ba_handle* h) {
  if (!h) return fail(SFM_EINVAL, "handle is NULL");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

int sfm_ba_solve_resident(sfm_ba_handle* h, const sfm_ba_options* opts_in, int32_t mode, sfm_ba_summary* summary,
                          sfm_ba_iteration* trace, int32_t trace_cap, int32_t* trace_len) {
  SFM_TRACE("sfm_ba_solve_resident");
  const auto t_start = std::chrono::steady_clock::now();
  auto now_s = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count(); };
  if (!h || !h->has_problem) return fail(SFM_EINVAL, "no problem set");
  sfm_ba_options opts;
  if (opts_in) opts = *opts_in; else sfm_ba_default_options(&opts);
  if (const char* why = invalid_option(opts)) return fail(SFM_EINVAL, std::string("invalid option: ") + why);
  sfm_ba_summary sm;
  std::memset(&sm, 0, sizeof(sm));
  int tl = 0;
  if (trace_len) *trace_len = 0;
  auto push = [&](const sfm_ba_iteration& it) {
    if (trace && tl < trace_cap) trace[tl] = it;
    ++tl;
    if (trace_len) *trace_len = std::min(tl, trace_cap);
  };
  if (mode < 0 || mode > 2 || h->d.N == 0) {
    // the reference adds no residual blocks for other modes (CTracker.cpp:692-693)
    sm.termination_type = SFM_CONVERGENCE;
    if (summary) *summary = sm;
    return 0;
  }
  HIPCHK(hipSetDevice(h->device));
  DevProblem& d = h->d;
  h->mode = mode;
  d.min_diag = opts.min_lm_diagonal;
  d.max_diag = opts.max_lm_diagonal;
  int rc;
  if (!opts.jacobi_scaling) {
    std::vector<double> ones(std::max(6 * size_t(d.C), 3 * size_t(d.P)), 1.0);
    HIPCHK(hipMemcpyAsync(d.scale_c, ones.data(), sizeof(double) * 6 * d.C, hipMemcpyHostToDevice, h->stream));
    if (d.P) HIPCHK(hipMemcpyAsync(d.scale_p, ones.data(), sizeof(double) * 3 * d.P, hipMemcpyHostToDevice, h->stream));
  }
  // constant blocks (CTracker.cpp:679-687): zero scale, so the scaled
  // Jacobian columns of the constant side vanish and its step is zero
  if (mode == SFM_BA_STRUCT_ONLY && d.C) HIPCHK(hipMemsetAsync(d.scale_c, 0, sizeof(double) * 6 * d.C, h->stream));
  if (mode == SFM_BA_POSE_ONLY && d.P) HIPCHK(hipMemsetAsync(d.scale_p, 0, sizeof(double) * 3 * d.P, h->stream));
  double* sc = d.scal_host;
  // (the distributed factor's panel loop runs in the host-driven loop: its
  // collectives are not gated; at the sizes it is for, a host round trip per
  // phase is noise)
  if (!h->host_fn && !h->coll_fn && !(sharded(h) && h->dist_pt > 0) && !env_flag("SFM_HOST_LM")) {
    // the same loop with its decisions on the device (k_lm_init /
    // k_lm_decide / k_lm_post): the initial evaluation and the iterations
    // are enqueued in batches, one host synchronisation per batch instead
    // of two per iteration.  With an RCCL communicator the all-reduces are
    // enqueued on the same stream and every rank decides from the same
    // reduced scalars; only the host-callback collective (tests) needs the
    // host loop.
    double cost = 0.0;
    bool nonfinite = false;
    rc = run_device_lm(h, opts, &cost, &sm, push, &nonfinite);
    if (rc) {
      if (nonfinite && summary) *summary = sm;
      return rc;
    }
    // (per-phase host times stay 0 here: the phases run asynchronously)
    sm.final_cost = cost;
    sm.wall_time_s = now_s();
    if (summary) *summary = sm;
    return 0;
  }
  double tj = now_s();
  if ((rc = evaluate(h, true, opts.jacobi_scaling != 0))) return rc;
  sm.jacobian_time_s += now_s() - tj;
  sm.num_jacobian_evaluations++;
  sm.num_residual_evaluations++;
  double cost = sc[kCost];
  sm.initial_cost = cost;
  if (!std::isfinite(cost)) {
    sm.termination_type = SFM_FAILURE;
    sm.final_cost = cost;
    if (summary) *summary = sm;
    return fail(SFM_EIO, "initial residual evaluation is not finite");
  }
  double grad_max = std::max(sc[kGradMaxCam], sc[kGradMaxPt]);
  double x_norm = std::sqrt(sc[kXNorm2Cam] + sc[kXNorm2Pt]);
  {
    sfm_ba_iteration it0;
    std::memset(&it0, 0, sizeof(it0));
    it0.cost = cost;
    it0.gradient_max_norm = grad_max;
    it0.trust_region_radius = opts.initial_trust_region_radius;
    it0.step_is_valid = 1;
    it0.step_is_successful = 1;
    push(it0);
  }
  if (grad_max <= opts.gradient_tolerance) {
    sm.termination_type = SFM_CONVERGENCE;
  } else {
    double radius = opts.initial_trust_region_radius;
    double decrease_factor = 2.0;
    int num_consecutive_invalid = 0;
    int iteration = 0;
    while (true) {
      if (iteration >= opts.max_num_iterations) { sm.termination_type = SFM_NO_CONVERGENCE; break; }
      ++iteration;
      sfm_ba_iteration itr;
      std::memset(&itr, 0, sizeof(itr));
      itr.iteration = iteration;
      const double tls = now_s();
      if ((rc = compute_step(h, radius))) return rc;
      sm.linear_solver_time_s += now_s() - tls;
      sm.num_linear_solves++;
      int chol_fail = 0;
      std::memcpy(&chol_fail, sc + kNumScalars, sizeof(int));
      // The persistent grids' waits are bounded (roles go by start order, so
      // a partly resident grid still progresses); a timeout reports here
      // (INTEGRATION.md §2).
      if (chol_fail & 4) return fail(SFM_EIO, "Cholesky tile hand-off timed out (persistent grid made no progress)");
      if (chol_fail & 2) return fail(SFM_EIO, "back-substitution hand-off timed out (persistent grid made no progress)");
      const bool solve_ok = chol_fail == 0 && !(sc[kBadStep] > 0.0) && !(sc[kBadCam] > 0.0) && !(sc[kBadBack] > 0.0);
      const double model_cost_change = sc[kModelChange] + sc[kModelChangePt];
      itr.step_is_valid = (solve_ok && model_cost_change >= 0.0) ? 1 : 0;
      itr.step_is_successful = 0;
      if (!itr.step_is_valid) {
        ++num_consecutive_invalid;
        sm.num_invalid_steps++;
        if (num_consecutive_invalid >= opts.max_num_consecutive_invalid_steps) {
          sm.termination_type = SFM_FAILURE;
          itr.cost = cost; itr.gradient_max_norm = grad_max; itr.trust_region_radius = radius;
          push(itr);
          break;
        }
        itr.cost = cost;
        itr.gradient_max_norm = grad_max;
      } else {
        num_consecutive_invalid = 0;
        double new_cost = sc[kNewCost];
        if (!std::isfinite(new_cost)) new_cost = std::numeric_limits<double>::max();
        sm.num_residual_evaluations++;
        itr.step_norm = std::sqrt(sc[kStep2Cam] + sc[kStep2Pt]);
        const double step_size_tolerance = opts.parameter_tolerance * (x_norm + opts.parameter_tolerance);
        if (itr.step_norm <= step_size_tolerance) {
          sm.termination_type = SFM_CONVERGENCE;
          itr.cost = cost; itr.gradient_max_norm = grad_max; itr.trust_region_radius = radius;
          push(itr);
          break;
        }
        itr.cost_change = cost - new_cost;
        if (std::fabs(itr.cost_change) <= opts.function_tolerance * cost) {
          sm.termination_type = SFM_CONVERGENCE;
          itr.cost = cost; itr.gradient_max_norm = grad_max; itr.trust_region_radius = radius;
          push(itr);
          break;
        }
        itr.relative_decrease = itr.cost_change / model_cost_change;
        itr.step_is_successful = itr.relative_decrease > opts.min_relative_decrease;
      }
      if (itr.step_is_successful) {
        sm.num_successful_steps++;
        const double q = 2.0 * itr.relative_decrease - 1.0;  // (2 rho - 1)^3, as k_lm_decide
        radius = radius / std::max(1.0 / 3.0, 1.0 - q * q * q);
        radius = std::min(opts.max_trust_region_radius, radius);
        decrease_factor = 2.0;
        std::swap(d.cam, d.cam_new);
        std::swap(d.X, d.X_new);
        tj = now_s();
        if ((rc = evaluate(h, false, opts.jacobi_scaling != 0))) return rc;
        sm.jacobian_time_s += now_s() - tj;
        sm.num_jacobian_evaluations++;
        sm.num_residual_evaluations++;
        cost = sc[kCost];
        if (!std::isfinite(cost)) { sm.termination_type = SFM_FAILURE; break; }
        grad_max = std::max(sc[kGradMaxCam], sc[kGradMaxPt]);
        x_norm = std::sqrt(sc[kXNorm2Cam] + sc[kXNorm2Pt]);
      } else {
        sm.num_unsuccessful_steps++;
        radius = radius / decrease_factor;
        decrease_factor *= 2.0;
      }
      itr.gradient_max_norm = grad_max;
      itr.cost = cost;
      itr.trust_region_radius = radius;
      push(itr);
      if (itr.step_is_successful) {
        if (grad_max <= opts.gradient_tolerance) { sm.termination_type = SFM_CONVERGENCE; break; }
      } else {
        if (radius < opts.min_trust_region_radius) { sm.termination_type = SFM_CONVERGENCE; break; }
      }
    }
    sm.num_iterations = iteration;
  }
  sm.final_cost = cost;
  sm.wall_time_s = now_s();
  if (summary) *summary = sm;
  return 0;
}

int sfm_ba_solve(const sfm_ba_options* opts, int32_t mode, int64_t n_obs, const double* obs_uv,
                 const int32_t* cam_idx, const int32_t* pt_idx, int32_t n_cams, const double* K9, double* rot,
                 double* t, int32_t n_pts, double* X, sfm_ba_summary* summary, sfm_ba_iteration* trace,
                 int32_t trace_cap, int32_t* trace_len) {
  SFM_TRACE("sfm_ba_solve");
  if (mode < 0 || mode > 2 || n_obs == 0) {
    if (summary) { std::memset(summary, 0, sizeof(*summary)); summary->termination_type = SFM_CONVERGENCE; }
    if (trace_len) *trace_len = 0;
    return 0;
  }
  int dev = 0;
  hipGetDevice(&dev);
  // One cached handle per device and calling thread: the drop-in is called
  // once per keyframe (CSfM.cpp:259, 970), so the stream, the pinned mirror
  // and (through the pool) the device buffers are created once, not per call
  // (measured at C1: create 1.7 ms + destroy 2.2 ms against a 1.9-ms solve).
  // The cache owns its handles: they are destroyed (stream, pinned mirror,
  // pooled device buffers) when the calling thread exits.
  struct HandleCache {
    std::map<int, sfm_ba_handle*> by_dev;
    ~HandleCache() {
      for (auto& kv : by_dev)
        if (kv.second) sfm_ba_destroy(kv.second);
    }
  };
  static thread_local HandleCache cache;
  sfm_ba_handle*& h = cache.by_dev[dev];
  int rc = 0;
  if (!h && (rc = sfm_ba_create(dev, &h))) {
    h = nullptr;
    return rc;
  }
  rc = sfm_ba_set_problem(h, n_obs, obs_uv, cam_idx, pt_idx, n_cams, K9, rot, t, n_pts, X);
  // small problems: the parameters ride in the solve's last control readback
  const size_t np = 6 * size_t(std::max(0, n_cams)) + 3 * size_t(std::max(0, n_pts));
  if (!rc && np * sizeof(double) <= kParamPrefetchMaxBytes) {
    if (h->param_host_cap < np) {
      if (h->param_host) {
        (void)hipStreamSynchronize(h->stream);
        (void)hipHostFree(h->param_host);
      }
      h->param_host = nullptr;
      h->param_host_cap = 0;
      if (hipHostMalloc(reinterpret_cast<void**>(&h->param_host), std::max<size_t>(np, 4096) * sizeof(double)) ==
          hipSuccess)
        h->param_host_cap = std::max<size_t>(np, 4096);
      else
        h->param_host = nullptr;
    }
    h->prefetch_params = h->param_host != nullptr;
  }
  h->param_host_valid = false;
  if (!rc) rc = sfm_ba_solve_resident(h, opts, mode, summary, trace, trace_cap, trace_len);
  h->prefetch_params = false;
  if (!rc && h->param_host_valid) {
    const double* cam = h->param_host;
    for (int c = 0; c < n_cams; ++c)
      for (int j = 0; j < 3; ++j) {
        rot[3 * c + j] = cam[6 * c + j];
        t[3 * c + j] = cam[6 * c + 3 + j];
      }
    if (n_pts) std::memcpy(X, h->param_host + 6 * size_t(n_cams), sizeof(double) * 3 * size_t(n_pts));
    h->param_host_valid = false;
    return 0;
  }
  h->param_host_valid = false;
  if (!rc) rc = sfm_ba_get_parameters(h, rot, t, X);
  return rc;
}

// The record array of the evaluate API (the solve writes no records):
// allocated on first use, kept with the problem.
static int ensure_records(sfm_ba_handle* h) {
  DevProblem& d = h->d;
  if (d.jrec || d.N_pad == 0) return 0;
  return dalloc(h, &d.jrec, size_t(kJRec) * size_t(d.N_pad));
}

int sfm_ba_evaluate(sfm_ba_handle* h, double* cost, double* res, double* jac) {
  SFM_TRACE("sfm_ba_evaluate");
  if (!h || !h->has_problem) return fail(SFM_EINVAL, "no problem set");
  HIPCHK(hipSetDevice(h->device));
  DevProblem& d = h->d;
  int rc;
  if ((rc = ensure_records(h))) return rc;
  launch_cam_prep(d, d.cam, false, h->stream);
  launch_jacobian(d, false, h->stream, true);  // the records are the output
  if (d.N == 0) HIPCHK(hipMemsetAsync(d.partials, 0, sizeof(double), h->stream));
  // the record-writing grid (jac_blocks_rec) wrote the cost partials: the
  // solve's larger grid's extra slots still hold the last solve's partials
  launch_reduce(d, kPCost, d.jac_blocks_rec, 0, kCost, h->stream);
  std::vector<double> rec(size_t(kJRec) * d.N_pad);
  std::vector<int32_t> order(size_t(d.N)), pos(size_t(d.N));
  if (d.N) {
    HIPCHK(hipMemcpyAsync(rec.data(), d.jrec, sizeof(double) * rec.size(), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipMemcpyAsync(order.data(), d.order, sizeof(int32_t) * order.size(), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipMemcpyAsync(pos.data(), d.pos, sizeof(int32_t) * pos.size(), hipMemcpyDeviceToHost, h->stream));
  }
  double c = 0;
  HIPCHK(hipMemcpyAsync(&c, d.scal + kCost, sizeof(double), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (cost) *cost = c;
  for (int64_t q = 0; q < d.N; ++q) {
    const int64_t i = order[q];
    const double* r = &rec[size_t(kJRec) * pos[q]];
    if (res) { res[2 * i] = r[kRes]; res[2 * i + 1] = r[kRes + 1]; }
    if (jac) {
      double* J = jac + 18 * i;
      for (int row = 0; row < 2; ++row) {
        for (int k = 0; k < 6; ++k) J[9 * row + k] = r[kJC + 6 * row + k];
        for (int k = 0; k < 3; ++k) J[9 * row + 6 + k] = r[kJX + 3 * row + k];
      }
    }
  }
  return 0;
}

int sfm_dist_factor_profile(int32_t device, int32_t n, int32_t nranks, int32_t panel_tiles, double* fac_ms,
                            double* pack_ms, double* unpack_ms, double* upd_ms, double* misc_ms) {
  if (n <= 0 || nranks < 1 || panel_tiles < 1 || !fac_ms || !pack_ms || !unpack_ms || !upd_ms || !misc_ms)
    return fail(SFM_EINVAL, "bad arguments");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return fail(SFM_ENODEV, "no device");
  HIPCHK(hipSetDevice(device));
  DevProblem d;
  d.n = n;
  d.ld = ((n + 1 + kNB - 1) / kNB) * kNB;
  d.nblk = d.ld / kNB;
  const int pt = panel_tiles, np = (d.nblk + pt - 1) / pt;
  const size_t bytes = sizeof(double) * size_t(d.ld) * d.ld;
  hipStream_t s = nullptr;
  HIPCHK(hipStreamCreate(&s));
  double *S = nullptr, *invd = nullptr, *ys = nullptr, *buf = nullptr;
  int *fl = nullptr, *flags = nullptr;
  const size_t nflag = d.nblk + 2 * size_t(d.nblk) * d.nblk + 16;
  HIPCHK(hipMalloc(&S, bytes));
  HIPCHK(hipMalloc(&invd, sizeof(double) * size_t(d.nblk) * kNB * kNB));
  HIPCHK(hipMemset(invd, 0, sizeof(double) * size_t(d.nblk) * kNB * kNB));
  HIPCHK(hipMalloc(&flags, sizeof(int) * nflag));
  HIPCHK(hipMemset(flags, 0, sizeof(int) * nflag));
  HIPCHK(hipMalloc(&ys, sizeof(double) * d.ld));
  HIPCHK(hipMalloc(&fl, sizeof(int)));
  HIPCHK(hipMemset(fl, 0, sizeof(int)));
  // one panel rectangle (the broadcast buffer) / the whole lower image (the
  // reduce-scatter's send buffer)
  HIPCHK(hipMalloc(&buf, bytes));
  HIPCHK(hipMemset(buf, 0, bytes));
  d.S = S; d.invL = invd; d.ysol = ys; d.fail = fl; d.flags = flags;
  d.cflags = flags + d.nblk;
  d.cticket = reinterpret_cast<unsigned long long*>(flags + d.nblk + 2 * size_t(d.nblk) * d.nblk);
  if (reinterpret_cast<uintptr_t>(d.cticket) % 8) d.cticket = reinterpret_cast<unsigned long long*>(flags + d.nblk + 2 * size_t(d.nblk) * d.nblk + 1);
  d.n_cu = device_cus(device);
  std::vector<hipEvent_t> ev(4 * size_t(np) + 8);
  for (auto& e : ev) HIPCHK(hipEventCreate(&e));
  auto el = [&](hipEvent_t a, hipEvent_t b) {
    float m = 0.f;
    (void)hipEventElapsedTime(&m, a, b);
    return double(m);
  };
  // offsets of every panel in a whole-image buffer (the reduce-scatter pack)
  std::vector<int64_t> off(static_cast<size_t>(np));
  int64_t tot = 0;
  for (int J = 0; J < np; ++J) {
    off[J] = tot;
    const int c0 = J * pt * kNB, c1 = std::min((J + 1) * pt * kNB, n + 1);
    tot += c1 > c0 ? int64_t(c1 - c0) * (n + 1 - c0) : 0;
  }
  int64_t* doff = nullptr;
  HIPCHK(hipMalloc(&doff, sizeof(int64_t) * np));
  HIPCHK(hipMemcpy(doff, off.data(), sizeof(int64_t) * np, hipMemcpyHostToDevice));
  int epoch = 0;
  for (int rank = 0; rank < nranks; ++rank) {
    launch_spd_fill(S, d.ld, n, 12345u, s);
    if (rank == 0) {  // reduce-scatter pack + unpack of the whole image, the back substitution
      HIPCHK(hipEventRecord(ev[0], s));
      launch_panel_copy(d, kPanelPack, pt, 0, n + 1, doff, 0, buf, s);
      HIPCHK(hipEventRecord(ev[1], s));
      launch_panel_copy(d, kPanelAdd, pt, 0, n + 1, doff, 0, buf, s);
      HIPCHK(hipEventRecord(ev[2], s));
    }
    for (int k = 0; k < np; ++k) {
      const int owner = k % nranks, t0 = k * pt, ncols = std::min(pt, d.nblk - t0);
      const int c0 = t0 * kNB, c1 = c0 + ncols * kNB;
      if (owner != rank) {  // a zero L for the panels this rank receives: its own panels stay SPD
        const int64_t cols = std::min(c1, n + 1) - c0;
        HIPCHK(hipMemsetAsync(buf + tot, 0, sizeof(double) * (cols * (n + 1 - c0) + int64_t(ncols) * kNB * kNB + 1), s));
      }
      HIPCHK(hipEventRecord(ev[8 + 4 * k], s));
      if (owner == rank) {
        launch_cholesky_panel(d, k, pt, ++epoch, s);
        HIPCHK(hipEventRecord(ev[8 + 4 * k + 1], s));
        launch_panel_copy(d, kPanelPack, pt, c0, c1, nullptr, tot, buf, s);
      } else {
        HIPCHK(hipEventRecord(ev[8 + 4 * k + 1], s));
        launch_panel_copy(d, kPanelUnpack, pt, c0, c1, nullptr, tot, buf, s);
      }
      HIPCHK(hipEventRecord(ev[8 + 4 * k + 2], s));
      launch_panel_update(d, k, k + 1, INT32_MAX / 2, pt, nranks, rank, s);
      HIPCHK(hipEventRecord(ev[8 + 4 * k + 3], s));
    }
    if (rank == 0) {
      HIPCHK(hipMemsetAsync(ys, 0xFF, sizeof(double) * d.ld, s));
      HIPCHK(hipEventRecord(ev[3], s));
      launch_backsolve(d, 1, s);
      HIPCHK(hipEventRecord(ev[4], s));
    }
    HIPCHK(hipStreamSynchronize(s));
    for (int k = 0; k < np; ++k) {
      const bool own = k % nranks == rank;
      if (own) fac_ms[k] = el(ev[8 + 4 * k], ev[8 + 4 * k + 1]);
      (own ? pack_ms : unpack_ms)[k] = el(ev[8 + 4 * k + 1], ev[8 + 4 * k + 2]);
      upd_ms[size_t(rank) * np + k] = el(ev[8 + 4 * k + 2], ev[8 + 4 * k + 3]);
    }
    if (rank == 0) {
      misc_ms[0] = el(ev[0], ev[1]);  // reduce-scatter pack
      misc_ms[1] = el(ev[1], ev[2]);  // unpack
      misc_ms[2] = el(ev[3], ev[4]);  // back substitution
    }
  }
  int f = 0;
  HIPCHK(hipMemcpy(&f, fl, sizeof(int), hipMemcpyDeviceToHost));
  misc_ms[3] = f;
  misc_ms[4] = double(tot);  // doubles of the whole panel image
  for (auto e : ev) hipEventDestroy(e);
  hipFree(S); hipFree(invd); hipFree(flags); hipFree(ys); hipFree(fl); hipFree(buf); hipFree(doff);
  hipStreamDestroy(s);
  return 0;
}

int sfm_dense_spd_solve(int32_t device, int32_t n, const double* A, const double* b, double* y, int32_t reps,
                        double* ms, int32_t* chol_fail) {
  if (n <= 0 || !A || !b || !y || reps < 1) return fail(SFM_EINVAL, "bad arguments");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return fail(SFM_ENODEV, "no device");
  HIPCHK(hipSetDevice(device));
  DevProblem d;
  d.n = n;
  d.ld = ((n + 1 + kNB - 1) / kNB) * kNB;
  d.nblk = d.ld / kNB;
  // augmented column-major-lower image: (i, j) at j*ld + i, i >= j
  std::vector<double> img(size_t(d.ld) * d.ld, 0.0);
  for (int j = 0; j < n; ++j)
    for (int i = j; i < n; ++i) img[size_t(j) * d.ld + i] = A[size_t(j) * n + i];  // row-major upper (j, i)
  for (int j = 0; j < n; ++j) img[size_t(j) * d.ld + n] = b[j];
  for (int j = n; j < d.ld; ++j) img[size_t(j) * d.ld + j] = 1.0;
  double *S = nullptr, *S0 = nullptr, *invd = nullptr, *ys = nullptr;
  int *fl = nullptr, *flags = nullptr;
  const size_t bytes = sizeof(double) * img.size();
  hipStream_t s = nullptr;
  HIPCHK(hipStreamCreate(&s));
  HIPCHK(hipMalloc(&S, bytes));
  HIPCHK(hipMalloc(&S0, bytes));
  HIPCHK(hipMalloc(&invd, sizeof(double) * size_t(d.nblk) * kNB * kNB));
  HIPCHK(hipMemset(invd, 0, sizeof(double) * size_t(d.nblk) * kNB * kNB));
  HIPCHK(hipMalloc(&flags, sizeof(int) * (d.nblk + 2 * size_t(d.nblk) * d.nblk + 16)));
  HIPCHK(hipMemset(flags, 0, sizeof(int) * (d.nblk + 2 * size_t(d.nblk) * d.nblk + 16)));
  HIPCHK(hipMalloc(&ys, sizeof(double) * d.ld));
  HIPCHK(hipMalloc(&fl, sizeof(int)));
  HIPCHK(hipMemcpy(S0, img.data(), bytes, hipMemcpyHostToDevice));
  d.S = S; d.invL = invd; d.ysol = ys; d.fail = fl; d.flags = flags;
  d.cflags = flags + d.nblk;
  d.cticket = reinterpret_cast<unsigned long long*>(flags + d.nblk + 2 * size_t(d.nblk) * d.nblk);
  if (reinterpret_cast<uintptr_t>(d.cticket) % 8) d.cticket = reinterpret_cast<unsigned long long*>(flags + d.nblk + 2 * size_t(d.nblk) * d.nblk + 1);
  d.n_cu = device_cus(device);
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  float total = 0.f;
  for (int r = 0; r < reps; ++r) {
    HIPCHK(hipMemcpyAsync(S, S0, bytes, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipEventRecord(e0, s));
    launch_cholesky(d, r + 1, s);
    launch_backsolve(d, r + 1, s);
    HIPCHK(hipEventRecord(e1, s));
    HIPCHK(hipEventSynchronize(e1));
    float m = 0.f;
    HIPCHK(hipEventElapsedTime(&m, e0, e1));
    if (r > 0 || reps == 1) total += m;
  }
  int f = 0;
  HIPCHK(hipMemcpy(&f, fl, sizeof(int), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(y, ys, sizeof(double) * n, hipMemcpyDeviceToHost));
  if (ms) *ms = total / (reps > 1 ? reps - 1 : 1);
  if (chol_fail) *chol_fail = f;
  hipEventDestroy(e0); hipEventDestroy(e1);
  hipFree(S); hipFree(S0); hipFree(invd); hipFree(flags); hipFree(ys); hipFree(fl);
  hipStreamDestroy(s);
  return 0;
}

int sfm_ba_bench_jacobian(sfm_ba_handle* h, int32_t reps, double* avg_ms) {
  if (!h || !h->has_problem || reps < 1) return fail(SFM_EINVAL, "bad arguments");
  HIPCHK(hipSetDevice(h->device));
  DevProblem& d = h->d;
  int rc;
  if ((rc = ensure_records(h))) return rc;
  launch_cam_prep(d, d.cam, false, h->stream);
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  launch_jacobian(d, true, h->stream, true);  // warm (the record-writing pass is what is measured)
  HIPCHK(hipEventRecord(e0, h->stream));
  for (int i = 0; i < reps; ++i) launch_jacobian(d, true, h->stream, true);
  HIPCHK(hipEventRecord(e1, h->stream));
  HIPCHK(hipEventSynchronize(e1));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, e0, e1));
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  if (avg_ms) *avg_ms = double(ms) / reps;
  return 0;
}

}  // extern "C"
