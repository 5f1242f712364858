/*
 * sfm_amd — MI355X-native bundle-adjustment + feature-tracking core for the
 * hulop/SfM pipeline.  Plain C ABI: no C++ types, no exceptions, caller-owned
 * arrays, 0 / negative-errno return codes, sfm_last_error() for the message.
 *
 * Drop-in boundary.  Each entry point names the reference
 * interface it replaces:
 *
 *   sfm_ba_solve
 *     replaces void CTracker::bundleAdjustmentStructAndPose(
 *         const vector<Point2d>& observations, const vector<int>& camIdx,
 *         const vector<Matx33d>& K, vector<double*>& R, vector<double*>& t,
 *         vector<double*>& pts3D, int isStructOrPose)
 *     declared /root/reference/CTracker.h:65, defined CTracker.cpp:670-702,
 *     called from CSfM::bundleAdjustment (CSfM.cpp:343).  The reference
 *     identifies parameter blocks by address (duplicated double* per
 *     observation); this ABI takes the deduplicated form: pt_idx[i] indexes
 *     X[n_pts][3] (include/sfm_ctracker_compat.hpp does the address
 *     dedup and the in-place scatter-back for C++ callers).
 *     Ceres' ceres::Solver::Summary, which the reference discards
 *     (CTracker.cpp:700-701), is returned in *summary.
 *
 *   sfm_match_features
 *     replaces CTracker::matchFeatures(pts0, desc0, pts1, desc1, idx0, idx1,
 *     minDistance, maxDistance)  (CTracker.h:55, CTracker.cpp:211-250) and,
 *     with min/max = 1.5/40 (CTracker.cpp:30-31), the member-window overload
 *     (CTracker.h:53, CTracker.cpp:114-149).  The index-subset overload
 *     (CTracker.h:56, CTracker.cpp:368-417) is the same call on gathered
 *     rows followed by an index map (sfm_amd/ctracker.py, the compat header).
 *
 *   sfm_klt_compute_optical_flow
 *     replaces bool CTracker::computeOpticalFlow()  (CTracker.h:60,
 *     CTracker.cpp:480-562): pyramidal Lucas-Kanade from the previous to
 *     the current frame (cv::calcOpticalFlowPyrLK, CTracker.cpp:513), the
 *     nearest-detected-point association (CFrame::
 *     findClosestPointIndexDistorted, CFrame.cpp:437-450) and the gate /
 *     replacement loop (CTracker.cpp:515-545) producing _prevIdx/_currIdx.
 *     The frames are CFrame::getFrameGrey() (8-bit grey), pushed once each
 *     with sfm_klt_push_frame (the pyramid stays resident in HBM).
 *
 * Every function is synchronous with respect to the caller's host buffers.
 */
#ifndef SFM_AMD_H_
#define SFM_AMD_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SFM_ABI_VERSION 1

/* Error codes (negative errno values). */
#define SFM_OK 0
#define SFM_EINVAL (-22)   /* bad argument / out-of-range index / non-finite input */
#define SFM_ENOMEM (-12)   /* device allocation failed */
#define SFM_ENODEV (-19)   /* no usable HIP device */
#define SFM_EIO (-5)       /* HIP / RCCL runtime error */
#define SFM_ENOTSUP (-95)  /* reserved: operation not supported */

/* BA_TYPE (CTracker.h:67). */
#define SFM_BA_STRUCT_ONLY 0
#define SFM_BA_POSE_ONLY 1
#define SFM_BA_STRUCT_AND_POSE 2

/* The Ceres options that matter for the reference's solve.  The reference
 * sets linear_solver_type = DENSE_SCHUR and silent logging and leaves every
 * other option at its Ceres default (CTracker.cpp:571-577);
 * sfm_ba_default_options() returns those defaults. */
typedef struct sfm_ba_options {
  int32_t max_num_iterations;                /* 50 */
  int32_t max_num_consecutive_invalid_steps; /* 5 */
  int32_t jacobi_scaling;                    /* 1 */
  int32_t reserved0;
  double function_tolerance;          /* 1e-6 */
  double gradient_tolerance;          /* 1e-10 */
  double parameter_tolerance;         /* 1e-8 */
  double initial_trust_region_radius; /* 1e4 */
  double max_trust_region_radius;     /* 1e16 */
  double min_trust_region_radius;     /* 1e-32 */
  double min_lm_diagonal;             /* 1e-6 */
  double max_lm_diagonal;             /* 1e32 */
  double min_relative_decrease;       /* 1e-3 */
} sfm_ba_options;

/* termination_type values (ceres::TerminationType subset). */
#define SFM_CONVERGENCE 0
#define SFM_NO_CONVERGENCE 1
#define SFM_FAILURE 2

typedef struct sfm_ba_summary {
  int32_t termination_type;
  int32_t num_iterations; /* LM iterations (iteration 0 = initial evaluation not counted) */
  int32_t num_successful_steps;
  int32_t num_unsuccessful_steps;
  int32_t num_invalid_steps;
  int32_t num_residual_evaluations; /* full residual-vector evaluations (Jacobian passes included) */
  int32_t num_jacobian_evaluations;
  int32_t num_linear_solves;
  double initial_cost;
  double final_cost;
  double wall_time_s;
  /* Per-phase host times: filled by the host-driven LM loop only
     (SFM_HOST_LM=1, or a host-callback collective).  The default
     device-driven loop enqueues its phases asynchronously; it leaves these
     0 and wall_time_s is the whole solve. */
  double jacobian_time_s;
  double linear_solver_time_s;
  double residual_time_s;
} sfm_ba_summary;

/* One entry per iteration (ceres::IterationSummary subset). */
typedef struct sfm_ba_iteration {
  int32_t iteration;
  int32_t step_is_valid;
  int32_t step_is_successful;
  int32_t reserved;
  double cost;
  double cost_change;
  double gradient_max_norm;
  double step_norm;
  double relative_decrease;
  double trust_region_radius;
} sfm_ba_iteration;

typedef struct sfm_ba_handle sfm_ba_handle;

int32_t sfm_abi_version(void);
const char* sfm_last_error(void);
void sfm_ba_default_options(sfm_ba_options* opts);
/* Number of visible HIP devices (0 without a GPU; never fails). */
int32_t sfm_device_count(void);

/* One-shot drop-in solve (host arrays in, results written in place):
 *   obs_uv [n_obs][2] undistorted pixel observations (CFrame::_pts, Kopt frame)
 *   cam_idx[n_obs] in [0, n_cams), pt_idx[n_obs] in [0, n_pts)
 *   K9 [n_cams][9] row-major Matx33d::val (only [0],[1],[2],[4],[5] are read)
 *   rot, t [n_cams][3] angle-axis / translation (CFrame::_rot, _t); X [n_pts][3]
 * mode: SFM_BA_* (any other value adds no residuals: returns 0, no change).
 * trace (optional): per-iteration records, capacity trace_cap, *trace_len set. */
int sfm_ba_solve(const sfm_ba_options* opts, int32_t mode, int64_t n_obs, const double* obs_uv,
                 const int32_t* cam_idx, const int32_t* pt_idx, int32_t n_cams, const double* K9, double* rot,
                 double* t, int32_t n_pts, double* X, sfm_ba_summary* summary, sfm_ba_iteration* trace,
                 int32_t trace_cap, int32_t* trace_len);

/* Resident-problem API (problem uploaded once, solved many times from HBM).
 * With sfm_ba_set_comm the problem is one landmark shard of a larger one:
 * every rank passes ALL cameras and its own points / observations. */
int sfm_ba_create(int32_t device, sfm_ba_handle** out);
int sfm_ba_destroy(sfm_ba_handle* h);
int sfm_ba_set_problem(sfm_ba_handle* h, int64_t n_obs, const double* obs_uv, const int32_t* cam_idx,
                       const int32_t* pt_idx, int32_t n_cams, const double* K9, const double* rot, const double* t,
                       int32_t n_pts, const double* X);
/* Restore the parameters given to sfm_ba_set_problem (device-to-device). */
int sfm_ba_reset_parameters(sfm_ba_handle* h);
int sfm_ba_solve_resident(sfm_ba_handle* h, const sfm_ba_options* opts, int32_t mode, sfm_ba_summary* summary,
                          sfm_ba_iteration* trace, int32_t trace_cap, int32_t* trace_len);
int sfm_ba_get_parameters(sfm_ba_handle* h, double* rot, double* t, double* X);
/* One residual + Jacobian pass at the current parameters (unscaled J).
 * res [n_obs][2], jac [n_obs][2][9] (columns dR | dt | dX) in the caller's
 * observation order; either may be NULL; *cost = 1/2 |r|^2 (may be NULL). */
int sfm_ba_evaluate(sfm_ba_handle* h, double* cost, double* res, double* jac);
/* `reps` back-to-back Jacobian passes on the resident problem (benchmark
 * of the HBM-bound kernel); *avg_ms = mean duration per pass (HIP events). */
int sfm_ba_bench_jacobian(sfm_ba_handle* h, int32_t reps, double* avg_ms);
/* Per-phase device time of the last solve (ms): [jacobian, cam_reduce,
 * point_eval, point_prep, schur, cholesky, backsolve, backsub, other]. */
int sfm_ba_phase_times(sfm_ba_handle* h, double* ms9);
/* Enable per-phase HIP-event timing for subsequent solves (events on the
 * solver stream, read at the per-iteration scalar sync: no extra syncs). */
int sfm_ba_set_profiling(sfm_ba_handle* h, int32_t on);
/* Synchronise the handle's stream. */
int sfm_ba_sync(sfm_ba_handle* h);

/* Multi-GPU (landmark sharding, RCCL over xGMI).  Rank 0 creates the id,
 * the caller distributes its 128 bytes (e.g. torch.distributed), every rank
 * calls sfm_ba_set_comm before sfm_ba_set_problem. */
int sfm_comm_unique_id(uint8_t out[128]);
int sfm_ba_set_comm(sfm_ba_handle* h, int32_t nranks, int32_t rank, const uint8_t id[128]);
/* Test hook: the same sharded path with the all-reduce done by a host
 * callback (in place on `count` doubles; op 0 = sum, 1 = max; return 0 on
 * success), e.g. over gloo: several ranks can then share ONE GPU, which
 * RCCL does not allow.  Replaces any RCCL communicator. */
typedef int (*sfm_allreduce_fn)(double* buf, int64_t count, int32_t op, void* user);
int sfm_ba_set_host_comm(sfm_ba_handle* h, int32_t nranks, int32_t rank, sfm_allreduce_fn fn, void* user);
/* The same hook with the distributed factor's collectives too (host
 * buffers; return 0 on success):
 *   SFM_COLL_ALLREDUCE       in place on buf[count], arg = op (0 sum, 1 max);
 *   SFM_COLL_BROADCAST       in place on buf[count] from rank `arg`;
 *   SFM_COLL_REDUCE_SCATTER  buf[nranks * count] in rank-segment order; the
 *                            sum of this rank's segment into out[count];
 *   SFM_COLL_REDUCE          the sum over the ranks of buf[count] into buf
 *                            on rank `arg` (the others' buf is unspecified;
 *                            out == buf for this kind).
 * (With sfm_ba_set_host_comm's all-reduce alone, the library builds the
 * others from it.) */
#define SFM_COLL_ALLREDUCE 0
#define SFM_COLL_BROADCAST 1
#define SFM_COLL_REDUCE_SCATTER 2
#define SFM_COLL_REDUCE 3
typedef int (*sfm_collective_fn)(int32_t kind, double* buf, double* out, int64_t count, int32_t arg, void* user);
int sfm_ba_set_host_collectives(sfm_ba_handle* h, int32_t nranks, int32_t rank, sfm_collective_fn fn, void* user);
/* Reduced-camera factor of a sharded solve: 0 (default) =
 * all-reduce of the packed system and a replicated factor on every rank;
 * k > 0 = 1-D block-cyclic panels of k 64-column tiles, each panel's partial
 * systems reduced into its owner, factored there and broadcast (the same
 * Ceres DENSE_SCHUR LLT, distributed; replaces the solve at
 * CTracker.cpp:700-701). */
int sfm_ba_set_distributed_factor(sfm_ba_handle* h, int32_t panel_tiles);

/* Hamming 2-NN matcher + the reference's sequential acceptance rule.
 *   pts0/pts1 [n][2] double positions, desc0/desc1 [n][desc_bytes] (BRISK: 64)
 *   idx0/idx1 capacity >= min(n0, n1); *n_matches = number written.
 * ratio_test 0.8 and (min,max) = (1.5, 40) px in the reference.
 * Falls back to no matches when n1 < 2 (reference UB, CTracker.cpp:224). */
int sfm_match_features(int32_t device, const double* pts0, const uint8_t* desc0, int32_t n0, const double* pts1,
                       const uint8_t* desc1, int32_t n1, int32_t desc_bytes, double ratio_test, double min_distance,
                       double max_distance, int32_t* idx0, int32_t* idx1, int32_t* n_matches);
/* The 2-NN search alone: best/second train index + Hamming distance per query. */
int sfm_knn2_hamming(int32_t device, const uint8_t* desc0, int32_t n0, const uint8_t* desc1, int32_t n1,
                     int32_t desc_bytes, int32_t* best_idx, int32_t* best_dist, int32_t* second_idx,
                     int32_t* second_dist);

/* ---- Frame-resident descriptor matcher --------
 * The per-frame hot loop of CSfM::tracking matches the previous frame's
 * keypoint subset against the current frame's (CTracker::matchFeatures(
 * prevIdx, currIdx, prevMatchIdx, currMatchIdx), CTracker.h:57,
 * CTracker.cpp:368-417, called at CSfM.cpp:518).  A matcher keeps the last
 * two frames' keypoints + descriptors resident in HBM (one upload per
 * frame), pools its buffers, and runs each call as one stream of launches
 * with one host sync.  Rules of every overload: 2-NN Hamming (ties to the
 * lower train index), accept iff d^2 > min^2 && d^2 < max^2 &&
 * float(d0)/float(d1) < ratio && (train unmatched || d0 < its best), a
 * better query replaces the slot's query; fewer than 2 train rows -> no
 * matches (the reference reads matches[i][1] out of range). */
typedef struct sfm_matcher sfm_matcher;
int sfm_matcher_create(int32_t device, int32_t desc_bytes, sfm_matcher** out);
int sfm_matcher_destroy(sfm_matcher* h);
/* New current frame: pts [n][2] undistorted (CFrame::_pts, what getPointsAt
 * returns), pts_distorted [n][2] (CFrame::getPointsDistorted; NULL = pts),
 * desc [n][desc_bytes]; the old current frame becomes the previous one
 * (_prevFrame = _currFrame, CSfM.cpp:626-629). */
int sfm_matcher_push_frame(sfm_matcher* h, const double* pts, const double* pts_distorted, const uint8_t* desc,
                           int32_t n);
/* CTracker::matchFeatures(prevFrameIdx, currFrameIdx, prevMatchIdx,
 * currMatchIdx) (CTracker.cpp:368-417): the keypoint subsets prev_idx of
 * the previous and curr_idx of the current frame, undistorted positions,
 * frame-global indices out (capacity >= min(n_prev, n_curr)).  The
 * reference uses (ratio, min, max) = (0.8, 1.5, 40) (CTracker.cpp:27-31). */
int sfm_matcher_match_subset(sfm_matcher* h, const int32_t* prev_idx, int32_t n_prev, const int32_t* curr_idx,
                             int32_t n_curr, double ratio_test, double min_distance, double max_distance,
                             int32_t* prev_match, int32_t* curr_match, int32_t* n_matches);
/* Keyframe store (CSfM::mapping's keyframe-pair matching, CSfM.cpp:141-221):
 * keyframe slot `slot` takes pts [n][2] and desc [n][desc_bytes], resident
 * on the device until the slot is stored again. */
int sfm_matcher_store_keyframe(sfm_matcher* h, int32_t slot, const double* pts, const uint8_t* desc, int32_t n);
/* The (pts0, desc0, pts1, desc1[, min, max]) overload of matchFeatures
 * (CTracker.cpp:419-477) on stored keyframe rows: query rows q_idx[n_q] of
 * slot q_slot (positions q_pts [n_q][2] when given -- e.g. projections, as
 * CSfM.cpp:199-206 passes them; q_idx must not repeat then -- else the
 * keyframe's own), train rows t_idx[n_t] of slot t_slot.  Subset-local
 * indices out (into q_idx / t_idx), bitwise sfm_matcher_match on the same
 * rows; capacity >= min(n_q, n_t). */
int sfm_matcher_match_keyframes(sfm_matcher* h, int32_t q_slot, const int32_t* q_idx, int32_t n_q, const double* q_pts,
                                int32_t t_slot, const int32_t* t_idx, int32_t n_t, double ratio_test,
                                double min_distance, double max_distance, int32_t* idx0, int32_t* idx1,
                                int32_t* n_matches);
/* bool CTracker::matchFeatures() (CTracker.cpp:419-477): the two whole
 * frames, DISTORTED positions when distorted != 0 (CTracker.cpp:429-430);
 * fills _prevIdx/_currIdx; the reference's bool is n >= _minFeatures. */
int sfm_matcher_match_frames(sfm_matcher* h, int32_t distorted, double ratio_test, double min_distance,
                             double max_distance, int32_t* prev_idx, int32_t* curr_idx, int32_t* n_matches);
/* The (pts0, desc0, pts1, desc1, idx0, idx1[, min, max]) overloads
 * (CTracker.cpp:114-149, 211-250) on host arrays through the handle's pooled
 * buffers (map-point re-finding, CSfM.cpp:208-210, 673). */
int sfm_matcher_match(sfm_matcher* h, const double* pts0, const uint8_t* desc0, int32_t n0, const double* pts1,
                      const uint8_t* desc1, int32_t n1, double ratio_test, double min_distance, double max_distance,
                      int32_t* idx0, int32_t* idx1, int32_t* n_matches);
/* The 2-NN search alone on host arrays. */
int sfm_matcher_knn2(sfm_matcher* h, const uint8_t* desc0, int32_t n0, const uint8_t* desc1, int32_t n1,
                     int32_t* best_idx, int32_t* best_dist, int32_t* second_idx, int32_t* second_dist);
/* Device time (ms, HIP events) of the last match: [2-NN search, whole call on the device]. */
int sfm_matcher_last_time(sfm_matcher* h, double* ms2);

/* CMap::getRepresentativeDescriptors (CMap.cpp:345-381),
 * the map-point descriptors matched at CSfM.cpp:673 and :208-210.  Point i
 * owns rows [row_off[i], row_off[i+1]) of desc [rows][desc_bytes] (one per
 * observing keyframe; row_off[0] = 0, every point >= 1 row).  best[i] = row
 * (within the point) minimising the sum of Hamming distances to the point's
 * rows, the first on ties; out [n_pts][desc_bytes] (optional) = those rows. */
int sfm_representative_descriptors(int32_t device, const uint8_t* desc, const int32_t* row_off, int32_t n_pts,
                                   int32_t desc_bytes, int32_t* best, uint8_t* out);

/* CMap's observation store, resident on the device (SURVEY.md §8f row 2;
 * map_store.hip): points, (frame, keypoint) observations in the multimap's
 * emplace order, descriptor rows per point.  Replaces the multimap gathers
 * of CMap.cpp:145-295 on the tracking path (CSfM.cpp:648-669).  Point
 * indices are the CMap's _lastPtNo numbering (0, 1, ... in creation order).
 * desc_bytes: 8 x a power of two (BRISK 64). */
typedef struct sfm_map sfm_map;
int sfm_map_create(int32_t device, int32_t desc_bytes, sfm_map** out);
int sfm_map_destroy(sfm_map* h);
int sfm_map_size(sfm_map* h, int32_t* n_pts, int64_t* n_obs, int64_t* n_desc_rows);
/* CMap::addNewPoints (CMap.cpp:36-78): pts3d [n_pts][3], frame_no
 * [n_frames], pts2d_idx [n_frames][n_pts] (the reference's
 * vector<vector<int>>, frame-major); new indices out (may be NULL). */
int sfm_map_add_new_points(sfm_map* h, int32_t n_pts, const double* pts3d, int32_t n_frames, const int32_t* frame_no,
                           const int32_t* pts2d_idx, int32_t* pts3d_idx);
/* CMap::addPointMatches (CMap.cpp:118-132). */
int sfm_map_add_point_matches(sfm_map* h, int32_t n, const int32_t* pts3d_idx, const int32_t* pts2d_idx,
                              int32_t frame_no);
/* CMap::addDescriptors (CMap.cpp:308-315): one row [desc_bytes] per point. */
int sfm_map_add_descriptors(sfm_map* h, int32_t n, const int32_t* pts3d_idx, const uint8_t* desc);
/* CMap::getPointsAtIdx (CMap.cpp:134-143) and its inverse (BA write-back). */
int sfm_map_get_points(sfm_map* h, int32_t n, const int32_t* pts3d_idx, double* pts3d);
int sfm_map_set_points(sfm_map* h, int32_t n, const int32_t* pts3d_idx, const double* pts3d);
/* CMap::getPointsInFrames(pts3DIdx, frameNo) (CMap.cpp:277-295): sorted
 * unique points observed in any of the frames.  *n_out = the count; an error
 * when it exceeds capacity. */
int sfm_map_points_in_frames(sfm_map* h, int32_t n_frames, const int32_t* frame_no, int32_t capacity,
                             int32_t* pts3d_idx, int32_t* n_out);
/* CMap::getPointsInFrame(pts3DIdx, pts2DIdx, frameNo) (CMap.cpp:225-240):
 * the frame's equal_range in multimap order; per entry, every 2D index the
 * point has in the frame (so n2 > n3 when a point was matched twice). */
int sfm_map_points_in_frame(sfm_map* h, int32_t frame_no, int32_t capacity, int32_t* pts3d_idx, int32_t* n3_out,
                            int32_t* pts2d_idx, int32_t* n2_out);
/* The BA gather of CSfM::bundleAdjustment (CSfM.cpp:321-340): getPointsInFrame
 * for every frame of frame_no (distinct) in ONE call.  Frame i's output of
 * sfm_map_points_in_frame is pts3d_idx[off3[i] .. off3[i+1]) and
 * pts2d_idx[off2[i] .. off2[i+1]); off3 / off2 [n_frames + 1].  Capacity
 * bounds both arrays; when it is too small the totals are still set in
 * off3[n_frames] / off2[n_frames] and SFM_EINVAL is returned. */
int sfm_map_points_in_frame_multi(sfm_map* h, int32_t n_frames, const int32_t* frame_no, int64_t capacity,
                                  int32_t* pts3d_idx, int32_t* off3, int32_t* pts2d_idx, int32_t* off2);
/* CMap::getRepresentativeDescriptors (CMap.cpp:345-381) from the resident
 * rows: desc_out [n][desc_bytes]; best_row (optional) = the row within the
 * point's rows (append order), first on ties.  Every point needs a row. */
int sfm_map_representative_descriptors(sfm_map* h, int32_t n, const int32_t* pts3d_idx, uint8_t* desc_out,
                                       int32_t* best_row);
/* CSfM::findMapPointsInCurrentFrame (CSfM.cpp:634-692) in one call, on the
 * device: the points seen in the keyframes frame_no[n_frames]
 * (getPointsInFrames, CSfM.cpp:648), minus the frame's already matched points
 * existing_pts[n_existing] (CSfM.cpp:651-662), projected with the frame's pose
 * x = K (R X + t) (R9 row-major rotation, t3, K9 row-major; CSfM.cpp:664-668),
 * their representative descriptors (CSfM.cpp:669), matched against the
 * current frame's keypoints train_idx[n_train] of the frame last pushed to
 * `mt` (sfm_matcher_push_frame) with the (min_distance, max_distance) window
 * of CSfM.cpp:671 (ratio 0.8, 0, _maxReprErr).  Results: pts3d_match[k] (map
 * point) and train_match[k] (frame-global keypoint index), *n_matches of them,
 * in the matcher's order (queries = the new points ascending).  The map and
 * the matcher must share device and descriptor width. */
int sfm_map_match_frame(sfm_map* h, sfm_matcher* mt, int32_t n_frames, const int32_t* frame_no, int32_t n_existing,
                        const int32_t* existing_pts, const double* R9, const double* t3, const double* K9,
                        int32_t n_train, const int32_t* train_idx, double ratio_test, double min_distance,
                        double max_distance, int32_t capacity, int32_t* pts3d_match, int32_t* train_match,
                        int32_t* n_matches);

/* CSfM::tracking's pose step (CSfM.cpp:533-565) in one call, replacing
 * matchFeatures(prevIdx, currIdx) + map->getPointsAtIdx + cv::solvePnPRansac:
 * the previous frame's keypoints with a map point (prev_pt3d[n_prev], one
 * entry per keypoint of the frame pushed before the current one, -1 = none)
 * matched against every keypoint of the current frame of `mt` (undistorted
 * positions; the reference's (ratio, min, max) = (0.8, 1.5, 40)), their map
 * points and keypoints gathered on the device and cv::solvePnPRansac run on
 * them (K9 row-major; the reference's (20, _maxReprErr, 0.99)), with one
 * upload, one download and one host synchronisation.  *n_matches: the match
 * count; below min_matches (MIN_FEATURES, CSfM.cpp:545) no PnP runs and
 * *found = 0.  Found: rvec/tvec and the inliers as (current keypoint,
 * map point) pairs, *n_inliers of them (capacity >= the number of
 * prev_pt3d entries >= 0).  Not found: rvec = tvec = 0, no inliers. */
int sfm_track_pnp(sfm_matcher* mt, sfm_map* map, int32_t n_prev, const int32_t* prev_pt3d, double ratio_test,
                  double min_distance, double max_distance, int32_t min_matches, const double* K9, int32_t iterations,
                  double reproj_err, double confidence, double* rvec, double* tvec, int32_t* found,
                  int32_t* n_matches, int32_t capacity, int32_t* inl_kp, int32_t* inl_pt3d, int32_t* n_inliers);

/* BRISK descriptor (CTracker::detectFeatures' _descriptor->compute,
 * CTracker.cpp:284): BRISK as published in its
 * reference implementation's form (oracle/brisk_oracle.py; the reference's
 * ethz-asl BRISK 2 library is absent, so parity with it is unpinned).
 * img [h][w] 8-bit grey; kps [n][3] = (x, y, size) as cv::KeyPoint.
 * Keypoints nearer the border than their scale's pattern are dropped (as
 * the reference's compute does): kept [n_kept] = their input indices,
 * angle [n_kept] degrees in [0, 360), desc [n_kept][64]. */
int sfm_brisk_describe(int32_t device, const uint8_t* img, int32_t w, int32_t h, const float* kps, int32_t n,
                       int32_t* kept, float* angle, uint8_t* desc, int32_t* n_kept);

/* BRISK detection (+ description): CTracker::detectFeatures
 * (CTracker.cpp:275-287) with BriskFeatureDetector(threshold 60, octaves 6,
 * suppressScaleNonmaxima) -- the published scale-space FAST detector in its
 * reference implementation's form (INTER_AREA layers, FAST non-maximum
 * suppression, refine3D; oracle/brisk_oracle.py), unpinned vs the absent
 * ethz-asl BRISK 2 library.  kps [capacity][5] = (x, y, size, angle,
 * response), octave [capacity] = layer.  desc [capacity][64] or NULL: with
 * NULL, detection only (angle -1, no border removal); otherwise the
 * descriptor's border rule drops keypoints as the reference's compute does.
 * Keypoints come in BRISK's order (layer, then row-major).  *n_out = the
 * count (an error when it exceeds capacity). */
int sfm_brisk_detect_describe(int32_t device, const uint8_t* img, int32_t w, int32_t h, int32_t threshold,
                              int32_t octaves, int32_t capacity, float* kps, int32_t* octave, uint8_t* desc,
                              int32_t* n_out);

/* Per-frame pose: cv::solvePnPRansac(objectPoints, imagePoints, K, dist = 0,
 * rvec, tvec, false, iterations, reproj_err, confidence, inliers,
 * SOLVEPNP_ITERATIVE) as CSfM::tracking calls it (CSfM.cpp:553-565:
 * iterations 20, reproj_err _maxReprErr = 7, confidence 0.99), OpenCV 3.0
 * semantics (oracle/pnp_oracle.py: RANSAC over 5-point EPnP hypotheses with
 * cv::RNG(-1), float32 point data, the best hypothesis's pose and inlier
 * mask returned).  obj [n][3], img [n][2] (undistorted pixels, Kopt), K9
 * row-major (fx, fy, cx, cy read).  Outputs: rvec/tvec (Rodrigues vector,
 * translation), inliers (ascending indices, capacity n; may be NULL),
 * *n_inliers, *found = 0 when no model exists (n < 5, or no hypothesis with
 * more than 4 inliers) -- the reference's `false` return. */
int sfm_pnp_ransac(int32_t device, int32_t n, const double* obj, const double* img, const double* K9,
                   int32_t iterations, double reproj_err, double confidence, double* rvec, double* tvec,
                   int32_t* inliers, int32_t* n_inliers, int32_t* found);

/* Two-view triangulation of new map points (GeometryUtils::triangulatePoints
 * at CSfM.cpp:156 / :918), as cv::triangulatePoints on P = K [R|t]: point i
 * seen at uv0[i] by camera cam0[i] and at uv1[i] by camera cam1[i]; P
 * [n_cams][12] row-major 3x4 projection matrices; X [n][3] out. */
int sfm_triangulate_points(int32_t device, int32_t n, const int32_t* cam0, const int32_t* cam1, const double* uv0,
                           const double* uv1, int32_t n_cams, const double* P, double* X);

/* Testing hook: solve the dense SPD system A y = b (A [n][n] row-major,
 * both triangles given; only the upper triangle is read) with the device
 * Cholesky + substitution kernels used for the reduced camera system.
 * reps > 1 repeats the factorisation for timing; *ms = mean device time per
 * factor+solve; *chol_fail = 1 if a pivot was not positive. */
int sfm_dense_spd_solve(int32_t device, int32_t n, const double* A, const double* b, double* y, int32_t reps,
                        double* ms, int32_t* chol_fail);
/* Measurement plumbing (bench.py, not a reference interface): the best
 * STREAM-copy bandwidth (read + write bytes / s, 16-B accesses) over a few
 * launch shapes, `bytes` per buffer, `reps` timed launches each. */
int sfm_bench_stream_copy(int32_t device, int64_t bytes, int32_t reps, double* best_gbs);
/* Measurement plumbing (tools/dist_factor_model.py): the device work of
 * the distributed factor (sfm_ba_set_distributed_factor) of an n x n system
 * at nranks ranks, each rank's share timed on this one GPU (no collective
 * runs; the broadcasts' bytes are the model's).  Per panel k (np panels):
 * fac_ms[k] its owner's factor, pack_ms[k] the owner's pack of it,
 * unpack_ms[k] a receiver's unpack, upd_ms[r * np + k] rank r's updates of
 * its later panels; misc_ms[5] = reduce-scatter pack, unpack, the back
 * substitution, failure bits, panel-image doubles. */
int sfm_dist_factor_profile(int32_t device, int32_t n, int32_t nranks, int32_t panel_tiles, double* fac_ms,
                            double* pack_ms, double* unpack_ms, double* upd_ms, double* misc_ms);

/* ---- Pyramidal Lucas-Kanade tracker -------------- */
typedef struct sfm_klt_params {
  int32_t win_size;          /* 21   (Size winSize(21,21), CTracker.cpp:484) */
  int32_t max_level;         /* 3    (CTracker.cpp:487) */
  int32_t max_count;         /* 20   (TermCriteria COUNT, CTracker.cpp:483) */
  int32_t reserved;
  double epsilon;            /* 0.03 (TermCriteria EPS; squared internally) */
  double min_eig_threshold;  /* 0.001 (CTracker.cpp:513) */
  double max_match_distance; /* 40  _maxMatchDistance  (CTracker.cpp:30) */
  double min_match_distance; /* 1.5 _minMatchDistance  (CTracker.cpp:31) */
  double max_org_feat_dist;  /* 1   _maxOrgFeatDist    (CTracker.cpp:33) */
} sfm_klt_params;

typedef struct sfm_klt_handle sfm_klt_handle;

void sfm_klt_default_params(sfm_klt_params* p);
/* One tracker per frame size; params NULL = defaults.  win_size odd, 3..31. */
int sfm_klt_create(int32_t device, int32_t width, int32_t height, const sfm_klt_params* params,
                   sfm_klt_handle** out);
int sfm_klt_destroy(sfm_klt_handle* h);
/* Pyramid levels actually built (buildOpticalFlowPyramid stops when a level
 * would not exceed the window): max_level + 1 at most. */
int32_t sfm_klt_num_levels(const sfm_klt_handle* h);
/* Upload a new current frame (grey u8, row stride in bytes) and build its
 * pyramid + Scharr derivatives; the old current frame becomes the previous
 * one (CTracker's _prevFrame/_currFrame swap, CSfM.cpp:626-629). */
int sfm_klt_push_frame(sfm_klt_handle* h, const uint8_t* grey, int32_t stride);
/* Pyramid level `level` of the previous (which=0) or current (which=1)
 * frame: img [h][w] u8 and dxy [h][w][2] int16 (either may be NULL). */
int sfm_klt_get_level(sfm_klt_handle* h, int32_t which, int32_t level, uint8_t* img, int16_t* dxy, int32_t* w,
                      int32_t* hh);
/* cv::calcOpticalFlowPyrLK(prev, curr, prev_pts, next_pts, status, ...)
 * between the two most recent frames; points [n][2] float. */
int sfm_klt_calc_flow(sfm_klt_handle* h, const float* prev_pts, int32_t n, float* next_pts, uint8_t* status);
/* CTracker::computeOpticalFlow: prev_pts_dist [n_prev][2] (previous frame's
 * CFrame::getPointsDistorted), curr_pts_dist [n_curr][2] (current frame's
 * detected points).  Writes *n_matches (prev_idx, curr_idx) pairs in the
 * reference's slot order (capacity >= n_prev); flowed [n_prev][2] and
 * status [n_prev] are optional outputs of the LK stage.  The reference's
 * bool is (*n_matches >= _minFeatures). */
int sfm_klt_compute_optical_flow(sfm_klt_handle* h, const double* prev_pts_dist, int32_t n_prev,
                                 const double* curr_pts_dist, int32_t n_curr, int32_t* prev_idx, int32_t* curr_idx,
                                 int32_t* n_matches, float* flowed, uint8_t* status);
/* Device time (ms) of the last push (pyramid), LK and association stages. */
int sfm_klt_phase_times(sfm_klt_handle* h, double* ms3);
/* One-shot calcOpticalFlowPyrLK on two host frames (creates a temporary tracker). */
int sfm_calc_optical_flow_pyr_lk(int32_t device, const uint8_t* prev, const uint8_t* next, int32_t width,
                                 int32_t height, const float* prev_pts, int32_t n, float* next_pts, uint8_t* status,
                                 const sfm_klt_params* params);

/* ---- Corner detector of the optical-flow tracker ---
 * CTracker::detectFeaturesOpticalFlow (CTracker.cpp:252-272):
 * goodFeaturesToTrack(grey, pts, 500, 0.05, 10) + cornerSubPix(grey, pts,
 * Size(5,5), Size(-1,-1), TermCriteria(COUNT|EPS, 20, 0.03)). */
typedef struct sfm_gftt_params {
  int32_t max_corners;     /* 500  maxFeats      (CTracker.cpp:253) */
  int32_t subpix_win;      /* 5    subPixWinSize (CTracker.cpp:257), 1..7; 0 = no cornerSubPix */
  int32_t subpix_max_iter; /* 20   TermCriteria COUNT (CTracker.cpp:256) */
  int32_t min_features;    /* 5    _minFeatures  (CTracker.cpp:32): the reference's bool is n >= this */
  double quality_level;    /* 0.05 qualityLvl    (CTracker.cpp:254) */
  double min_distance;     /* 10   minDistance   (CTracker.cpp:255) */
  double subpix_epsilon;   /* 0.03 TermCriteria EPS (CTracker.cpp:256) */
} sfm_gftt_params;
void sfm_gftt_default_params(sfm_gftt_params* p);
/* CTracker::detectFeatures (CTracker.cpp:275-287) on the handle's current
 * frame (the one sfm_klt_push_frame uploaded): the same BRISK detector and
 * descriptor as sfm_brisk_detect_describe, with no second upload of the
 * image -- one upload per frame serves the KLT pyramid, the corner detector
 * and BRISK.  Outputs and errors as sfm_brisk_detect_describe. */
int sfm_klt_brisk_detect_describe(sfm_klt_handle* h, int32_t threshold, int32_t octaves, int32_t capacity,
                                  float* kps, int32_t* octave, uint8_t* desc, int32_t* n_out);

/* Corners of the handle's current frame (after sfm_klt_push_frame), in the
 * reference's order (response descending), refined to subpixel; pts
 * [capacity][2] float, capacity >= max_corners (<= 4096). */
int sfm_klt_detect_features(sfm_klt_handle* h, const sfm_gftt_params* params, float* pts, int32_t capacity,
                            int32_t* n_pts);
/* Device time (ms) of the last sfm_klt_detect_features. */
int sfm_klt_detect_time(sfm_klt_handle* h, double* ms);
/* One-shot form on a host frame (temporary handle). */
int sfm_good_features_to_track(int32_t device, const uint8_t* grey, int32_t width, int32_t height, int32_t stride,
                               const sfm_gftt_params* params, float* pts, int32_t capacity, int32_t* n_pts);

/* Synthetic scenes, host-only.  Points [p_begin, p_end) of a
 * scene with n_pts_total points; every camera is returned.  Observations are
 * sorted by (point, camera); pt_idx is relative to p_begin.
 * n_obs = (p_end - p_begin) * views.  NULL *_true / *_init pointers allowed. */
void sfm_scene_default_intrinsics(double K9[9]);
int sfm_scene_generate(int32_t n_cams, int32_t n_pts_total, int32_t p_begin, int32_t p_end, int32_t views,
                       uint64_t seed, double pixel_sigma, double pt_sigma, double rot_sigma, double t_sigma,
                       double* K9, double* rot_true, double* t_true, double* X_true, double* rot_init,
                       double* t_init, double* X_init, double* obs_uv, int32_t* cam_idx, int32_t* pt_idx);

#ifdef __cplusplus
}
#endif
#endif /* SFM_AMD_H_ */
