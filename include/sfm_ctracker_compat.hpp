// sfm_ctracker_compat.hpp -- header-only C++ shim that gives the reference's
// CTracker hot-path signatures on top of the plain C ABI of sfm_amd.h.
//
// A maintainer swaps the Ceres body of
//   void CTracker::bundleAdjustmentStructAndPose(const vector<Point2d>&,
//       const vector<int>&, const vector<Matx33d>&, vector<double*>& R,
//       vector<double*>& t, vector<double*>& pts3D, int isStructOrPose)
//   (/root/reference/CTracker.h:65, CTracker.cpp:670-702)
// for a call to sfm_compat::bundleAdjustmentStructAndPose(...) with the same
// arguments.  The shim
//   1. deduplicates the per-observation point pointers into pt_idx in
//      first-seen order (the reference identifies Ceres parameter blocks by
//      address, CSfM.cpp:321-340),
//   2. packs the structure-of-arrays the ABI takes,
//   3. calls sfm_ba_solve,
//   4. scatters the solution back through the caller's pointers, exactly
//      where Ceres would have written it.
// Cameras are identified by camIdx (index into R / t / K), as in the
// reference.  On an error nothing is written back and the ABI code is
// returned (the reference has no error channel; callers may ignore it).
//
// Types are templates so the header does not depend on OpenCV: Point2 needs
// .x/.y, Matx33 needs .val[9] (row-major, cv::Matx33d layout), the
// descriptor matrix needs .rows / .cols / .data (cv::Mat of CV_8U).
#ifndef SFM_CTRACKER_COMPAT_HPP_
#define SFM_CTRACKER_COMPAT_HPP_

#include <algorithm>
#include <cstdint>
#include <unordered_map>
#include <vector>

#include "sfm_amd.h"

namespace sfm_compat {

// Packed form of one BA problem (what sfm_ba_solve consumes).
struct PackedProblem {
  std::vector<double> uv, K9, rot, t, X;
  std::vector<int32_t> cam_idx, pt_idx;
  std::vector<double*> point_ptr;  // distinct point blocks, first-seen order
};

template <class Point2, class Matx33>
inline int pack_problem(const std::vector<Point2>& observations, const std::vector<int>& camIdx,
                        const std::vector<Matx33>& K, const std::vector<double*>& R, const std::vector<double*>& t,
                        const std::vector<double*>& pts3D, PackedProblem* out) {
  const size_t n = observations.size();
  if (camIdx.size() != n || pts3D.size() != n || R.size() != t.size() || K.size() < R.size()) return SFM_EINVAL;
  PackedProblem& p = *out;
  p.uv.resize(2 * n);
  p.cam_idx.resize(n);
  p.pt_idx.resize(n);
  p.point_ptr.clear();
  std::unordered_map<const double*, int32_t> id;
  id.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    p.uv[2 * i] = observations[i].x;
    p.uv[2 * i + 1] = observations[i].y;
    if (camIdx[i] < 0 || size_t(camIdx[i]) >= R.size()) return SFM_EINVAL;
    p.cam_idx[i] = camIdx[i];
    auto it = id.find(pts3D[i]);
    if (it == id.end()) {
      it = id.emplace(pts3D[i], int32_t(p.point_ptr.size())).first;
      p.point_ptr.push_back(pts3D[i]);
    }
    p.pt_idx[i] = it->second;
  }
  const size_t C = R.size(), P = p.point_ptr.size();
  p.K9.resize(9 * C);
  p.rot.resize(3 * C);
  p.t.resize(3 * C);
  for (size_t c = 0; c < C; ++c) {
    for (int k = 0; k < 9; ++k) p.K9[9 * c + k] = K[c].val[k];
    for (int k = 0; k < 3; ++k) {
      p.rot[3 * c + k] = R[c][k];
      p.t[3 * c + k] = t[c][k];
    }
  }
  p.X.resize(3 * P);
  for (size_t q = 0; q < P; ++q)
    for (int k = 0; k < 3; ++k) p.X[3 * q + k] = p.point_ptr[q][k];
  return SFM_OK;
}

// Drop-in for CTracker::bundleAdjustmentStructAndPose (CTracker.cpp:670-702).
// opts == nullptr: the reference's options (DENSE_SCHUR, Ceres defaults,
// CTracker.cpp:571-577).  summary (optional) receives what Ceres' Summary
// would have said; the reference discards it (CTracker.cpp:700-701).
template <class Point2, class Matx33>
inline int bundleAdjustmentStructAndPose(const std::vector<Point2>& observations, const std::vector<int>& camIdx,
                                         const std::vector<Matx33>& K, std::vector<double*>& R,
                                         std::vector<double*>& t, std::vector<double*>& pts3D, int isStructOrPose,
                                         const sfm_ba_options* opts = nullptr, sfm_ba_summary* summary = nullptr) {
  PackedProblem p;
  int rc = pack_problem(observations, camIdx, K, R, t, pts3D, &p);
  if (rc) return rc;
  sfm_ba_options o;
  if (opts) o = *opts; else sfm_ba_default_options(&o);
  sfm_ba_summary sm;
  rc = sfm_ba_solve(&o, isStructOrPose, int64_t(observations.size()), p.uv.data(), p.cam_idx.data(),
                    p.pt_idx.data(), int32_t(R.size()), p.K9.data(), p.rot.data(), p.t.data(),
                    int32_t(p.point_ptr.size()), p.X.data(), &sm, nullptr, 0, nullptr);
  if (rc) return rc;
  for (size_t c = 0; c < R.size(); ++c)
    for (int k = 0; k < 3; ++k) {
      R[c][k] = p.rot[3 * c + k];
      t[c][k] = p.t[3 * c + k];
    }
  for (size_t q = 0; q < p.point_ptr.size(); ++q)
    for (int k = 0; k < 3; ++k) p.point_ptr[q][k] = p.X[3 * q + k];
  if (summary) *summary = sm;
  return SFM_OK;
}

// Drop-in for CTracker::matchFeatures(pts0, desc0, pts1, desc1, idx0, idx1,
// minDistance, maxDistance) (CTracker.h:55, CTracker.cpp:211-250); with
// (1.5, 40) it is the member-window overload (CTracker.h:53,
// CTracker.cpp:114-149).  Like the reference it APPENDS the matches to
// matchIdx0 / matchIdx1 (push_back, CTracker.cpp:238-239) and returns
// nothing useful: the int is the ABI code (0 on success).
template <class Point2, class DescMat>
inline int matchFeatures(const std::vector<Point2>& pts0, const DescMat& desc0, const std::vector<Point2>& pts1,
                         const DescMat& desc1, std::vector<int>& matchIdx0, std::vector<int>& matchIdx1,
                         double minDistance = 1.5, double maxDistance = 40.0, int32_t device = 0,
                         double ratio = 0.8) {
  const int32_t n0 = int32_t(pts0.size()), n1 = int32_t(pts1.size());
  std::vector<double> p0(2 * size_t(n0)), p1(2 * size_t(n1));
  for (int32_t i = 0; i < n0; ++i) { p0[2 * i] = pts0[i].x; p0[2 * i + 1] = pts0[i].y; }
  for (int32_t i = 0; i < n1; ++i) { p1[2 * i] = pts1[i].x; p1[2 * i + 1] = pts1[i].y; }
  const int32_t cap = n0 < n1 ? n0 : n1;
  std::vector<int32_t> i0(size_t(cap > 0 ? cap : 0)), i1(size_t(cap > 0 ? cap : 0));
  int32_t nm = 0;
  const int rc = sfm_match_features(device, p0.data(), static_cast<const uint8_t*>(desc0.data), n0, p1.data(),
                                    static_cast<const uint8_t*>(desc1.data), n1, int32_t(desc0.cols), ratio,
                                    minDistance, maxDistance, i0.data(), i1.data(), &nm);
  if (rc) return rc;
  matchIdx0.insert(matchIdx0.end(), i0.begin(), i0.begin() + nm);
  matchIdx1.insert(matchIdx1.end(), i1.begin(), i1.begin() + nm);
  return SFM_OK;
}

// Per-frame pose, the cv::solvePnPRansac call of CSfM::tracking
// (/root/reference/CSfM.cpp:553-565):
//   solvePnPRansac(currMatch3D, currMatch2D, K, Mat::zeros(4,1,CV_64FC1), rvec, tvec,
//                  false, iter = 20, _maxReprErr = 7, 0.99, inlierIdx, SOLVEPNP_ITERATIVE)
// becomes
//   sfm_compat::solvePnPRansac(currMatch3D, currMatch2D, K, rvec3, tvec3, inlierIdx, 20, 7.0, 0.99)
// with Point3 = anything with .val[3] (cv::Matx31d) or .x/.y/.z via the
// overload below, Point2 .x/.y, Matx33 .val[9]; rvec3 / tvec3 are double[3]
// (cv::Mat(3,1,CV_64F, ptr) wraps them).  Returns true when a model was
// found (the reference's bool), false otherwise (inliers cleared); ABI
// errors also return false, with sfm_last_error() set.
template <class Point3, class Point2, class Matx33>
inline bool solvePnPRansac(const std::vector<Point3>& objectPoints, const std::vector<Point2>& imagePoints,
                           const Matx33& K, double rvec[3], double tvec[3], std::vector<int>& inliers,
                           int iterationsCount = 20, double reprojectionError = 7.0, double confidence = 0.99,
                           int device = 0) {
  inliers.clear();
  const size_t n = objectPoints.size();
  if (imagePoints.size() != n) return false;
  std::vector<double> obj(3 * n), img(2 * n);
  for (size_t i = 0; i < n; ++i) {
    for (int m = 0; m < 3; ++m) obj[3 * i + m] = objectPoints[i].val[m];
    img[2 * i] = imagePoints[i].x;
    img[2 * i + 1] = imagePoints[i].y;
  }
  double K9[9];
  for (int m = 0; m < 9; ++m) K9[m] = K.val[m];
  std::vector<int32_t> inl(std::max<size_t>(1, n));
  int32_t n_inl = 0, found = 0;
  if (sfm_pnp_ransac(device, int32_t(n), obj.data(), img.data(), K9, iterationsCount, reprojectionError, confidence,
                     rvec, tvec, inl.data(), &n_inl, &found) != 0)
    return false;
  inliers.assign(inl.begin(), inl.begin() + n_inl);
  return found != 0;
}

// Frame-resident matcher: drop-ins for the per-frame matchFeatures
// overloads.  CTracker keeps _prevFrame / _currFrame (CTracker.h:80-81); the
// shim keeps the same two frames' keypoints + descriptors resident on the
// device.  After CFrame::setKeyPoints of a new frame (CTracker.cpp:275-287):
//   matcher.pushFrame(frame.getPoints(), frame.getPointsDistorted(), frame.getDescriptors());
// then, in place of the reference's bodies,
//   _tracker.matchFeatures(prev2DIdx, curr2DIdx, prevMatch2DIdx, currMatch2DIdx);   (CSfM.cpp:518)
//     -> matcher.matchFeatures(prev2DIdx, curr2DIdx, prevMatch2DIdx, currMatch2DIdx);
//   bool ok = _tracker.matchFeatures();                                                (CSfM.cpp:823)
//     -> bool ok = matcher.matchFeatures(_prevIdx, _currIdx, _minFeatures);
// (the _prevMatch/_currMatch point lists stay the caller's getPointsAt
// gathers, CTracker.cpp:470-471).  Point2 needs .x/.y; DescMat .rows /
// .cols / .data (cv::Mat of CV_8U, continuous).
class FeatureMatcher {
 public:
  explicit FeatureMatcher(int32_t descBytes = 64, int32_t device = 0, double ratioTest = 0.8,
                          double minMatchDistance = 1.5, double maxMatchDistance = 40.0)
      : ratio_(ratioTest), min_(minMatchDistance), max_(maxMatchDistance) {
    rc_ = sfm_matcher_create(device, descBytes, &h_);
  }
  ~FeatureMatcher() {
    if (h_) sfm_matcher_destroy(h_);
  }
  FeatureMatcher(const FeatureMatcher&) = delete;
  FeatureMatcher& operator=(const FeatureMatcher&) = delete;
  int status() const { return rc_; }

  // The new current frame (the previous current frame becomes the previous one).
  template <class Point2, class DescMat>
  int pushFrame(const std::vector<Point2>& pts, const std::vector<Point2>& ptsDistorted, const DescMat& desc) {
    if (!h_) return rc_;
    const int32_t n = int32_t(pts.size());
    if (int32_t(ptsDistorted.size()) != n || int32_t(desc.rows) != n) return SFM_EINVAL;
    std::vector<double> p(2 * size_t(n)), d(2 * size_t(n));
    for (int32_t i = 0; i < n; ++i) {
      p[2 * i] = pts[i].x; p[2 * i + 1] = pts[i].y;
      d[2 * i] = ptsDistorted[i].x; d[2 * i + 1] = ptsDistorted[i].y;
    }
    n_[0] = n_[1];
    n_[1] = n;
    return sfm_matcher_push_frame(h_, p.data(), d.data(), static_cast<const uint8_t*>(desc.data), n);
  }

  // void CTracker::matchFeatures(const vector<int>& prevFrameIdx, const
  // vector<int>& currFrameIdx, vector<int>& prevMatchIdx, vector<int>&
  // currMatchIdx) (CTracker.h:57, CTracker.cpp:368-417): appends
  // frame-global indices (push_back, :406-407).  Returns the ABI code.
  int matchFeatures(const std::vector<int>& prevFrameIdx, const std::vector<int>& currFrameIdx,
                    std::vector<int>& prevMatchIdx, std::vector<int>& currMatchIdx) {
    if (!h_) return rc_;
    const size_t cap = std::max<size_t>(1, std::min(prevFrameIdx.size(), currFrameIdx.size()));
    std::vector<int32_t> a(cap), b(cap);
    int32_t nm = 0;
    const int rc = sfm_matcher_match_subset(h_, prevFrameIdx.data(), int32_t(prevFrameIdx.size()),
                                            currFrameIdx.data(), int32_t(currFrameIdx.size()), ratio_, min_, max_,
                                            a.data(), b.data(), &nm);
    if (rc) return rc;
    prevMatchIdx.insert(prevMatchIdx.end(), a.begin(), a.begin() + nm);
    currMatchIdx.insert(currMatchIdx.end(), b.begin(), b.begin() + nm);
    return SFM_OK;
  }

  // bool CTracker::matchFeatures() (CTracker.h:59, CTracker.cpp:419-477):
  // clears and fills _prevIdx / _currIdx from the two whole frames on their
  // distorted positions; returns matchCount >= minFeatures.
  bool matchFeatures(std::vector<int>& prevIdx, std::vector<int>& currIdx, int minFeatures = 5,
                     int* rc_out = nullptr) {
    prevIdx.clear();
    currIdx.clear();
    int rc = rc_;
    if (h_) {
      const size_t cap = std::max<size_t>(1, size_t(std::min(n_[0], n_[1])));
      std::vector<int32_t> a(cap), b(cap);
      int32_t nm = 0;
      rc = sfm_matcher_match_frames(h_, 1, ratio_, min_, max_, a.data(), b.data(), &nm);
      if (rc == SFM_OK) {
        prevIdx.assign(a.begin(), a.begin() + nm);
        currIdx.assign(b.begin(), b.begin() + nm);
      }
    }
    if (rc_out) *rc_out = rc;
    return rc == SFM_OK && int(prevIdx.size()) >= minFeatures;
  }

  // The (pts0, desc0, pts1, desc1, idx0, idx1[, minDistance, maxDistance])
  // overloads (CTracker.cpp:114-149, 211-250) through the pooled handle.
  template <class Point2, class DescMat>
  int matchFeatures(const std::vector<Point2>& pts0, const DescMat& desc0, const std::vector<Point2>& pts1,
                    const DescMat& desc1, std::vector<int>& matchIdx0, std::vector<int>& matchIdx1,
                    double minDistance, double maxDistance) {
    if (!h_) return rc_;
    const int32_t n0 = int32_t(pts0.size()), n1 = int32_t(pts1.size());
    std::vector<double> p0(2 * size_t(n0)), p1(2 * size_t(n1));
    for (int32_t i = 0; i < n0; ++i) { p0[2 * i] = pts0[i].x; p0[2 * i + 1] = pts0[i].y; }
    for (int32_t i = 0; i < n1; ++i) { p1[2 * i] = pts1[i].x; p1[2 * i + 1] = pts1[i].y; }
    const size_t cap = std::max<size_t>(1, size_t(std::min(n0, n1)));
    std::vector<int32_t> a(cap), b(cap);
    int32_t nm = 0;
    const int rc = sfm_matcher_match(h_, p0.data(), static_cast<const uint8_t*>(desc0.data), n0, p1.data(),
                                     static_cast<const uint8_t*>(desc1.data), n1, ratio_, minDistance, maxDistance,
                                     a.data(), b.data(), &nm);
    if (rc) return rc;
    matchIdx0.insert(matchIdx0.end(), a.begin(), a.begin() + nm);
    matchIdx1.insert(matchIdx1.end(), b.begin(), b.begin() + nm);
    return SFM_OK;
  }
  template <class Point2, class DescMat>
  int matchFeatures(const std::vector<Point2>& pts0, const DescMat& desc0, const std::vector<Point2>& pts1,
                    const DescMat& desc1, std::vector<int>& matchIdx0, std::vector<int>& matchIdx1) {
    return matchFeatures(pts0, desc0, pts1, desc1, matchIdx0, matchIdx1, min_, max_);
  }

  sfm_matcher* handle() const { return h_; }

 private:
  sfm_matcher* h_ = nullptr;
  int rc_ = SFM_OK;
  double ratio_, min_, max_;
  int32_t n_[2] = {0, 0};
};

// sfm_brisk_detect_describe's packed output -> cv::KeyPoint-like objects
template <class KeyPoint>
inline void unpack_keypoints(const std::vector<float>& k, const std::vector<int32_t>& oct,
                             const std::vector<uint8_t>& d, int32_t n, std::vector<KeyPoint>& keypoints,
                             std::vector<uint8_t>& descriptors) {
  keypoints.resize(size_t(n));
  for (int32_t i = 0; i < n; ++i) {
    keypoints[i].pt.x = k[5 * size_t(i)];
    keypoints[i].pt.y = k[5 * size_t(i) + 1];
    keypoints[i].size = k[5 * size_t(i) + 2];
    keypoints[i].angle = k[5 * size_t(i) + 3];
    keypoints[i].response = k[5 * size_t(i) + 4];
    keypoints[i].octave = oct[i];
  }
  descriptors.assign(d.begin(), d.begin() + 64 * size_t(n));
}

// Drop-in for CTracker::computeOpticalFlow (CTracker.h:60,
// CTracker.cpp:480-562).  The reference reads its member frames
// (_prevFrame/_currFrame: getFrameGrey(), getPointsDistorted()) and fills
// _prevIdx/_currIdx; the shim keeps the two frames' pyramids resident on
// the device (one push per frame, the previous current frame becomes the
// previous one, like the _prevFrame = _currFrame swap, CSfM.cpp:626-629).
//   OpticalFlowTracker flow(width, height);       // once per frame size
//   flow.pushFrame(_currFrame.getFrameGrey());    // every new frame
//   bool ok = flow.computeOpticalFlow(_prevFrame.getPointsDistorted(),
//                                     _currFrame.getPointsDistorted(),
//                                     _prevIdx, _currIdx, _minFeatures);
// GreyMat needs .data (uint8), .step (row bytes, cv::Mat's MatStep converts),
// .cols, .rows; Point2 needs .x/.y.  Like the reference, the index vectors
// are cleared first and the result is matchCount >= minFeatures.  The
// _prevMatch/_currMatch point lists are the caller's getPointsAt gathers
// (CTracker.cpp:548-549), unchanged.
class OpticalFlowTracker {
 public:
  OpticalFlowTracker(int32_t width, int32_t height, int32_t device = 0, const sfm_klt_params* params = nullptr) {
    rc_ = sfm_klt_create(device, width, height, params, &h_);
  }
  ~OpticalFlowTracker() {
    if (h_) sfm_klt_destroy(h_);
  }
  OpticalFlowTracker(const OpticalFlowTracker&) = delete;
  OpticalFlowTracker& operator=(const OpticalFlowTracker&) = delete;
  int status() const { return rc_; }

  template <class GreyMat>
  int pushFrame(const GreyMat& grey) {
    if (!h_) return rc_;
    return sfm_klt_push_frame(h_, static_cast<const uint8_t*>(grey.data), int32_t(static_cast<size_t>(grey.step)));
  }

  // Drop-in for CTracker::detectFeaturesOpticalFlow (CTracker.h:48,
  // CTracker.cpp:252-272) on the frame pushed last: goodFeaturesToTrack
  // (500, 0.05, 10) + cornerSubPix (5x5, 20, 0.03); `pts` receives the
  // refined corners in the reference's order (what it hands to
  // CFrame::setPoints); returns pts.size() >= minFeatures.
  //   bool CTracker::detectFeaturesOpticalFlow() {
  //     std::vector<cv::Point2f> pts;
  //     if (!_flow.detectFeaturesOpticalFlow(pts, _minFeatures)) return false;
  //     _currFrame.setPoints(pts);
  //     return true;
  //   }
  template <class Point2f>
  bool detectFeaturesOpticalFlow(std::vector<Point2f>& pts, int minFeatures = 5,
                                 const sfm_gftt_params* params = nullptr, int* rc_out = nullptr) {
    pts.clear();
    int rc = rc_;
    if (h_) {
      sfm_gftt_params p;
      if (params) p = *params;
      else sfm_gftt_default_params(&p);
      std::vector<float> buf(2 * size_t(p.max_corners > 0 ? p.max_corners : 1));
      int32_t n = 0;
      rc = sfm_klt_detect_features(h_, &p, buf.data(), p.max_corners, &n);
      if (rc == SFM_OK) {
        pts.resize(size_t(n));
        for (int32_t i = 0; i < n; ++i) {
          pts[i].x = buf[2 * i];
          pts[i].y = buf[2 * i + 1];
        }
      }
    }
    if (rc_out) *rc_out = rc;
    return rc == SFM_OK && int(pts.size()) >= minFeatures;
  }

  // CTracker::detectFeatures (CTracker.cpp:275-287) on the frame pushed
  // last, without a second upload (sfm_klt_brisk_detect_describe): the same
  // outputs as sfm_compat::detectFeatures(grey, ...) below.
  template <class KeyPoint>
  int detectFeaturesBrisk(std::vector<KeyPoint>& keypoints, std::vector<uint8_t>& descriptors, int threshold = 60,
                          int octaves = 6, int32_t capacity = 20000) {
    keypoints.clear();
    descriptors.clear();
    if (!h_) return rc_;
    std::vector<float> k;
    std::vector<int32_t> oct;
    std::vector<uint8_t> d;
    int32_t n = 0;
    // the call reports the count before it rejects a short buffer: one retry
    // at that size, so a frame with more keypoints never fails (the
    // reference's detectFeatures has no cap)
    int rc = SFM_OK;
    for (int attempt = 0; attempt < 2; ++attempt) {
      k.assign(5 * size_t(capacity), 0.0f);
      oct.assign(size_t(capacity), 0);
      d.assign(64 * size_t(capacity), 0);
      rc = sfm_klt_brisk_detect_describe(h_, threshold, octaves, capacity, k.data(), oct.data(), d.data(), &n);
      if (rc == SFM_OK || n <= capacity) break;
      capacity = n;
    }
    if (rc) return rc;
    unpack_keypoints(k, oct, d, n, keypoints, descriptors);
    return SFM_OK;
  }

  template <class Point2>
  bool computeOpticalFlow(const std::vector<Point2>& prevPtsDistorted, const std::vector<Point2>& currPtsDistorted,
                          std::vector<int>& prevIdx, std::vector<int>& currIdx, int minFeatures = 5,
                          int* rc_out = nullptr) {
    prevIdx.clear();
    currIdx.clear();
    int rc = rc_;
    if (h_) {
      const int32_t n = int32_t(prevPtsDistorted.size()), m = int32_t(currPtsDistorted.size());
      std::vector<double> p(2 * size_t(n)), c(2 * size_t(m));
      for (int32_t i = 0; i < n; ++i) { p[2 * i] = prevPtsDistorted[i].x; p[2 * i + 1] = prevPtsDistorted[i].y; }
      for (int32_t i = 0; i < m; ++i) { c[2 * i] = currPtsDistorted[i].x; c[2 * i + 1] = currPtsDistorted[i].y; }
      std::vector<int32_t> pi(size_t(n > 0 ? n : 1)), ci(size_t(n > 0 ? n : 1));
      int32_t nm = 0;
      rc = sfm_klt_compute_optical_flow(h_, p.data(), n, c.data(), m, pi.data(), ci.data(), &nm, nullptr, nullptr);
      if (rc == SFM_OK) {
        prevIdx.assign(pi.begin(), pi.begin() + nm);
        currIdx.assign(ci.begin(), ci.begin() + nm);
      }
    }
    if (rc_out) *rc_out = rc;
    return rc == SFM_OK && int(prevIdx.size()) >= minFeatures;
  }

 private:
  sfm_klt_handle* h_ = nullptr;
  int rc_ = SFM_OK;
};

// Drop-in for the body of CTracker::detectFeatures (CTracker.h:47,
// CTracker.cpp:275-287): _detector->detect + _descriptor->compute with
// BriskFeatureDetector(60, 6, true) (CTracker.cpp:43-45) on the current
// frame's grey image, then CFrame::setKeyPoints with the survivors:
//   bool CTracker::detectFeatures() {
//     std::vector<cv::KeyPoint> kp; cv::Mat desc;
//     std::vector<uint8_t> d;
//     if (sfm_compat::detectFeatures(_currFrame.getFrameGrey(), kp, d)) return false;
//     desc = cv::Mat(int(kp.size()), 64, CV_8U, d.data()).clone();
//     _currFrame.setKeyPoints(kp, desc);             // unchanged (CTracker.cpp:286)
//     return true;
//   }
// GreyMat: .data (uint8), .step (row bytes), .cols, .rows; KeyPoint:
// cv::KeyPoint's public fields (.pt.x, .pt.y, .size, .angle, .response,
// .octave).  Keypoints come in BRISK's order with the descriptor's border
// rule applied, as compute() leaves them; `descriptors` receives
// [kp.size()][64] bytes.  Returns the ABI code (0 on success).  Parity is
// with BRISK as published (oracle/brisk_oracle.py); the ethz-asl BRISK 2
// library the reference links is absent, so parity with it is unpinned.
template <class GreyMat, class KeyPoint>
inline int detectFeatures(const GreyMat& grey, std::vector<KeyPoint>& keypoints, std::vector<uint8_t>& descriptors,
                          int threshold = 60, int octaves = 6, int32_t capacity = 20000, int32_t device = 0) {
  keypoints.clear();
  descriptors.clear();
  const int32_t w = int32_t(grey.cols), h = int32_t(grey.rows);
  const size_t step = static_cast<size_t>(grey.step);
  const uint8_t* img = static_cast<const uint8_t*>(grey.data);
  std::vector<uint8_t> packed;
  if (step != size_t(w)) {  // the ABI takes a continuous [h][w] image
    packed.resize(size_t(w) * size_t(h));
    for (int32_t y = 0; y < h; ++y)
      std::copy(img + size_t(y) * step, img + size_t(y) * step + size_t(w), packed.begin() + size_t(y) * size_t(w));
    img = packed.data();
  }
  std::vector<float> k;
  std::vector<int32_t> oct;
  std::vector<uint8_t> d;
  int32_t n = 0;
  int rc = SFM_OK;
  for (int attempt = 0; attempt < 2; ++attempt) {  // one retry at the reported count
    k.assign(5 * size_t(capacity), 0.0f);
    oct.assign(size_t(capacity), 0);
    d.assign(64 * size_t(capacity), 0);
    rc = sfm_brisk_detect_describe(device, img, w, h, threshold, octaves, capacity, k.data(), oct.data(), d.data(),
                                   &n);
    if (rc == SFM_OK || n <= capacity) break;
    capacity = n;
  }
  if (rc) return rc;
  unpack_keypoints(k, oct, d, n, keypoints, descriptors);
  return SFM_OK;
}

// CMap's observation store on the device (CMap.h:36-99, CMap.cpp), for the
// CMap methods the tracking and BA paths call.  CMap keeps its host members
// (_pts3D and the rest); this object replaces the two multimaps, the
// per-point _frameNo / _pts2DIdx lists and the _descriptor rows
// (INTEGRATION.md §4f).  Point indices are CMap's _lastPtNo numbering.
// Every method returns the ABI code (0 on success); the output vectors are
// APPENDED to, as the reference's push_back loops do.
class MapStore {
 public:
  explicit MapStore(int32_t descBytes = 64, int32_t device = 0) : desc_bytes_(descBytes) {
    rc_ = sfm_map_create(device, descBytes, &h_);
  }
  ~MapStore() {
    if (h_) sfm_map_destroy(h_);
  }
  MapStore(const MapStore&) = delete;
  MapStore& operator=(const MapStore&) = delete;
  int status() const { return rc_; }
  sfm_map* handle() const { return h_; }

  // CMap::getNPoints (CMap.cpp:114-116)
  int getNPoints() const {
    int32_t np = 0;
    int64_t no = 0, nd = 0;
    return h_ && sfm_map_size(h_, &np, &no, &nd) == SFM_OK ? int(np) : 0;
  }

  // CMap::addNewPoints (CMap.cpp:36-78): pts2DIdx[j][i] = frame j's 2D
  // index of new point i; pts3DIdx receives the new indices.  Matx31 needs
  // .val[3] (cv::Matx31d).
  template <class Matx31>
  int addNewPoints(const std::vector<Matx31>& pts3D, const std::vector<std::vector<int>>& pts2DIdx,
                   const std::vector<int>& frameNo, std::vector<int>& pts3DIdx) {
    if (!h_) return rc_;
    const size_t n = pts3D.size(), nf = frameNo.size();
    if (pts2DIdx.size() != nf) return SFM_EINVAL;
    std::vector<double> X(3 * n);
    for (size_t i = 0; i < n; ++i)
      for (int m = 0; m < 3; ++m) X[3 * i + m] = pts3D[i].val[m];
    std::vector<int32_t> flat(nf * n);
    for (size_t j = 0; j < nf; ++j) {
      if (pts2DIdx[j].size() < n) return SFM_EINVAL;
      std::copy(pts2DIdx[j].begin(), pts2DIdx[j].begin() + n, flat.begin() + j * n);
    }
    std::vector<int32_t> idx(std::max<size_t>(1, n));
    const int rc = sfm_map_add_new_points(h_, int32_t(n), n ? X.data() : nullptr, int32_t(nf), frameNo.data(),
                                          flat.data(), idx.data());
    if (rc) return rc;
    pts3DIdx.insert(pts3DIdx.end(), idx.begin(), idx.begin() + n);
    return SFM_OK;
  }

  // CMap::addPointMatches (CMap.cpp:118-132)
  int addPointMatches(const std::vector<int>& pts3DIdx, const std::vector<int>& pts2DIdx, int frameNo) {
    if (!h_) return rc_;
    if (pts2DIdx.size() < pts3DIdx.size()) return SFM_EINVAL;
    return sfm_map_add_point_matches(h_, int32_t(pts3DIdx.size()), pts3DIdx.data(), pts2DIdx.data(), frameNo);
  }

  // CMap::addDescriptors (CMap.cpp:308-315): row i of `descriptors` (.rows,
  // .cols = descBytes, .data; cv::Mat CV_8U, continuous) to point pts3DIdx[i].
  template <class DescMat>
  int addDescriptors(const std::vector<int>& pts3DIdx, const DescMat& descriptors) {
    if (!h_) return rc_;
    if (size_t(descriptors.rows) < pts3DIdx.size() || int32_t(descriptors.cols) != desc_bytes_) return SFM_EINVAL;
    return sfm_map_add_descriptors(h_, int32_t(pts3DIdx.size()), pts3DIdx.data(),
                                   static_cast<const uint8_t*>(descriptors.data));
  }

  // CMap::getPointsInFrames(pts3DIdx, frameNo) (CMap.cpp:270-288): appends
  // the points seen in any of the frames, then the reference's sort + unique
  // over the whole vector.
  int getPointsInFrames(std::vector<int>& pts3DIdx, const std::vector<int>& frameNo) {
    if (!h_) return rc_;
    std::vector<int32_t> out(std::max(1, getNPoints()));
    int32_t n = 0;
    const int rc = sfm_map_points_in_frames(h_, int32_t(frameNo.size()), frameNo.data(), int32_t(out.size()),
                                            out.data(), &n);
    if (rc) return rc;
    pts3DIdx.insert(pts3DIdx.end(), out.begin(), out.begin() + n);
    std::sort(pts3DIdx.begin(), pts3DIdx.end());
    pts3DIdx.erase(std::unique(pts3DIdx.begin(), pts3DIdx.end()), pts3DIdx.end());
    return SFM_OK;
  }

  // CMap::getPointsInFrame(pts3DIdx, pts2DIdx, frameNo) (CMap.cpp:225-240):
  // per equal_range entry its point, then every 2D index the point has in
  // that frame (a point matched k times in the frame gives k entries with k
  // 2D indices each).
  int getPointsInFrame(std::vector<int>& pts3DIdx, std::vector<int>& pts2DIdx, int frameNo) {
    if (!h_) return rc_;
    int32_t np = 0;
    int64_t no = 0, nd = 0;
    if (int rc = sfm_map_size(h_, &np, &no, &nd)) return rc;
    int32_t cap = int32_t(std::max<int64_t>(1, no));
    for (int attempt = 0; attempt < 2; ++attempt) {  // the 2D list can outgrow n_obs: retry at the reported size
      std::vector<int32_t> a(static_cast<size_t>(cap)), b(static_cast<size_t>(cap));
      int32_t n3 = 0, n2 = 0;
      const int rc = sfm_map_points_in_frame(h_, frameNo, cap, a.data(), &n3, b.data(), &n2);
      if (rc == SFM_OK) {
        pts3DIdx.insert(pts3DIdx.end(), a.begin(), a.begin() + n3);
        pts2DIdx.insert(pts2DIdx.end(), b.begin(), b.begin() + n2);
        return SFM_OK;
      }
      if (std::max(n3, n2) <= cap) return rc;
      cap = std::max(n3, n2);
    }
    return SFM_EINVAL;
  }

  // getPointsInFrame for every frame of frameNo in one device query (the
  // per-keyframe loop of CSfM::bundleAdjustment, CSfM.cpp:321-340):
  // pts3DIdx[k] / pts2DIdx[k] receive frame frameNo[k]'s lists, as
  // getPointsInFrame would append them.  A frame may not be listed twice.
  int getPointsInFrameMulti(const std::vector<int>& frameNo, std::vector<std::vector<int>>& pts3DIdx,
                            std::vector<std::vector<int>>& pts2DIdx) {
    if (!h_) return rc_;
    const size_t nf = frameNo.size();
    pts3DIdx.resize(nf);
    pts2DIdx.resize(nf);
    int32_t np = 0;
    int64_t no = 0, nd = 0;
    if (int rc = sfm_map_size(h_, &np, &no, &nd)) return rc;
    std::vector<int32_t> fr(frameNo.begin(), frameNo.end()), o3(nf + 1), o2(nf + 1);
    int64_t cap = std::max<int64_t>(1, no);
    for (int attempt = 0; attempt < 2; ++attempt) {  // the 2D lists can outgrow n_obs: retry at the reported size
      std::vector<int32_t> a(static_cast<size_t>(cap)), b(static_cast<size_t>(cap));
      const int rc = sfm_map_points_in_frame_multi(h_, int32_t(nf), fr.data(), cap, a.data(), o3.data(), b.data(),
                                                   o2.data());
      if (rc == SFM_OK) {
        for (size_t k = 0; k < nf; ++k) {
          pts3DIdx[k].insert(pts3DIdx[k].end(), a.begin() + o3[k], a.begin() + o3[k + 1]);
          pts2DIdx[k].insert(pts2DIdx[k].end(), b.begin() + o2[k], b.begin() + o2[k + 1]);
        }
        return SFM_OK;
      }
      const int64_t need = std::max<int64_t>(o3[nf], o2[nf]);
      if (need <= cap) return rc;
      cap = need;
    }
    return SFM_EINVAL;
  }

  // CMap::getPointsInFrame_Mutable(pts3D, pts2DIdx, frameNo) (CMap.cpp:206-223),
  // the BA gather of CSfM::bundleAdjustment (CSfM.cpp:331): one pointer per
  // entry into the caller's point storage (CMap::_pts3D, Matx31 .val[3]).
  template <class Matx31>
  int getPointsInFrame_Mutable(std::vector<Matx31>& hostPts3D, std::vector<double*>& pts3D,
                               std::vector<int>& pts2DIdx, int frameNo) {
    std::vector<int> idx;
    const int rc = getPointsInFrame(idx, pts2DIdx, frameNo);
    if (rc) return rc;
    for (int p : idx) {
      if (p < 0 || size_t(p) >= hostPts3D.size()) return SFM_EINVAL;
      pts3D.push_back(hostPts3D[size_t(p)].val);
    }
    return SFM_OK;
  }

  // The device copy of the points after BA wrote the host ones back through
  // the pointers (CSfM.cpp:343), and the reverse: CMap::getPointsAtIdx
  // restated with its argument honoured (CMap.cpp:134-143 loops over every
  // point and ignores pts3DIdx, a reference bug not replicated).
  template <class Matx31>
  int setPointsAtIdx(const std::vector<int>& pts3DIdx, const std::vector<Matx31>& pts3D) {
    if (!h_) return rc_;
    const size_t n = pts3DIdx.size();
    if (pts3D.size() < n) return SFM_EINVAL;
    std::vector<double> X(3 * std::max<size_t>(1, n));
    for (size_t i = 0; i < n; ++i)
      for (int m = 0; m < 3; ++m) X[3 * i + m] = pts3D[i].val[m];
    return sfm_map_set_points(h_, int32_t(n), pts3DIdx.data(), X.data());
  }
  template <class Matx31>
  int getPointsAtIdx(const std::vector<int>& pts3DIdx, std::vector<Matx31>& pts3D) {
    if (!h_) return rc_;
    const size_t n = pts3DIdx.size();
    std::vector<double> X(3 * std::max<size_t>(1, n));
    if (n)
      if (int rc = sfm_map_get_points(h_, int32_t(n), pts3DIdx.data(), X.data())) return rc;
    for (size_t i = 0; i < n; ++i) {
      Matx31 m;
      for (int k = 0; k < 3; ++k) m.val[k] = X[3 * i + k];
      pts3D.push_back(m);
    }
    return SFM_OK;
  }

  // CMap::getRepresentativeDescriptors (CMap.cpp:345-381): per point, its row
  // with the smallest sum of Hamming distances to the others (first on
  // ties), appended to `descriptors` as [n][descBytes] bytes (wrap with
  // cv::Mat(n, descBytes, CV_8U, ptr) for the reference's Mat).
  int getRepresentativeDescriptors(const std::vector<int>& pts3DIdx, std::vector<uint8_t>& descriptors) {
    if (!h_) return rc_;
    const size_t n = pts3DIdx.size();
    if (n == 0) return SFM_OK;
    std::vector<uint8_t> d(n * size_t(desc_bytes_));
    const int rc = sfm_map_representative_descriptors(h_, int32_t(n), pts3DIdx.data(), d.data(), nullptr);
    if (rc) return rc;
    descriptors.insert(descriptors.end(), d.begin(), d.end());
    return SFM_OK;
  }

  // CSfM::findMapPointsInCurrentFrame's query (CSfM.cpp:634-692) as one
  // device call (sfm_map_match_frame): the points of keyframes frameNo minus
  // `existing`, projected by x = K (R X + t) (R9, K9 row-major), matched by
  // their representative descriptors against keypoints trainIdx of the frame
  // last pushed to `mt`; appends the (map point, frame keypoint) pairs.
  int matchFrame(FeatureMatcher& mt, const std::vector<int>& frameNo, const std::vector<int>& existing,
                 const double* R9, const double* t3, const double* K9, const std::vector<int>& trainIdx,
                 double ratio, double minDistance, double maxDistance, std::vector<int>& pts3DIdx,
                 std::vector<int>& kpIdx) {
    if (!h_) return rc_;
    if (trainIdx.size() < 2) return SFM_OK;
    std::vector<int32_t> p3(trainIdx.size()), k2(trainIdx.size());
    int32_t n = 0;
    const int rc = sfm_map_match_frame(h_, mt.handle(), int32_t(frameNo.size()), frameNo.data(),
                                       int32_t(existing.size()), existing.data(), R9, t3, K9,
                                       int32_t(trainIdx.size()), trainIdx.data(), ratio, minDistance, maxDistance,
                                       int32_t(trainIdx.size()), p3.data(), k2.data(), &n);
    if (rc) return rc;
    pts3DIdx.insert(pts3DIdx.end(), p3.begin(), p3.begin() + n);
    kpIdx.insert(kpIdx.end(), k2.begin(), k2.begin() + n);
    return SFM_OK;
  }

 private:
  sfm_map* h_ = nullptr;
  int rc_ = SFM_OK;
  int32_t desc_bytes_ = 64;
};

}  // namespace sfm_compat

#endif  // SFM_CTRACKER_COMPAT_HPP_
