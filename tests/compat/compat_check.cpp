// Compile-and-run check of include/sfm_ctracker_compat.hpp on the CPU:
// packing/deduplication of the reference's pointer-identified point blocks,
// and the error path of the drop-in call without a GPU (nothing written).
#include <cstdio>
#include <vector>
#include "sfm_ctracker_compat.hpp"

struct Pt { double x, y; };          // cv::Point2d layout
struct M33 { double val[9]; };       // cv::Matx33d layout
struct Grey { const unsigned char* data; size_t step; int cols, rows; };  // cv::Mat (CV_8U) fields used

int main() {
  double X[3][3] = {{1, 2, 3}, {4, 5, 6}, {7, 8, 9}};
  double r0[3] = {0, 0, 0}, r1[3] = {0.1, 0.2, 0.3}, t0[3] = {0, 0, 8}, t1[3] = {1, 1, 8};
  std::vector<double*> R = {r0, r1}, T = {t0, t1};
  M33 k{{1000, 0, 640, 0, 1000, 360, 0, 0, 1}};
  std::vector<M33> K = {k, k};
  // observation order: point 2, point 0, point 2, point 1, point 0 (addresses repeat)
  std::vector<Pt> obs = {{1, 1}, {2, 2}, {3, 3}, {4, 4}, {5, 5}};
  std::vector<int> cam = {0, 0, 1, 1, 1};
  std::vector<double*> pts = {X[2], X[0], X[2], X[1], X[0]};
  sfm_compat::PackedProblem p;
  if (sfm_compat::pack_problem(obs, cam, K, R, T, pts, &p) != 0) return 1;
  const int want_idx[5] = {0, 1, 0, 2, 1};
  for (int i = 0; i < 5; ++i)
    if (p.pt_idx[i] != want_idx[i]) { std::printf("pt_idx mismatch at %d\n", i); return 2; }
  if (p.point_ptr.size() != 3 || p.X[0] != 7 || p.X[3] != 1 || p.X[6] != 4) return 3;
  if (p.K9[9 + 2] != 640 || p.rot[3 + 1] != 0.2 || p.t[3 + 2] != 8 || p.uv[2 * 3 + 1] != 4) return 4;
  // bad camera index -> EINVAL
  std::vector<int> bad = {0, 0, 2, 1, 1};
  if (sfm_compat::pack_problem(obs, bad, K, R, T, pts, &p) != SFM_EINVAL) return 5;
  // without a GPU the drop-in returns the ABI error and writes nothing back
  if (sfm_device_count() == 0) {
    const int rc = sfm_compat::bundleAdjustmentStructAndPose(obs, cam, K, R, T, pts, SFM_BA_STRUCT_AND_POSE);
    if (rc != SFM_ENODEV || X[0][0] != 1 || r1[0] != 0.1) { std::printf("rc=%d\n", rc); return 6; }
  }
  // optical flow shim: without a GPU creation fails and nothing is matched
  if (sfm_device_count() == 0) {
    sfm_compat::OpticalFlowTracker flow(64, 48);
    if (flow.status() != SFM_ENODEV) { std::printf("klt rc=%d\n", flow.status()); return 7; }
    std::vector<unsigned char> img(64 * 48, 7);
    Grey g{img.data(), 64, 64, 48};
    if (flow.pushFrame(g) != SFM_ENODEV) return 8;
    std::vector<int> pi = {1}, ci = {2};
    int rc = 0;
    std::vector<Pt> prev = {{10, 10}}, curr = {{11, 11}};
    if (flow.computeOpticalFlow(prev, curr, pi, ci, 5, &rc) || rc != SFM_ENODEV || !pi.empty() || !ci.empty()) return 9;
    struct Pt2f { float x, y; };
    std::vector<Pt2f> corners = {{1.f, 2.f}};
    if (flow.detectFeaturesOpticalFlow(corners, 5, nullptr, &rc) || rc != SFM_ENODEV || !corners.empty()) return 10;
  }
  std::printf("compat ok\n");
  return 0;
}
