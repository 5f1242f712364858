// GPU run of include/sfm_ctracker_compat.hpp exactly as the reference's C++
// pipeline would call it (the binding INTEGRATION.md tells a maintainer to
// paste).  Inputs / outputs are raw little-endian arrays in a directory,
// written and checked by tests/test_gpu_compat.py against the oracle.
//
//   compat_gpu ba <dir>     CSfM::bundleAdjustment (CSfM.cpp:310-348): the
//                           problem gathered keyframe by keyframe (frame-major
//                           order, K / R / t per keyframe, one aliased double*
//                           per observation into the map's point storage, as
//                           CMap::getPointsInFrame_Mutable yields them,
//                           CMap.cpp:206-223), then the drop-in
//                           bundleAdjustmentStructAndPose writes back in place.
//   compat_gpu flow <dir>   detectFeaturesOpticalFlow on two frames +
//                           computeOpticalFlow (CTracker.cpp:252-272, 480-562).
//   compat_gpu match <dir>  the frame-resident matcher: matchFeatures(prevIdx,
//                           currIdx, ...) (CSfM.cpp:518), matchFeatures()
//                           (CSfM.cpp:823) and the (pts, desc, ..., 0, 7)
//                           overload (CSfM.cpp:673).
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "sfm_ctracker_compat.hpp"

struct Pt { double x, y; };                 // cv::Point2d
struct Pt2f { float x, y; };                // cv::Point2f
struct M33 { double val[9]; };              // cv::Matx33d
struct M31 { double val[3]; };              // cv::Matx31d (CMap::_pts3D element)
struct Grey { const unsigned char* data; size_t step; int cols, rows; };
struct Desc { const unsigned char* data; int rows, cols; };   // cv::Mat CV_8U fields used

template <class T>
static std::vector<T> rd(const std::string& dir, const char* name) {
  std::vector<T> v;
  FILE* f = std::fopen((dir + "/" + name).c_str(), "rb");
  if (!f) return v;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  v.resize(size_t(n) / sizeof(T));
  if (!v.empty() && std::fread(v.data(), sizeof(T), v.size(), f) != v.size()) v.clear();
  std::fclose(f);
  return v;
}
template <class T>
static void wr(const std::string& dir, const char* name, const std::vector<T>& v) {
  FILE* f = std::fopen((dir + "/" + name).c_str(), "wb");
  if (!v.empty()) std::fwrite(v.data(), sizeof(T), v.size(), f);
  std::fclose(f);
}

// meta.i32 = [C, P]; kf_K.f64 [C][9]; kf_rot.f64 / kf_t.f64 [C][3];
// kf_pts.f64 = every keyframe's 2-D points back to back, kf_npts.i32 [C];
// view_off.i32 [C+1], view_pt.i32 / view_2d.i32: keyframe c sees map point
// view_pt[k] at its 2-D point view_2d[k], k in [view_off[c], view_off[c+1]);
// map.f64 [P][3].
static int run_ba(const std::string& dir) {
  auto meta = rd<int32_t>(dir, "meta.i32");
  const int C = meta[0], P = meta[1];
  auto kK = rd<double>(dir, "kf_K.f64"), krot = rd<double>(dir, "kf_rot.f64"), kt = rd<double>(dir, "kf_t.f64");
  auto kpts = rd<double>(dir, "kf_pts.f64");
  auto knp = rd<int32_t>(dir, "kf_npts.i32");
  auto voff = rd<int32_t>(dir, "view_off.i32"), vpt = rd<int32_t>(dir, "view_pt.i32"),
       v2d = rd<int32_t>(dir, "view_2d.i32");
  auto mp = rd<double>(dir, "map.f64");
  struct KeyFrame { M33 K; double rot[3], t[3]; std::vector<Pt> pts; };
  std::vector<KeyFrame> kf(C);
  size_t off = 0;
  for (int c = 0; c < C; ++c) {
    for (int k = 0; k < 9; ++k) kf[c].K.val[k] = kK[9 * c + k];
    for (int k = 0; k < 3; ++k) { kf[c].rot[k] = krot[3 * c + k]; kf[c].t[k] = kt[3 * c + k]; }
    kf[c].pts.resize(knp[c]);
    for (int i = 0; i < knp[c]; ++i) kf[c].pts[i] = Pt{kpts[off + 2 * i], kpts[off + 2 * i + 1]};
    off += 2 * size_t(knp[c]);
  }
  std::vector<M31> pts3D(P);
  for (int p = 0; p < P; ++p)
    for (int k = 0; k < 3; ++k) pts3D[p].val[k] = mp[3 * p + k];
  // CSfM::bundleAdjustment's gather, keyframe by keyframe
  std::vector<double*> R, t, pts3d;
  std::vector<Pt> pts2d;
  std::vector<int> camIdx;
  std::vector<M33> K;
  for (int i = 0; i < C; ++i) {
    K.push_back(kf[i].K);
    t.push_back(kf[i].t);
    R.push_back(kf[i].rot);
    std::vector<int> pts2dIdx;
    for (int k = voff[i]; k < voff[i + 1]; ++k) {        // getPointsInFrame_Mutable
      pts3d.push_back(pts3D[vpt[k]].val);
      pts2dIdx.push_back(v2d[k]);
    }
    for (int j : pts2dIdx) pts2d.push_back(kf[i].pts[j]);  // getPointsAt
    for (size_t j = camIdx.size(); j < pts3d.size(); ++j) camIdx.push_back(i);
  }
  sfm_ba_summary sm;
  const int rc = sfm_compat::bundleAdjustmentStructAndPose(pts2d, camIdx, K, R, t, pts3d,
                                                           SFM_BA_STRUCT_AND_POSE, nullptr, &sm);
  if (rc) { std::printf("ba rc=%d %s\n", rc, sfm_last_error()); return 1; }
  std::vector<double> orot(3 * size_t(C)), ot(3 * size_t(C)), oX(3 * size_t(P));
  for (int c = 0; c < C; ++c)
    for (int k = 0; k < 3; ++k) { orot[3 * c + k] = kf[c].rot[k]; ot[3 * c + k] = kf[c].t[k]; }
  for (int p = 0; p < P; ++p)
    for (int k = 0; k < 3; ++k) oX[3 * p + k] = pts3D[p].val[k];
  wr(dir, "out_rot.f64", orot);
  wr(dir, "out_t.f64", ot);
  wr(dir, "out_X.f64", oX);
  wr(dir, "out_summary.f64", std::vector<double>{double(sm.termination_type), double(sm.num_iterations),
                                                 sm.initial_cost, sm.final_cost});
  return 0;
}

// meta.i32 = [w, h]; prev.u8 / curr.u8 [h][w]
static int run_flow(const std::string& dir) {
  auto meta = rd<int32_t>(dir, "meta.i32");
  const int w = meta[0], h = meta[1];
  auto f0 = rd<uint8_t>(dir, "prev.u8"), f1 = rd<uint8_t>(dir, "curr.u8");
  sfm_compat::OpticalFlowTracker flow(w, h);
  if (flow.status()) { std::printf("flow create rc=%d\n", flow.status()); return 1; }
  Grey g0{f0.data(), size_t(w), w, h}, g1{f1.data(), size_t(w), w, h};
  std::vector<Pt2f> c0, c1;
  int rc = 0;
  if (flow.pushFrame(g0)) return 2;
  flow.detectFeaturesOpticalFlow(c0, 5, nullptr, &rc);
  if (rc) return 3;
  if (flow.pushFrame(g1)) return 4;
  flow.detectFeaturesOpticalFlow(c1, 5, nullptr, &rc);
  if (rc) return 5;
  std::vector<Pt> p0(c0.size()), p1(c1.size());
  for (size_t i = 0; i < c0.size(); ++i) p0[i] = Pt{c0[i].x, c0[i].y};
  for (size_t i = 0; i < c1.size(); ++i) p1[i] = Pt{c1[i].x, c1[i].y};
  std::vector<int> pi, ci;
  const bool ok = flow.computeOpticalFlow(p0, p1, pi, ci, 5, &rc);
  if (rc) return 6;
  std::vector<float> o0, o1;
  for (auto& c : c0) { o0.push_back(c.x); o0.push_back(c.y); }
  for (auto& c : c1) { o1.push_back(c.x); o1.push_back(c.y); }
  wr(dir, "out_c0.f32", o0);
  wr(dir, "out_c1.f32", o1);
  wr(dir, "out_pi.i32", pi);
  wr(dir, "out_ci.i32", ci);
  wr(dir, "out_ok.i32", std::vector<int32_t>{ok ? 1 : 0});
  return 0;
}

// meta.i32 = [n0, n1, nbytes]; f0_pts / f0_dist / f1_pts / f1_dist .f64;
// f0_desc / f1_desc .u8; sub0 / sub1 .i32 (index subsets)
static int run_match(const std::string& dir) {
  auto meta = rd<int32_t>(dir, "meta.i32");
  const int n0 = meta[0], n1 = meta[1], nb = meta[2];
  auto rp = [&](const char* nm) {
    auto v = rd<double>(dir, nm);
    std::vector<Pt> p(v.size() / 2);
    for (size_t i = 0; i < p.size(); ++i) p[i] = Pt{v[2 * i], v[2 * i + 1]};
    return p;
  };
  auto p0 = rp("f0_pts.f64"), q0 = rp("f0_dist.f64"), p1 = rp("f1_pts.f64"), q1 = rp("f1_dist.f64");
  auto d0 = rd<uint8_t>(dir, "f0_desc.u8"), d1 = rd<uint8_t>(dir, "f1_desc.u8");
  auto s0 = rd<int32_t>(dir, "sub0.i32"), s1 = rd<int32_t>(dir, "sub1.i32");
  Desc D0{d0.data(), n0, nb}, D1{d1.data(), n1, nb};
  sfm_compat::FeatureMatcher m(nb);
  if (m.status()) { std::printf("matcher create rc=%d\n", m.status()); return 1; }
  if (m.pushFrame(p0, q0, D0) || m.pushFrame(p1, q1, D1)) return 2;
  std::vector<int> a, b;
  if (m.matchFeatures(std::vector<int>(s0.begin(), s0.end()), std::vector<int>(s1.begin(), s1.end()), a, b)) return 3;
  std::vector<int> pi, ci;
  int rc = 0;
  const bool ok = m.matchFeatures(pi, ci, 5, &rc);
  if (rc) return 4;
  std::vector<int> w0, w1;
  if (m.matchFeatures(p0, D0, p1, D1, w0, w1, 0.0, 7.0)) return 5;
  // the one-shot free function (member-window overload, CTracker.cpp:114-149)
  std::vector<int> f0, f1;
  if (sfm_compat::matchFeatures(p0, D0, p1, D1, f0, f1)) return 6;
  wr(dir, "out_sub_a.i32", a);
  wr(dir, "out_sub_b.i32", b);
  wr(dir, "out_all_a.i32", pi);
  wr(dir, "out_all_b.i32", ci);
  wr(dir, "out_ok.i32", std::vector<int32_t>{ok ? 1 : 0});
  wr(dir, "out_w7_a.i32", w0);
  wr(dir, "out_w7_b.i32", w1);
  wr(dir, "out_free_a.i32", f0);
  wr(dir, "out_free_b.i32", f1);
  return 0;
}

int main(int argc, char** argv) {
  if (argc != 3) { std::printf("usage: compat_gpu ba|flow|match <dir>\n"); return 64; }
  const std::string mode = argv[1], dir = argv[2];
  int rc = mode == "ba" ? run_ba(dir) : mode == "flow" ? run_flow(dir) : mode == "match" ? run_match(dir) : 64;
  if (rc == 0) std::printf("compat_gpu %s ok\n", mode.c_str());
  return rc;
}
