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
//   compat_gpu pnp <dir>    solvePnPRansac as CSfM::tracking calls it
//                           (CSfM.cpp:553-565), cv::Matx31d object points.
//   compat_gpu brisk <dir>  the detectFeatures body (CTracker.cpp:275-287):
//                           keypoints as cv::KeyPoint + descriptor rows.
//   compat_gpu map <dir>    a CMap-shaped store (CMap.cpp:36-381) driven by a
//                           script of addNewPoints / addPointMatches /
//                           addDescriptors calls and queries, as CSfM::mapping
//                           and CSfM::tracking make them.
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "sfm_ctracker_compat.hpp"

struct Pt { double x, y; };                 // cv::Point2d
struct Pt2f { float x, y; };                // cv::Point2f
struct M33 { double val[9]; };              // cv::Matx33d
struct M31 { double val[3]; };              // cv::Matx31d (CMap::_pts3D element)
struct Grey { const unsigned char* data; size_t step; int cols, rows; };
struct Desc { const unsigned char* data; int rows, cols; };   // cv::Mat CV_8U fields used
struct KeyPoint { Pt2f pt; float size, angle, response; int octave, class_id; };   // cv::KeyPoint

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

// meta.i32 = [n, iterations]; par.f64 = [reprojectionError, confidence];
// obj.f64 [n][3]; img.f64 [n][2]; K.f64 [9]
static int run_pnp(const std::string& dir) {
  auto meta = rd<int32_t>(dir, "meta.i32");
  auto par = rd<double>(dir, "par.f64");
  const int n = meta[0], iters = meta[1];
  auto ob = rd<double>(dir, "obj.f64"), im = rd<double>(dir, "img.f64"), kk = rd<double>(dir, "K.f64");
  std::vector<M31> currMatch3D(n);
  std::vector<Pt> currMatch2D(n);
  for (int i = 0; i < n; ++i) {
    for (int k = 0; k < 3; ++k) currMatch3D[i].val[k] = ob[3 * i + k];
    currMatch2D[i] = Pt{im[2 * i], im[2 * i + 1]};
  }
  M33 K;
  for (int k = 0; k < 9; ++k) K.val[k] = kk[k];
  double rv[3] = {0, 0, 0}, tv[3] = {0, 0, 0};
  std::vector<int> inlierIdx;
  const bool found = sfm_compat::solvePnPRansac(currMatch3D, currMatch2D, K, rv, tv, inlierIdx, iters, par[0], par[1]);
  wr(dir, "out_found.i32", std::vector<int32_t>{found ? 1 : 0});
  wr(dir, "out_pose.f64", std::vector<double>{rv[0], rv[1], rv[2], tv[0], tv[1], tv[2]});
  wr(dir, "out_inliers.i32", inlierIdx);
  return 0;
}

// meta.i32 = [w, h, threshold, octaves, step]; img.u8 [h][step] (rows padded
// to `step` bytes, as a cv::Mat ROI of a wider image would be)
static int run_brisk(const std::string& dir) {
  auto meta = rd<int32_t>(dir, "meta.i32");
  auto img = rd<uint8_t>(dir, "img.u8");
  Grey g{img.data(), size_t(meta[4]), meta[0], meta[1]};
  std::vector<KeyPoint> kp;
  std::vector<uint8_t> desc;
  const int rc = sfm_compat::detectFeatures(g, kp, desc, meta[2], meta[3]);
  if (rc) { std::printf("brisk rc=%d %s\n", rc, sfm_last_error()); return 1; }
  std::vector<float> k;
  std::vector<int32_t> oct;
  for (auto& p : kp) {
    k.insert(k.end(), {p.pt.x, p.pt.y, p.size, p.angle, p.response});
    oct.push_back(p.octave);
  }
  wr(dir, "out_kp.f32", k);
  wr(dir, "out_octave.i32", oct);
  wr(dir, "out_desc.u8", desc);
  // the same frame pushed into the optical-flow tracker, BRISK on its
  // resident copy (OpticalFlowTracker::detectFeaturesBrisk: one upload)
  sfm_compat::OpticalFlowTracker flow(meta[0], meta[1]);
  if (flow.status() || flow.pushFrame(g)) { std::printf("brisk flow rc=%d %s\n", flow.status(), sfm_last_error()); return 1; }
  std::vector<KeyPoint> kr;
  std::vector<uint8_t> dr;
  if (int r2 = flow.detectFeaturesBrisk(kr, dr, meta[2], meta[3])) {
    std::printf("brisk resident rc=%d %s\n", r2, sfm_last_error());
    return 1;
  }
  k.clear();
  oct.clear();
  for (auto& p : kr) {
    k.insert(k.end(), {p.pt.x, p.pt.y, p.size, p.angle, p.response});
    oct.push_back(p.octave);
  }
  wr(dir, "out_kp_res.f32", k);
  wr(dir, "out_octave_res.i32", oct);
  wr(dir, "out_desc_res.u8", dr);
  // a capacity far below the frame's keypoint count: both entry points retry
  // once at the reported count and return the same keypoints
  std::vector<KeyPoint> ks;
  std::vector<uint8_t> ds;
  if (int r3 = sfm_compat::detectFeatures(g, ks, ds, meta[2], meta[3], 16)) {
    std::printf("brisk small-capacity rc=%d %s\n", r3, sfm_last_error());
    return 1;
  }
  if (ks.size() != kp.size() || ds != desc) { std::printf("brisk small-capacity mismatch\n"); return 1; }
  if (int r4 = flow.detectFeaturesBrisk(ks, ds, meta[2], meta[3], 16)) {
    std::printf("brisk resident small-capacity rc=%d %s\n", r4, sfm_last_error());
    return 1;
  }
  if (ks.size() != kr.size() || ds != dr) { std::printf("brisk resident small-capacity mismatch\n"); return 1; }
  return 0;
}

// script.txt: one call per line (see tests/test_gpu_compat.py), answers of
// the queries to out.txt, one line each.
static int run_map(const std::string& dir) {
  std::ifstream in(dir + "/script.txt");
  std::ofstream out(dir + "/out.txt");
  sfm_compat::MapStore cmap(64);
  if (cmap.status()) { std::printf("map create rc=%d\n", cmap.status()); return 1; }
  std::vector<M31> pts3DHost;  // CMap::_pts3D (host member, the BA pointers' target)
  std::string line;
  auto ints = [](std::istringstream& is, int n) { std::vector<int> v(n); for (auto& x : v) is >> x; return v; };
  auto hexrow = [](const std::string& h) {
    std::vector<uint8_t> b(h.size() / 2);
    for (size_t i = 0; i < b.size(); ++i) b[i] = uint8_t(std::stoi(h.substr(2 * i, 2), nullptr, 16));
    return b;
  };
  auto tohex = [](const std::vector<uint8_t>& b) {
    static const char* hx = "0123456789abcdef";
    std::string s;
    for (uint8_t c : b) { s += hx[c >> 4]; s += hx[c & 15]; }
    return s;
  };
  int rc = 0;
  while (std::getline(in, line)) {
    std::istringstream is(line);
    std::string op;
    is >> op;
    if (op == "N") {           // addNewPoints: nf n frames[nf] idx2d[nf][n] X[n][3]
      int nf, n;
      is >> nf >> n;
      auto frames = ints(is, nf);
      std::vector<std::vector<int>> p2(nf);
      for (auto& v : p2) v = ints(is, n);
      std::vector<M31> X(n);
      for (auto& m : X) is >> m.val[0] >> m.val[1] >> m.val[2];
      std::vector<int> idx;
      if ((rc = cmap.addNewPoints(X, p2, frames, idx))) break;
      pts3DHost.insert(pts3DHost.end(), X.begin(), X.end());
      out << "N";
      for (int i : idx) out << ' ' << i;
      out << '\n';
    } else if (op == "M") {    // addPointMatches: frame n p3[n] p2[n]
      int f, n;
      is >> f >> n;
      auto a = ints(is, n), b = ints(is, n);
      if ((rc = cmap.addPointMatches(a, b, f))) break;
    } else if (op == "D") {    // addDescriptors: n p3[n] hex rows
      int n;
      is >> n;
      auto a = ints(is, n);
      std::vector<uint8_t> rows;
      for (int i = 0; i < n; ++i) { std::string h; is >> h; auto r = hexrow(h); rows.insert(rows.end(), r.begin(), r.end()); }
      Desc d{rows.data(), n, 64};
      if ((rc = cmap.addDescriptors(a, d))) break;
    } else if (op == "QF") {   // getPointsInFrames: nf frames
      int nf;
      is >> nf;
      auto frames = ints(is, nf);
      std::vector<int> p;
      if ((rc = cmap.getPointsInFrames(p, frames))) break;
      out << "QF";
      for (int i : p) out << ' ' << i;
      out << '\n';
    } else if (op == "Q") {    // getPointsInFrame(pts3DIdx, pts2DIdx, f)
      int f;
      is >> f;
      std::vector<int> a, b;
      if ((rc = cmap.getPointsInFrame(a, b, f))) break;
      out << "Q " << a.size();
      for (int i : a) out << ' ' << i;
      out << ' ' << b.size();
      for (int i : b) out << ' ' << i;
      out << '\n';
    } else if (op == "QB") {   // getPointsInFrameMulti (the BA gather): nf frames -> one line
      int nf;
      is >> nf;
      auto frames = ints(is, nf);
      std::vector<std::vector<int>> a, b;
      if ((rc = cmap.getPointsInFrameMulti(frames, a, b))) break;
      out << "QB";
      for (int k = 0; k < nf; ++k) {
        out << ' ' << a[k].size();
        for (int i : a[k]) out << ' ' << i;
        out << ' ' << b[k].size();
        for (int i : b[k]) out << ' ' << i;
      }
      out << '\n';
    } else if (op == "QM") {   // getPointsInFrame_Mutable: the pointers, as point indices
      int f;
      is >> f;
      std::vector<double*> ptr;
      std::vector<int> b;
      if ((rc = cmap.getPointsInFrame_Mutable(pts3DHost, ptr, b, f))) break;
      out << "QM " << ptr.size();
      for (double* q : ptr) out << ' ' << (q - pts3DHost[0].val) / 3;
      out << ' ' << b.size();
      for (int i : b) out << ' ' << i;
      out << '\n';
    } else if (op == "R") {    // getRepresentativeDescriptors: n p3
      int n;
      is >> n;
      auto a = ints(is, n);
      std::vector<uint8_t> d;
      if ((rc = cmap.getRepresentativeDescriptors(a, d))) break;
      out << "R " << tohex(d) << '\n';
    } else if (op == "S") {    // setPointsAtIdx (BA write-back): n p3 X
      int n;
      is >> n;
      auto a = ints(is, n);
      std::vector<M31> X(n);
      for (auto& m : X) is >> m.val[0] >> m.val[1] >> m.val[2];
      if ((rc = cmap.setPointsAtIdx(a, X))) break;
    } else if (op == "G") {    // getPointsAtIdx: n p3
      int n;
      is >> n;
      auto a = ints(is, n);
      std::vector<M31> X;
      if ((rc = cmap.getPointsAtIdx(a, X))) break;
      char buf[64];
      out << "G";
      for (auto& m : X)
        for (double v : m.val) { std::snprintf(buf, sizeof buf, " %.17g", v); out << buf; }
      out << '\n';
    } else if (op == "C") {    // getNPoints
      out << "C " << cmap.getNPoints() << '\n';
    } else if (!op.empty()) {
      std::printf("map: bad op %s\n", op.c_str());
      return 2;
    }
  }
  if (rc) { std::printf("map rc=%d %s\n", rc, sfm_last_error()); return 1; }
  return 0;
}

int main(int argc, char** argv) {
  if (argc != 3) { std::printf("usage: compat_gpu ba|flow|match|pnp|brisk|map <dir>\n"); return 64; }
  const std::string mode = argv[1], dir = argv[2];
  int rc = mode == "ba" ? run_ba(dir) : mode == "flow" ? run_flow(dir) : mode == "match" ? run_match(dir)
         : mode == "pnp" ? run_pnp(dir) : mode == "brisk" ? run_brisk(dir) : mode == "map" ? run_map(dir) : 64;
  if (rc == 0) std::printf("compat_gpu %s ok\n", mode.c_str());
  return rc;
}
