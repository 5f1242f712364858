// Host side of sfm_ba_set_problem's layout, as plain C++ (no HIP): the
// keyframe-sized problems' checks and counts (k_validate's work done on the
// host), the camera runs and wavefront chunk table, the small path's XCD
// slice sizes and the bound of the camera-run blob staged for upload.
// Factored out of ba_solver.hip so that the CPU sanitizer build
// (tests/asan, `make asan`) runs exactly this code under ASan/UBSan.
//
// Reference: the observation / parameter-block layout is CSfM.cpp:310-341
// (one Ceres residual block per observation, CTracker.cpp:679-694); the
// checks are what the device validation (ba_setup.hip k_validate) reports.
#ifndef SFM_BA_HOST_LAYOUT_H_
#define SFM_BA_HOST_LAYOUT_H_

#include <algorithm>
#include <array>
#include <climits>
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace sfm {
namespace hostlayout {

// One 64-wide wavefront chunk of a camera's run (the int4 the device reads:
// camera, first camera-major position, count, the first observation's index
// in camera-major order).
struct Chunk {
  int32_t cam, pos, cnt, first;
};
static_assert(sizeof(Chunk) == 16, "Chunk must match the device's int4");

// The checks and counts of the observation arrays (k_validate's, on the host).
//   cam_cnt [C + 4]: [0..2] the first observation with a camera index out of
//     range / a point index out of range / a non-finite uv (INT32_MAX: none),
//     [3] = INT32_MAX, [4 + c] observations of camera c;
//   pc [P + 1]: observations of point p (pc[P] = 0);
//   cam_slice (want_slices): [C][8] observations of camera c in point slice s
//     (the 8 XCD slices of k_small_chunks' key: slice of p = floor(8 p / P));
//   pairs_est: sum over points of pc (pc - 1) / 2 -- every unordered pair of a
//     point's observations, i.e. the Schur pair total when no camera sees a
//     point twice (same-camera duplicates make it undercount; it is used for
//     the Schur pass's lane choice and, doubled, as the pair buffer's bound).
// Fast pass: the checks OR-ed without branches and the counts in four
// interleaved histograms (consecutive observations of one camera would
// otherwise chain every increment through a store-to-load dependency); only a
// problem with a bad observation takes the exact first-index pass.
inline void check_and_count(int64_t N, const double* obs_uv, const int32_t* cam_idx, const int32_t* pt_idx, int C,
                            int P, bool want_slices, int32_t* cam_cnt, int32_t* pc, std::vector<int32_t>* cam_slice,
                            int64_t* pairs_est) {
  int32_t first[3] = {INT32_MAX, INT32_MAX, INT32_MAX};
  std::fill(cam_cnt, cam_cnt + size_t(C) + 4, 0);
  std::fill(pc, pc + size_t(P) + 1, 0);
  cam_slice->clear();
  *pairs_est = 0;
  const uint64_t* uvb = reinterpret_cast<const uint64_t*>(obs_uv);
  auto nonfinite = [](uint64_t b) { return uint32_t(((b >> 52) & 0x7ff) == 0x7ff); };
  uint32_t bad = 0;
  {
    std::vector<int32_t> cc4(4 * (size_t(C) + 1), 0), pc4(4 * (size_t(P) + 1), 0);
    want_slices = want_slices && P > 0;
    // slice s = floor(8 p / P) holds p >= ceil(s P / 8): seven comparisons
    uint32_t sb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 1; k < 8; ++k) sb[k] = uint32_t((int64_t(k) * P + 7) / 8);
    auto slice_of = [&](uint32_t p) {
      uint32_t v = 0;
      for (int k = 1; k < 8; ++k) v += uint32_t(p >= sb[k]);
      return v;
    };
    std::vector<int32_t> cs4(want_slices ? 4 * 8 * (size_t(C) + 1) : 0, 0);
    int64_t i = 0;
    for (; i + 4 <= N; i += 4) {
      for (int u = 0; u < 4; ++u) {
        const uint32_t c = uint32_t(cam_idx[i + u]), p = uint32_t(pt_idx[i + u]);
        const uint32_t b = uint32_t(c >= uint32_t(C)) | uint32_t(p >= uint32_t(P)) | nonfinite(uvb[2 * (i + u)]) |
                           nonfinite(uvb[2 * (i + u) + 1]);
        bad |= b;
        // (an out-of-range index lands in the spare slot C / P: the counts
        // are discarded with the error anyway)
        const uint32_t cc = c < uint32_t(C) ? c : uint32_t(C);
        ++cc4[u * (size_t(C) + 1) + cc];
        ++pc4[u * (size_t(P) + 1) + (p < uint32_t(P) ? p : uint32_t(P))];
        if (want_slices) ++cs4[(u * (size_t(C) + 1) + cc) * 8 + slice_of(p)];
      }
    }
    for (; i < N; ++i) {
      const uint32_t c = uint32_t(cam_idx[i]), p = uint32_t(pt_idx[i]);
      bad |= uint32_t(c >= uint32_t(C)) | uint32_t(p >= uint32_t(P)) | nonfinite(uvb[2 * i]) |
             nonfinite(uvb[2 * i + 1]);
      const uint32_t cc = c < uint32_t(C) ? c : uint32_t(C);
      ++cc4[cc];
      ++pc4[p < uint32_t(P) ? p : uint32_t(P)];
      if (want_slices) ++cs4[size_t(cc) * 8 + slice_of(p)];
    }
    if (want_slices) {
      cam_slice->assign(8 * size_t(C), 0);
      for (size_t e = 0; e < 8 * size_t(C); ++e)
        (*cam_slice)[e] = cs4[e] + cs4[8 * (size_t(C) + 1) + e] + cs4[16 * (size_t(C) + 1) + e] +
                          cs4[24 * (size_t(C) + 1) + e];
    }
    for (int c = 0; c < C; ++c)
      cam_cnt[4 + size_t(c)] =
          cc4[c] + cc4[(size_t(C) + 1) + c] + cc4[2 * (size_t(C) + 1) + c] + cc4[3 * (size_t(C) + 1) + c];
    for (int p = 0; p < P; ++p) {
      pc[p] = pc4[p] + pc4[(size_t(P) + 1) + p] + pc4[2 * (size_t(P) + 1) + p] + pc4[3 * (size_t(P) + 1) + p];
      *pairs_est += int64_t(pc[p]) * (pc[p] - 1) / 2;
    }
  }
  if (bad) {
    for (int64_t i = 0; i < N; ++i) {
      const int32_t c = cam_idx[i], p = pt_idx[i];
      const bool cok = c >= 0 && c < C, pok = p >= 0 && p < P;
      const bool uok = std::isfinite(obs_uv[2 * i]) && std::isfinite(obs_uv[2 * i + 1]);
      if (!cok && first[0] == INT32_MAX) first[0] = int32_t(i);
      if (!pok && first[1] == INT32_MAX) first[1] = int32_t(i);
      if (!uok && first[2] == INT32_MAX) first[2] = int32_t(i);
    }
  }
  cam_cnt[0] = first[0];
  cam_cnt[1] = first[1];
  cam_cnt[2] = first[2];
  cam_cnt[3] = INT32_MAX;
}

// Camera runs: camera-major, each camera's run padded to a whole number of
// 64-wide wavefront chunks; wcam[w] = the camera of chunk slot w; the chunk
// table camera-major (the device groups it into 8 point slices).
struct Runs {
  std::vector<int32_t> cam_off, cam_rng, wcam;
  std::vector<Chunk> chunks;
  int64_t npad = 0;
};
inline void camera_runs(int C, const int32_t* n_obs_of_cam, Runs* r) {
  r->cam_off.assign(size_t(C) + 1, 0);
  r->cam_rng.assign(2 * size_t(C), 0);
  int64_t npad = 0;
  for (int c = 0; c < C; ++c) {
    const int32_t n_c = n_obs_of_cam[c];
    r->cam_off[c + 1] = r->cam_off[c] + n_c;
    r->cam_rng[2 * c] = int32_t(npad);
    r->cam_rng[2 * c + 1] = int32_t(npad + n_c);
    npad += (n_c + 63) / 64 * 64;
  }
  r->npad = npad;
  r->wcam.assign(size_t(npad / 64) + 1, 0);
  for (int c = 0; c < C; ++c)
    for (int64_t w = r->cam_rng[2 * c] / 64;
         w < (int64_t(r->cam_rng[2 * c]) + r->cam_off[c + 1] - r->cam_off[c] + 63) / 64; ++w)
      r->wcam[size_t(w)] = c;
  r->chunks.clear();
  for (int c = 0; c < C; ++c) {
    const int32_t n_c = r->cam_off[c + 1] - r->cam_off[c];
    for (int32_t k = 0; 64 * k < n_c; ++k)
      r->chunks.push_back(Chunk{c, r->cam_rng[2 * c] + 64 * k, std::min<int32_t>(64, n_c - 64 * k),
                                r->cam_off[c] + 64 * k});
  }
}

// Small path: the chunk table's slice sizes from the host's per-camera slice
// counts (camera c's chunk k starts at its 64 k-th observation in point
// order, whose slice the counts' running sum gives) -> the largest slice.
inline int32_t small_slice_max(int C, const int32_t* n_obs_of_cam, const std::vector<int32_t>& cam_slice) {
  std::array<int32_t, 8> jcnt{};
  for (int c = 0; c < C; ++c) {
    const int32_t n_c = n_obs_of_cam[c];
    int32_t cum = 0;
    int sl = 0;
    for (int32_t k = 0; 64 * k < n_c; ++k) {
      while (sl < 7 && cum + cam_slice[8 * size_t(c) + sl] <= 64 * k) cum += cam_slice[8 * size_t(c) + sl++];
      ++jcnt[size_t(sl)];
    }
  }
  return *std::max_element(jcnt.begin(), jcnt.end());
}

// Bytes the camera-run blob (cam_rng | wcam | cam_off | chunks, and on the
// small path pt_off | the scatters' slot counters) can take, staged behind
// the still-in-flight input blob: 2 C + (npad / 64 + 1) + (C + 1) ints, 16 B
// per chunk (npad / 64 <= N / 64 + C chunks), P + 1 + P + C ints, padding.
inline size_t runs_blob_bound(int C, int64_t N, int P) {
  return 64 * (size_t(C) + 1) + 2 * size_t(N) + 8 * (size_t(P) + 1) + 4 * size_t(C) + 2048;
}

}  // namespace hostlayout
}  // namespace sfm

#endif  // SFM_BA_HOST_LAYOUT_H_
