// Host-side problem layout for keyframe-sized problems (sfm_ba_set_problem).
//
// The reference rebuilds its ceres::Problem on every keyframe BA
// (/root/reference/CTracker.cpp:672-691), and at that size (tens of cameras,
// a few thousand points: CSfM.cpp:252-259) the device setup of ba_setup.hip
// is launch-bound: ~30 sort/scan/gather kernels and two host round trips for
// 20k observations.  This file builds the same arrays on the host, written
// straight into the pinned staging buffer that then goes up in one DMA:
//   * validation and the per-camera / per-point counts (k_validate);
//   * the point-major order, a stable sort by (point, camera): a stable
//     counting sort by point, then a stable insertion sort by camera inside
//     each point's (short) run -- the order sort_pairs64 produces;
//   * the camera-major order of the point-major ids, stable by camera (a
//     counting sort: the order of sort_pairs32 with iota values), and the
//     padded camera-major arrays (k_fill_cm);
//   * the chunk table grouped by point slice, stable (k_chunk_keys +
//     sort_pairs32 + k_chunk_gather);
//   * the Schur pair lists: emitted in (camera-major entry, o2 ascending)
//     order and placed by a stable counting sort on the block key, i.e.
//     exactly the device's k_pair_fill + stable radix sort; seg is the
//     counting sort's offsets (k_seg's lower bounds), blk the block table.
// Integer work only, every output bitwise the device path's (GPU test
// tests/test_gpu_scale.py::test_host_setup_equals_device_setup).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include "ba_setup.h"

namespace sfm {

void host_validate(int64_t N, const double* uv, const int32_t* cam, const int32_t* pt, int C, int P, int32_t err[3],
                   int32_t* cam_cnt, std::vector<int32_t>& pt_cnt) {
  err[0] = err[1] = err[2] = INT32_MAX;
  std::fill(cam_cnt, cam_cnt + C, 0);
  pt_cnt.assign(size_t(P) + 1, 0);
  for (int64_t i = 0; i < N; ++i) {
    const int c = cam[i], p = pt[i];
    const bool cok = c >= 0 && c < C, pok = p >= 0 && p < P;
    const bool uok = std::isfinite(uv[2 * i]) && std::isfinite(uv[2 * i + 1]);
    if (!cok && err[0] == INT32_MAX) err[0] = int32_t(i);
    if (!pok && err[1] == INT32_MAX) err[1] = int32_t(i);
    if (!uok && err[2] == INT32_MAX) err[2] = int32_t(i);
    if (cok && pok) {
      ++cam_cnt[c];
      ++pt_cnt[p];
    }
  }
}

int64_t host_orders(int64_t N, const int32_t* cam, const int32_t* pt, int C, int P, const std::vector<int32_t>& pt_cnt,
                    const std::vector<int32_t>& cam_off, HostOrders& o) {
  o.pt_off.assign(size_t(P) + 1, 0);
  for (int p = 0; p < P; ++p) o.pt_off[p + 1] = o.pt_off[p] + pt_cnt[p];
  // point-major: stable by point, then stable by camera inside each run
  o.order.resize(size_t(N));
  {
    std::vector<int32_t> cur(o.pt_off.begin(), o.pt_off.end() - (P > 0 ? 1 : 0));
    for (int64_t i = 0; i < N; ++i) o.order[cur[pt[i]]++] = int32_t(i);
  }
  for (int p = 0; p < P; ++p) {
    int32_t* r = o.order.data() + o.pt_off[p];
    const int n = o.pt_off[p + 1] - o.pt_off[p];
    for (int a = 1; a < n; ++a) {
      const int32_t v = r[a];
      int b = a - 1;
      while (b >= 0 && cam[r[b]] > cam[v]) {
        r[b + 1] = r[b];
        --b;
      }
      r[b + 1] = v;
    }
  }
  o.cam_pm.resize(size_t(N));
  o.pt_s.resize(size_t(N));
  for (int64_t q = 0; q < N; ++q) {
    o.cam_pm[q] = cam[o.order[q]];
    o.pt_s[q] = pt[o.order[q]];
  }
  // camera-major order of the point-major ids (stable by camera)
  o.cm_order.resize(size_t(N));
  {
    std::vector<int32_t> cur(cam_off.begin(), cam_off.end() - (C > 0 ? 1 : 0));
    for (int64_t q = 0; q < N; ++q) o.cm_order[cur[o.cam_pm[q]]++] = int32_t(q);
  }
  // Schur pair count: o2 in o1's point run with camera >= c1, o2 != o1
  int64_t n_pairs = 0;
  for (int64_t q = 0; q < N; ++q) {
    const int c1 = o.cam_pm[q], p = o.pt_s[q];
    for (int32_t o2 = o.pt_off[p]; o2 < o.pt_off[p + 1]; ++o2) n_pairs += (o.cam_pm[o2] >= c1 && o2 != q) ? 1 : 0;
  }
  return n_pairs;
}

void host_fill(int64_t N, const double* uv, int C, int P, const HostOrders& o, const std::vector<int32_t>& cam_off,
               const std::vector<int32_t>& cam_rng, const std::vector<int32_t>& wcam, int64_t npad,
               const std::vector<int4>& chunks, int64_t n_pairs, const HostLayoutOut& out) {
  std::memcpy(out.pt_off, o.pt_off.data(), sizeof(int32_t) * (size_t(P) + 1));
  std::memcpy(out.order, o.order.data(), sizeof(int32_t) * size_t(N));
  std::memcpy(out.cam_pm, o.cam_pm.data(), sizeof(int32_t) * size_t(N));
  for (int64_t q = 0; q < N; ++q) {
    out.uv_pm[2 * q] = uv[2 * size_t(o.order[q])];
    out.uv_pm[2 * q + 1] = uv[2 * size_t(o.order[q]) + 1];
  }
  // padded camera-major arrays (k_fill_cm)
  for (int64_t i = 0; i < npad; ++i) {
    const int c = wcam[i >> 6];
    const int32_t j = int32_t(i - cam_rng[2 * c]);
    const int32_t n_c = cam_off[c + 1] - cam_off[c];
    const int32_t q = o.cm_order[cam_off[c] + std::min(j, n_c - 1)];
    out.cm_p[i] = o.pt_s[q];
    out.uv_cm[2 * i] = out.uv_pm[2 * size_t(q)];
    out.uv_cm[2 * i + 1] = out.uv_pm[2 * size_t(q) + 1];
    out.cam_obs[i] = j < n_c ? q : -1;
    if (j < n_c) out.pos[q] = int32_t(i);
  }
  // chunk table grouped by the point slice of a chunk's first observation
  const int nch = int(chunks.size());
  {
    std::vector<uint32_t> key(static_cast<size_t>(nch));
    int32_t cnt[9] = {0};
    for (int t = 0; t < nch; ++t) {
      const int p0 = o.pt_s[o.cm_order[chunks[t].w]];
      key[t] = uint32_t(int64_t(p0) * 8 / std::max(1, P));
      ++cnt[key[t] + 1];
    }
    for (int g = 0; g < 8; ++g) cnt[g + 1] += cnt[g];
    for (int g = 0; g <= 8; ++g) out.jgrp[g] = cnt[g];
    int32_t cur[8];
    std::copy(cnt, cnt + 8, cur);
    for (int t = 0; t < nch; ++t) {
      const int4 v = chunks[t];
      out.jchunks[cur[key[t]]++] = make_int4(v.x, v.y, v.z, 0);
    }
  }
  // Schur pair lists: stable counting sort on the block key
  const int64_t n_blk = int64_t(C) * (C + 1) / 2;
  auto row_start = [C](int c1) { return int64_t(c1) * C - int64_t(c1) * (c1 - 1) / 2; };
  std::fill(out.seg, out.seg + n_blk + 1, 0);
  for (int64_t i = 0; i < N; ++i) {
    const int32_t o1 = o.cm_order[i];
    const int c1 = o.cam_pm[o1], p = o.pt_s[o1];
    const int64_t rs = row_start(c1) - c1;
    for (int32_t o2 = o.pt_off[p]; o2 < o.pt_off[p + 1]; ++o2) {
      const int c2 = o.cam_pm[o2];
      if (c2 >= c1 && o2 != o1) ++out.seg[rs + c2 + 1];
    }
  }
  for (int64_t b = 0; b < n_blk; ++b) out.seg[b + 1] += out.seg[b];
  std::vector<int32_t> cur(out.seg, out.seg + std::max<int64_t>(1, n_blk));
  for (int64_t i = 0; i < N; ++i) {
    const int32_t o1 = o.cm_order[i];
    const int c1 = o.cam_pm[o1], p = o.pt_s[o1];
    const int64_t rs = row_start(c1) - c1;
    for (int32_t o2 = o.pt_off[p]; o2 < o.pt_off[p + 1]; ++o2) {
      const int c2 = o.cam_pm[o2];
      if (c2 >= c1 && o2 != o1) out.bpts[cur[rs + c2]++] = p;
    }
  }
  (void)n_pairs;
  for (int c1 = 0; c1 < C; ++c1)
    for (int c2 = c1; c2 < C; ++c2) out.blk[row_start(c1) - c1 + c2] = make_int2(c1, c2);
}

}  // namespace sfm
