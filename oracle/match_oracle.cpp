// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY (see ba_oracle.cpp header).
//
// Restatement of the reference's per-frame feature matcher:
//   CTracker::matchFeatures(pts0, desc0, pts1, desc1, idx0, idx1, min, max)
//     /root/reference/CTracker.cpp:211-250  (T3)
//   CTracker::matchFeatures(pts0, desc0, pts1, desc1, idx0, idx1)
//     CTracker.cpp:114-149 (T4, member window 1.5 / 40 px, CTracker.cpp:30-31)
//   CTracker::matchFeatures(prevIdx, currIdx, prevMatchIdx, currMatchIdx)
//     CTracker.cpp:368-417 (T2: same rule on index-gathered subsets)
//   CTracker::matchFeatures() CTracker.cpp:419-477 (T4 on the member frames)
// and of the external 2-NN search they call, brisk::BruteForceMatcher::knnMatch
// (k = 2, Hamming; CTracker.cpp:117, 214, 381, 433), whose library is not
// vendored.  Restated knnMatch semantics: integer Hamming
// distance over the descriptor bytes, reported as float (DMatch::distance);
// ties broken by the lower train index (OpenCV brute-force convention; the
// BRISK tie order itself is unpinned).
//
// Sequential resolution (CTracker.cpp:221-249), restated verbatim:
//   ratio   = float(d0) / float(d1)               (float division)
//   d       = |pts0[i] - pts1[j0]|^2              (double)
//   accept  = d > min^2 && d < max^2 && ratio < 0.8 &&
//             (j0 unmatched || d0 < bestDist[j0])
//   new j0  -> append (i, j0);  improved j0 -> overwrite the query index at
//   j0's original slot.
// Reference UB: with fewer than 2 train rows
// matches[i][1] is read out of range.  Restated as "no matches".
//
// Also CMap::getRepresentativeDescriptors (CMap.cpp:345-381), below.
//
// PARITY UNPINNED: no reference test or fixture covers the matcher.
// ============================================================================
#include <cstdint>
#include <cstring>
#include <vector>

extern "C" {

static inline int hamming(const uint8_t* a, const uint8_t* b, int nbytes) {
  int d = 0;
  int k = 0;
  for (; k + 8 <= nbytes; k += 8) {
    uint64_t x, y;
    std::memcpy(&x, a + k, 8);
    std::memcpy(&y, b + k, 8);
    d += __builtin_popcountll(x ^ y);
  }
  for (; k < nbytes; ++k) d += __builtin_popcount(unsigned(a[k] ^ b[k]));
  return d;
}

// 2-NN by Hamming distance: best/second train index and distance per query.
int oracle_knn2_hamming(const uint8_t* desc0, int32_t n0, const uint8_t* desc1, int32_t n1, int32_t nbytes,
                        int32_t* best_idx, int32_t* best_dist, int32_t* second_idx, int32_t* second_dist) {
  for (int i = 0; i < n0; ++i) {
    int d0 = 1 << 30, j0 = -1, d1 = 1 << 30, j1 = -1;
    const uint8_t* q = desc0 + size_t(i) * nbytes;
    for (int j = 0; j < n1; ++j) {
      const int d = hamming(q, desc1 + size_t(j) * nbytes, nbytes);
      if (d < d0) { d1 = d0; j1 = j0; d0 = d; j0 = j; }
      else if (d < d1) { d1 = d; j1 = j; }
    }
    best_idx[i] = j0; best_dist[i] = d0; second_idx[i] = j1; second_dist[i] = d1;
  }
  return 0;
}

// Returns the number of matches written to idx0/idx1 (capacity >= min(n0,n1)).
int oracle_match_features(const double* pts0, const uint8_t* desc0, int32_t n0, const double* pts1,
                          const uint8_t* desc1, int32_t n1, int32_t nbytes, double ratio_test, double min_distance,
                          double max_distance, int32_t* idx0, int32_t* idx1) {
  if (n0 <= 0 || n1 < 2) return 0;
  std::vector<int32_t> bi(n0), bd(n0), si(n0), sd(n0);
  oracle_knn2_hamming(desc0, n0, desc1, n1, nbytes, bi.data(), bd.data(), si.data(), sd.data());
  std::vector<double> matchDistance(n1, -1.0);
  std::vector<int> matchedIdx(n1, -1);
  const double minSq = min_distance * min_distance, maxSq = max_distance * max_distance;
  int matchCount = 0;
  for (int i = 0; i < n0; ++i) {
    const int prevIdx = i, currIdx = bi[i];
    const float f0 = float(bd[i]), f1 = float(sd[i]);
    const double ratio = f0 / f1;
    const double dx = pts0[2 * prevIdx] - pts1[2 * currIdx], dy = pts0[2 * prevIdx + 1] - pts1[2 * currIdx + 1];
    const double d = dx * dx + dy * dy;
    const bool minDist = d > minSq, maxDist = d < maxSq, crossRatio = ratio < ratio_test;
    const bool newMatch = matchDistance[currIdx] == -1;
    const bool betterMatch = f0 < matchDistance[currIdx];
    if (minDist && maxDist && crossRatio && (newMatch || betterMatch)) {
      if (newMatch) {
        idx0[matchCount] = prevIdx;
        idx1[matchCount] = currIdx;
        matchedIdx[currIdx] = matchCount;
        ++matchCount;
      } else {
        idx0[matchedIdx[currIdx]] = prevIdx;
      }
      matchDistance[currIdx] = f0;
    }
  }
  return matchCount;
}

// CMap::getRepresentativeDescriptors (/root/reference/CMap.cpp:345-381),
// restated: per point, the symmetric Hamming distance matrix of its rows
// (NORM_HAMMING, float), column sums (reduce dim 0), then the first row with
// the strictly smallest sum.  Returns -1 if a point has no rows (the
// reference would read row -1).
int oracle_representative_descriptors(const uint8_t* desc, const int32_t* row_off, int32_t n_pts, int32_t nbytes,
                                      int32_t* best) {
  for (int32_t i = 0; i < n_pts; ++i) {
    const int32_t r0 = row_off[i], k = row_off[i + 1] - r0;
    if (k <= 0) return -1;
    std::vector<float> dist(size_t(k) * k, 0.0f);
    for (int j = 0; j < k; ++j)
      for (int q = j + 1; q < k; ++q) {
        const float d = float(hamming(desc + size_t(r0 + j) * nbytes, desc + size_t(r0 + q) * nbytes, nbytes));
        dist[size_t(j) * k + q] = d;
        dist[size_t(q) * k + j] = d;
      }
    int min_idx = -1;
    float min_d = 3.402823466e+38f;
    for (int c = 0; c < k; ++c) {
      float s = 0.0f;
      for (int j = 0; j < k; ++j) s += dist[size_t(j) * k + c];
      if (s < min_d) {
        min_d = s;
        min_idx = c;
      }
    }
    best[i] = min_idx;
  }
  return 0;
}

}  // extern "C"
