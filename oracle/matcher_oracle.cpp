// ============================================================================
// ORACLE -- TEST INFRASTRUCTURE ONLY (checker / CPU baseline; never in the product).
// CPU restatement of the matcher pieces on the hot path:
//   DescriptorDistance64 / DescriptorDistance64Masked   src/cORBmatcher.cpp:2443-2477
//   best / second-best scan (bestDist/bestDist2 update)  src/cORBmatcher.cpp:67-163
//   SearchForTriangulationRaw (mbCheckOrientation=false) src/cORBmatcher.cpp:968-1156
//   CheckDistEpipolarLine                               src/misc.cpp:54-70
// The distance code is self-contained C in the reference but its file pulls in OpenCV,
// so it is restated, not compiled.  Parity: exact integer equality.
// ============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <utility>
#include <vector>

extern "C" {

int oracle_descriptor_distance64(const uint64_t* a, const uint64_t* b, int dim) {
  uint64_t dist = 0;
  for (int d = 0; d < dim / 8; ++d) dist += __builtin_popcountll(a[d] ^ b[d]);
  return (int)dist;
}

int oracle_descriptor_distance64_masked(const uint64_t* a, const uint64_t* b, const uint64_t* ma,
                                        const uint64_t* mb, int dim) {
  uint64_t dist = 0;
  for (int i = 0; i < dim / 8; ++i) {
    uint64_t x = a[i] ^ b[i];
    dist += __builtin_popcountll(x & ma[i]);
    dist += __builtin_popcountll(x & mb[i]);
  }
  return (int)(dist / 2);
}

// out: best_idx, best_dist, second_dist per query (second_idx implied by scan order)
int oracle_hamming_top2(const uint8_t* q, int nq, const uint8_t* t, int nt, int bytes,
                        int* best_idx, int* best_dist, int* second_dist) {
  for (int i = 0; i < nq; i++) {
    int b1 = 0x7FFFFFFF, b2 = 0x7FFFFFFF, i1 = -1;
    for (int j = 0; j < nt; j++) {
      int d = oracle_descriptor_distance64((const uint64_t*)(q + (size_t)i * bytes),
                                           (const uint64_t*)(t + (size_t)j * bytes), bytes);
      if (d < b1) { b2 = b1; b1 = d; i1 = j; }
      else if (d < b2) b2 = d;
    }
    best_idx[i] = i1;
    best_dist[i] = i1 < 0 ? 8 * bytes + 1 : b1;
    second_dist[i] = b2 == 0x7FFFFFFF ? 8 * bytes + 1 : b2;
  }
  return 0;
}

static bool check_dist_epipolar_line(const double* r1, const double* r2, const double* E,
                                     double thresh) {
  // nom = ray2^T * E * ray1 ; Ex1 = E*ray1 ; Etx2 = E^T*ray2
  double Ex1[3], Etx2[3];
  for (int r = 0; r < 3; r++) {
    Ex1[r] = E[3 * r] * r1[0] + E[3 * r + 1] * r1[1] + E[3 * r + 2] * r1[2];
    Etx2[r] = E[r] * r2[0] + E[3 + r] * r2[1] + E[6 + r] * r2[2];
  }
  double nom = r2[0] * Ex1[0] + r2[1] * Ex1[1] + r2[2] * Ex1[2];
  double den = Ex1[0] * Ex1[0] + Ex1[1] * Ex1[1] + Ex1[2] * Ex1[2] + Etx2[0] * Etx2[0] +
               Etx2[1] * Etx2[1] + Etx2[2] * Etx2[2];
  if (den == 0.0) return false;
  return (nom * nom) / den < thresh;
}

int oracle_search_for_triangulation_raw(const uint8_t* desc1, int n1, const uint8_t* desc2,
                                        int n2, int bytes, const int* cam1, const int* cam2,
                                        const uint8_t* has_mp1, const uint8_t* has_mp2,
                                        const double* rays1, const double* rays2,
                                        const double* E /* ncams x ncams x 9 */, double thresh,
                                        int ncams, int* matches12) {
  const int TH_LOW = 2 * bytes;  // cORBmatcher ctor without masks (:61-63)
  std::vector<bool> vbMatched2(n2, false);
  int nmatches = 0;
  for (int i = 0; i < n1; i++) matches12[i] = -1;
  for (int idx1 = 0; idx1 < n1; ++idx1) {
    if (has_mp1[idx1]) continue;
    std::vector<std::pair<int, size_t>> vDistIndex;
    std::vector<int> vDistCamIndex;
    for (int idx2 = 0; idx2 < n2; ++idx2) {
      if (vbMatched2[idx2] || has_mp2[idx2]) continue;
      if (cam1[idx1] != cam2[idx2]) continue;
      int dist = oracle_descriptor_distance64((const uint64_t*)(desc1 + (size_t)idx1 * bytes),
                                              (const uint64_t*)(desc2 + (size_t)idx2 * bytes), bytes);
      if (dist > TH_LOW) continue;
      vDistIndex.push_back(std::make_pair(dist, (size_t)idx2));
      vDistCamIndex.push_back(cam2[idx2]);
    }
    if (vDistIndex.empty()) continue;
    std::sort(vDistIndex.begin(), vDistIndex.end());
    int BestDist = vDistIndex.front().first;
    int DistTh = (int)std::lrint(2.0 * BestDist);
    for (size_t id = 0; id < vDistIndex.size(); ++id) {
      if (vDistIndex[id].first > DistTh) break;
      int currentIdx2 = (int)vDistIndex[id].second;
      int c2 = cam2[currentIdx2];
      if (check_dist_epipolar_line(rays1 + 3 * (size_t)idx1, rays2 + 3 * (size_t)currentIdx2,
                                   E + 9 * ((size_t)cam1[idx1] * ncams + c2), thresh)) {
        vbMatched2[currentIdx2] = true;
        matches12[idx1] = currentIdx2;
        nmatches++;
        break;
      }
    }
  }
  return nmatches;
}

}  // extern "C"
