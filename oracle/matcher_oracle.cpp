// ============================================================================
// ORACLE -- TEST INFRASTRUCTURE ONLY (checker / CPU baseline; never in the product).
// CPU restatement of the matcher pieces on the hot path:
//   DescriptorDistance64 / DescriptorDistance64Masked   src/cORBmatcher.cpp:2443-2477
//   best / second-best scan (bestDist/bestDist2 update)  src/cORBmatcher.cpp:67-163
//   SearchForTriangulationRaw (mbCheckOrientation=false) src/cORBmatcher.cpp:968-1156
//   CheckDistEpipolarLine                               src/misc.cpp:54-70
//   cMultiFrame grid + GetFeaturesInArea                src/cMultiFrame.cpp:154-184, 272-353
//   windowed searches (SearchByProjection x2, SearchForInitialization, WindowSearch)
//                                                       src/cORBmatcher.cpp:67-166, 326-473,
//                                                       579-726, 1991-2123
// The distance code is self-contained C in the reference but its file pulls in OpenCV,
// so it is restated, not compiled.  Parity: exact integer equality.
// ============================================================================
#include <algorithm>
#include <climits>
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

// cv::Matx products accumulate s = 0; s += a(i,k) * b(k,j) for k = 0.. (Matx_MatMulOp).
static void matx_mul(const double* a, const double* b, double* c, int m, int l, int n) {
  for (int i = 0; i < m; i++)
    for (int j = 0; j < n; j++) {
      double s = 0;
      for (int k = 0; k < l; k++) s += a[i * l + k] * b[k * n + j];
      c[i * n + j] = s;
    }
}

static bool check_dist_epipolar_line(const double* r1, const double* r2, const double* E,
                                     double thresh) {
  // nom = ray2.t() * E12 * ray1 (left to right); Ex1 = E12 * ray1; Etx2 = E12.t() * ray2
  double r2tE[3], nom, Ex1[3], Et[9], Etx2[3];
  matx_mul(r2, E, r2tE, 1, 3, 3);
  matx_mul(r2tE, r1, &nom, 1, 3, 1);
  matx_mul(E, r1, Ex1, 3, 3, 1);
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) Et[3 * r + c] = E[3 * c + r];
  matx_mul(Et, r2, Etx2, 3, 3, 1);
  const double den = Ex1[0] * Ex1[0] + Ex1[1] * Ex1[1] + Ex1[2] * Ex1[2] + Etx2[0] * Etx2[0] +
                     Etx2[1] * Etx2[1] + Etx2[2] * Etx2[2];
  if (den == 0.0) return false;
  const double dsqr = (nom * nom) / den;
  return dsqr < thresh;
}

int oracle_check_dist_epipolar_line(const double* r1, const double* r2, const double* E,
                                    double thresh, double* dsqr) {
  // as check_dist_epipolar_line, also reporting dsqr (NaN when den == 0)
  double r2tE[3], nom, Ex1[3], Et[9], Etx2[3];
  matx_mul(r2, E, r2tE, 1, 3, 3);
  matx_mul(r2tE, r1, &nom, 1, 3, 1);
  matx_mul(E, r1, Ex1, 3, 3, 1);
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) Et[3 * r + c] = E[3 * c + r];
  matx_mul(Et, r2, Etx2, 3, 3, 1);
  const double den = Ex1[0] * Ex1[0] + Ex1[1] * Ex1[1] + Ex1[2] * Ex1[2] + Etx2[0] * Etx2[0] +
                     Etx2[1] * Etx2[1] + Etx2[2] * Etx2[2];
  if (dsqr) *dsqr = den == 0.0 ? NAN : (nom * nom) / den;
  return check_dist_epipolar_line(r1, r2, E, thresh) ? 1 : 0;
}

// masks1 / masks2 nullable: the cORBmatcher was built with havingMasks (mdBRIEF), which also
// selects the thresholds TH_LOW = floor(featDim) instead of 2 * featDim (:52-65).
int oracle_search_for_triangulation_raw_ex(const uint8_t* desc1, const uint8_t* masks1, int n1,
                                           const uint8_t* desc2, const uint8_t* masks2, int n2,
                                           int bytes, const int* cam1, const int* cam2,
                                           const uint8_t* has_mp1, const uint8_t* has_mp2,
                                           const double* rays1, const double* rays2,
                                           const double* E /* ncams x ncams x 9 */,
                                           double thresh, int ncams, int* matches12) {
  const bool havingMasks = masks1 != nullptr && masks2 != nullptr;
  const int TH_LOW = havingMasks ? (int)std::floor((double)bytes) : 2 * bytes;
  std::vector<bool> vbMatched2(n2, false);
  int nmatches = 0;
  for (int i = 0; i < n1; i++) matches12[i] = -1;
  for (int idx1 = 0; idx1 < n1; ++idx1) {
    if (has_mp1[idx1]) continue;
    const uint64_t* d1 = (const uint64_t*)(desc1 + (size_t)idx1 * bytes);
    const uint64_t* m1 = havingMasks ? (const uint64_t*)(masks1 + (size_t)idx1 * bytes) : nullptr;
    std::vector<std::pair<int, size_t>> vDistIndex;
    std::vector<int> vDistCamIndex;
    for (int idx2 = 0; idx2 < n2; ++idx2) {
      if (vbMatched2[idx2] || has_mp2[idx2]) continue;
      if (cam1[idx1] != cam2[idx2]) continue;
      const uint64_t* d2 = (const uint64_t*)(desc2 + (size_t)idx2 * bytes);
      int dist = havingMasks
          ? oracle_descriptor_distance64_masked(d1, d2, m1,
                (const uint64_t*)(masks2 + (size_t)idx2 * bytes), bytes)
          : oracle_descriptor_distance64(d1, d2, bytes);
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

int oracle_search_for_triangulation_raw(const uint8_t* desc1, int n1, const uint8_t* desc2,
                                        int n2, int bytes, const int* cam1, const int* cam2,
                                        const uint8_t* has_mp1, const uint8_t* has_mp2,
                                        const double* rays1, const double* rays2,
                                        const double* E, double thresh, int ncams,
                                        int* matches12) {
  return oracle_search_for_triangulation_raw_ex(desc1, nullptr, n1, desc2, nullptr, n2, bytes,
                                                cam1, cam2, has_mp1, has_mp2, rays1, rays2, E,
                                                thresh, ncams, matches12);
}

}  // extern "C"

// ---- projection-guided (windowed) matching ------------------------------------------------
// The cMultiFrame grid as the reference keeps it, mGrids[cam][ix][iy] = keypoint indices in
// push_back order (src/cMultiFrame.cpp:154-184, PosInGrid :342-353, 64 x 48 cells), the literal
// GetFeaturesInArea loops (:272-340), and the selection loops of the four windowed searches
// with mbCheckOrientation = false.  A query is one GetFeaturesInArea call: (x, y, r),
// (cam, minLevel, maxLevel) and its descriptor (+ mask when mdBRIEF masks are learned).
namespace {

struct OFrame {
  int ncams = 0, bytes = 0;
  std::vector<int> minx, miny;                 // mnMinX / mnMinY are ints in the reference
  std::vector<double> winv, hinv;              // mfGridElementWidthInv / HeightInv
  std::vector<std::vector<int>> cells;         // [(cam * 64 + ix) * 48 + iy]
  const float* xy = nullptr;
  const int* oct = nullptr;
  const uint8_t* desc = nullptr;
  const uint8_t* mask = nullptr;
};

void o_frame(OFrame& F, int ncams, const double* gp, const float* xy, const int* cam,
             const int* oct, const uint8_t* desc, const uint8_t* mask, int n, int bytes) {
  F.ncams = ncams; F.bytes = bytes; F.xy = xy; F.oct = oct; F.desc = desc; F.mask = mask;
  for (int c = 0; c < ncams; c++) {
    F.minx.push_back((int)gp[4 * c]);
    F.miny.push_back((int)gp[4 * c + 1]);
    F.winv.push_back(gp[4 * c + 2]);
    F.hinv.push_back(gp[4 * c + 3]);
  }
  F.cells.assign((size_t)ncams * 64 * 48, std::vector<int>());
  for (int i = 0; i < n; i++) {
    const int c = cam[i];
    if (c < 0 || c >= ncams) continue;
    const int posX = (int)std::lrint((xy[2 * i] - F.minx[c]) * F.winv[c]);
    const int posY = (int)std::lrint((xy[2 * i + 1] - F.miny[c]) * F.hinv[c]);
    if (posX < 0 || posX >= 64 || posY < 0 || posY >= 48) continue;
    F.cells[((size_t)c * 64 + posX) * 48 + posY].push_back(i);
  }
}

std::vector<int> o_features_in_area(const OFrame& F, int cam, double x, double y, double r,
                                    int minLevel, int maxLevel) {
  std::vector<int> v;
  int nMinCellX = (int)std::floor((x - F.minx[cam] - r) * F.winv[cam]);
  nMinCellX = std::max(0, nMinCellX);
  if (nMinCellX >= 64) return v;
  int nMaxCellX = (int)std::ceil((x - F.minx[cam] + r) * F.winv[cam]);
  nMaxCellX = std::min(64 - 1, nMaxCellX);
  if (nMaxCellX < 0) return v;
  int nMinCellY = (int)std::floor((y - F.miny[cam] - r) * F.hinv[cam]);
  nMinCellY = std::max(0, nMinCellY);
  if (nMinCellY >= 48) return v;
  int nMaxCellY = (int)std::ceil((y - F.miny[cam] + r) * F.hinv[cam]);
  nMaxCellY = std::min(48 - 1, nMaxCellY);
  if (nMaxCellY < 0) return v;
  bool bCheckLevels = true, bSameLevel = false;
  if (minLevel == -1 && maxLevel == -1) bCheckLevels = false;
  else if (minLevel == maxLevel) bSameLevel = true;
  for (int ix = nMinCellX; ix <= nMaxCellX; ++ix)
    for (int iy = nMinCellY; iy <= nMaxCellY; ++iy)
      for (int k : F.cells[((size_t)cam * 64 + ix) * 48 + iy]) {
        if (bCheckLevels && !bSameLevel) {
          if (F.oct[k] < minLevel || F.oct[k] > maxLevel) continue;
        } else if (bSameLevel) {
          if (F.oct[k] != minLevel) continue;
        }
        if (std::fabs(F.xy[2 * k] - x) > r || std::fabs(F.xy[2 * k + 1] - y) > r) continue;
        v.push_back(k);
      }
  return v;
}

int o_dist(const OFrame& F, const uint8_t* qd, const uint8_t* qm, int k) {
  const uint64_t* a = reinterpret_cast<const uint64_t*>(qd);
  const uint64_t* b = reinterpret_cast<const uint64_t*>(F.desc + (size_t)k * F.bytes);
  if (!qm) return oracle_descriptor_distance64(a, b, F.bytes);
  return oracle_descriptor_distance64_masked(a, b, reinterpret_cast<const uint64_t*>(qm),
                                             reinterpret_cast<const uint64_t*>(F.mask + (size_t)k * F.bytes),
                                             F.bytes);
}

}  // namespace

extern "C" {

// grid as CSR: cell_ptr [ncams*64*48 + 1], cell_kp [n]; returns the number of keypoints kept
int oracle_frame_grid(int ncams, const double* gp, const float* xy, const int* cam, int n,
                      int* cell_ptr, int* cell_kp) {
  OFrame F;
  o_frame(F, ncams, gp, xy, cam, nullptr, nullptr, nullptr, n, 0);
  int k = 0;
  for (size_t c = 0; c < F.cells.size(); c++) {
    cell_ptr[c] = k;
    for (int v : F.cells[c]) cell_kp[k++] = v;
  }
  cell_ptr[F.cells.size()] = k;
  return k;
}

// every query's GetFeaturesInArea list with distances (CSR); returns the total (entries past
// cap are counted, not written)
int oracle_window_candidates(int ncams, const double* gp, const float* xy, const int* cam,
                             const int* oct, const uint8_t* desc, const uint8_t* mask, int n,
                             int bytes, int nq, const double* q_xyr, const int* q_cl,
                             const uint8_t* q_desc, const uint8_t* q_mask, int* cand_ptr,
                             int* cand_kp, int* cand_dist, int cap) {
  OFrame F;
  o_frame(F, ncams, gp, xy, cam, oct, desc, mask, n, bytes);
  int k = 0;
  for (int q = 0; q < nq; q++) {
    cand_ptr[q] = k;
    const std::vector<int> v = o_features_in_area(F, q_cl[3 * q], q_xyr[3 * q], q_xyr[3 * q + 1],
                                                  q_xyr[3 * q + 2], q_cl[3 * q + 1], q_cl[3 * q + 2]);
    for (int i : v) {
      if (k < cap) {
        cand_kp[k] = i;
        cand_dist[k] = o_dist(F, q_desc + (size_t)q * bytes, q_mask ? q_mask + (size_t)q * bytes : nullptr, i);
      }
      k++;
    }
  }
  cand_ptr[nq] = k;
  return k;
}

// rule 0 SearchByProjection(F, MPs) :67-166, rule 1 SearchByProjection(Current, Last)
// :1991-2123, rule 2 SearchForInitialization :579-726, rule 3 WindowSearch :326-473.
// assigned [n] in/out (F.mvpMapPoints != NULL / vpMapPointMatches2), match [nq] out.
int oracle_window_match(int rule, int ncams, const double* gp, const float* xy, const int* cam,
                        const int* oct, const uint8_t* desc, const uint8_t* mask, int n, int bytes,
                        int nq, const double* q_xyr, const int* q_cl, const uint8_t* q_desc,
                        const uint8_t* q_mask, int th, double nnratio, uint8_t* assigned,
                        int* match) {
  OFrame F;
  o_frame(F, ncams, gp, xy, cam, oct, desc, mask, n, bytes);
  int nmatches = 0;
  std::vector<int> vMatchedDistance(n, INT_MAX), vnMatches21(n, -1);
  for (int q = 0; q < nq; q++) match[q] = -1;
  for (int q = 0; q < nq; q++) {
    const std::vector<int> vIdx = o_features_in_area(F, q_cl[3 * q], q_xyr[3 * q], q_xyr[3 * q + 1],
                                                     q_xyr[3 * q + 2], q_cl[3 * q + 1], q_cl[3 * q + 2]);
    if (vIdx.empty()) continue;
    const uint8_t* qd = q_desc + (size_t)q * bytes;
    const uint8_t* qm = q_mask ? q_mask + (size_t)q * bytes : nullptr;
    int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx = -1, bestLevel = -1, bestLevel2 = -1;
    if (rule == 2) {
      for (int i2 : vIdx) {
        const int dist = o_dist(F, qd, qm, i2);
        if (vMatchedDistance[i2] <= dist) continue;
        if (dist < bestDist) { bestDist2 = bestDist; bestDist = dist; bestIdx = i2; }
        else if (dist < bestDist2) bestDist2 = dist;
      }
      if (bestDist <= th && bestDist < (double)bestDist2 * nnratio) {
        if (vnMatches21[bestIdx] >= 0) { match[vnMatches21[bestIdx]] = -1; nmatches--; }
        match[q] = bestIdx;
        vnMatches21[bestIdx] = q;
        vMatchedDistance[bestIdx] = bestDist;
        nmatches++;
      }
      continue;
    }
    for (int idx : vIdx) {
      if (assigned[idx]) continue;
      const int dist = o_dist(F, qd, qm, idx);
      if (rule == 1) {
        if (dist < bestDist) { bestDist = dist; bestIdx = idx; }
        continue;
      }
      if (dist < bestDist) {
        bestDist2 = bestDist; bestDist = dist;
        bestLevel2 = bestLevel; bestLevel = F.oct[idx];
        bestIdx = idx;
      } else if (dist < bestDist2) {
        bestLevel2 = F.oct[idx];
        bestDist2 = dist;
      }
    }
    bool accept = false;
    if (rule == 0) accept = bestDist <= th && !(bestLevel == bestLevel2 && bestDist > nnratio * bestDist2);
    else if (rule == 1) accept = bestDist <= th;
    else accept = bestDist <= bestDist2 * nnratio && bestDist <= th;
    if (accept) {
      assigned[bestIdx] = 1;
      match[q] = bestIdx;
      nmatches++;
    }
  }
  return nmatches;
}

}  // extern "C"
