// ============================================================================
// ORACLE -- TEST INFRASTRUCTURE ONLY (checker; never in the product).
// CPU restatement of the map-point refresh LocalBundleAdjustment runs after its write-back
// (src/cOptimizer.cpp:885-902):
//   cMapPoint::ComputeDistinctiveDescriptors  src/cMapPoint.cpp:297-390, literally: the full
//     N x N distance matrix, the upper-triangle row of every i < N-1 and median() of
//     include/misc.h:97-105 (std::nth_element at size/2), first strict minimum wins
//   cMapPoint::UpdateNormalAndDepth           src/cMapPoint.cpp:453-496 with cv::Vec3d
//     semantics [ext, OpenCV]: v / a == v * (1. / a), cv::norm = sqrt of the in-order sum of
//     squares
// ============================================================================
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <vector>

extern "C" int oracle_descriptor_distance64(const uint64_t* a, const uint64_t* b, int dim);
extern "C" int oracle_descriptor_distance64_masked(const uint64_t* a, const uint64_t* b,
                                                   const uint64_t* ma, const uint64_t* mb, int dim);

namespace {
template <typename T>
T median(std::vector<T>& v) {   // include/misc.h:97-105
  if (v.size() > 0) {
    std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
    return v[v.size() / 2];
  }
  return T(0);
}

double vnorm(const double* v) {
  double s = 0;
  for (int k = 0; k < 3; k++) s += v[k] * v[k];
  return std::sqrt(s);
}
}  // namespace

extern "C" {

// descriptors desc [rows][bytes] (masks nullable), per point the rows obs_row[obs_ptr[p]..);
// best[p] = chosen index within the point's list (-1: no descriptor)
int oracle_distinctive_descriptors(const uint8_t* desc, const uint8_t* masks, int bytes,
                                   const int* obs_ptr, const int* obs_row, int n_points,
                                   int* best) {
  for (int p = 0; p < n_points; p++) {
    const int q0 = obs_ptr[p];
    const size_t N = (size_t)(obs_ptr[p + 1] - q0);
    if (N == 0) { best[p] = -1; continue; }
    auto row = [&](const uint8_t* base, size_t i) {
      return reinterpret_cast<const uint64_t*>(base + (size_t)obs_row[q0 + i] * bytes);
    };
    std::vector<int> D(N * N, 0);
    for (size_t i = 0; i < N; ++i)
      for (size_t j = i + 1; j < N; ++j) {
        const int dij = masks ? oracle_descriptor_distance64_masked(row(desc, i), row(desc, j),
                                                                    row(masks, i), row(masks, j), bytes)
                              : oracle_descriptor_distance64(row(desc, i), row(desc, j), bytes);
        D[i * N + j] = dij;
        D[j * N + i] = dij;
      }
    int BestMedian = INT_MAX, BestIdx = 0;
    if (N > 2) {
      for (size_t i = 0; i < N - 1; ++i) {
        std::vector<int> vDists;
        for (size_t j = i + 1; j < N; ++j) vDists.push_back(D[i * N + j]);
        const int medianV = median(vDists);
        if (medianV < BestMedian) {
          BestMedian = medianV;
          BestIdx = (int)i;
        }
      }
    }
    best[p] = BestIdx;
  }
  return 0;
}

int oracle_update_normal_depth(const double* pts, int n, const int* obs_ptr, const int* obs_kf,
                               const double* kf_c, const int* ref_kf, const int* ref_level,
                               const double* scale, int nlev, double* normal, double* dmin,
                               double* dmax) {
  for (int p = 0; p < n; p++) {
    if (obs_ptr[p + 1] <= obs_ptr[p]) continue;
    const double* X = pts + 3 * p;
    double nrm[3] = {0, 0, 0};
    int cnt = 0;
    for (int q = obs_ptr[p]; q < obs_ptr[p + 1]; q++) {
      const double* O = kf_c + 3 * obs_kf[q];
      const double ni[3] = {X[0] - O[0], X[1] - O[1], X[2] - O[2]};
      const double ia = 1. / vnorm(ni);   // normali / cv::norm(normali)
      for (int k = 0; k < 3; k++) nrm[k] = nrm[k] + ni[k] * ia;
      ++cnt;
    }
    const double* R = kf_c + 3 * ref_kf[p];
    const double PC[3] = {X[0] - R[0], X[1] - R[1], X[2] - R[2]};
    const double dist = vnorm(PC);
    const int level = ref_level[p] >= 0 ? ref_level[p] : 1;
    const double scaleFactor = scale[level], levelScaleFactor = scale[level];
    dmin[p] = (1.0 / scaleFactor) * dist / levelScaleFactor;
    dmax[p] = scaleFactor * dist * scale[nlev - 1 - level];
    const double in = 1. / cnt;   // normal / n
    for (int k = 0; k < 3; k++) normal[3 * p + k] = nrm[k] * in;
  }
  return 0;
}

}  // extern "C"
