// Map-point refresh after LocalBundleAdjustment's write-back, batched over points
// (include/mcs_mappoint.h):
//   cMapPoint::ComputeDistinctiveDescriptors  src/cMapPoint.cpp:297-390 (median: include/misc.h:97-105)
//   cMapPoint::UpdateNormalAndDepth           src/cMapPoint.cpp:453-496
#include "common.hpp"
#include "../../include/mcs_mappoint.h"

namespace mcs {
namespace {

// DescriptorDistance64[Masked] (src/cORBmatcher.cpp:2443-2477) of two rows of NW dwords
template <int NW, bool MASKED>
__device__ __forceinline__ int row_dist(const uint32_t* a, const uint32_t* b, const uint32_t* ma,
                                        const uint32_t* mb) {
  int s = 0;
  if (MASKED) {
    int s1 = 0, s2 = 0;
#pragma unroll
    for (int k = 0; k < NW; k++) {
      const uint32_t x = a[k] ^ b[k];
      s1 += __popc(x & ma[k]);
      s2 += __popc(x & mb[k]);
    }
    s = (s1 + s2) / 2;
  } else {
#pragma unroll
    for (int k = 0; k < NW; k++) s += __popc(a[k] ^ b[k]);
  }
  return s;
}

// One wave per point.  Row i of the upper triangle (distances to the later descriptors j > i,
// m = N - 1 - i of them) is spread over the lanes, 64 columns at a time; its median is the
// element of rank m >> 1 (std::nth_element at size/2), found by bisection on the distance
// value with ballot counts (distances lie in [0, 8 * bytes]).  The first row with the
// smallest median wins (strict <, rows in order), as the reference's loop.
template <int NW, bool MASKED>
__global__ __launch_bounds__(256) void k_distinctive(const uint8_t* __restrict__ desc,
                                                     const uint8_t* __restrict__ masks,
                                                     const int32_t* __restrict__ obs_ptr,
                                                     const int32_t* __restrict__ obs_row,
                                                     int n_points, int32_t* __restrict__ best,
                                                     uint8_t* __restrict__ out_desc,
                                                     uint8_t* __restrict__ out_mask) {
  const int p = blockIdx.x * 4 + (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (p >= n_points) return;
  const int q0 = obs_ptr[p], N = obs_ptr[p + 1] - q0;
  const int bytes = 4 * NW;
  auto rowp = [&](const uint8_t* base, int i) {
    return reinterpret_cast<const uint32_t*>(base + (int64_t)obs_row[q0 + i] * bytes);
  };
  if (N == 0) {
    if (lane == 0) best[p] = -1;
    return;
  }
  int bi = 0;
  if (N > 2) {
    int bmed = 0x7FFFFFFF;
    for (int i = 0; i < N - 1; i++) {
      uint32_t di[NW], mi[NW];
      const uint32_t* ri = rowp(desc, i);
#pragma unroll
      for (int k = 0; k < NW; k++) di[k] = ri[k];
      if (MASKED) {
        const uint32_t* rm = rowp(masks, i);
#pragma unroll
        for (int k = 0; k < NW; k++) mi[k] = rm[k];
      }
      const int m = N - 1 - i, kth = m >> 1;
      // the row's distances, chunk c in register c (rows beyond 64 x kChunks: loop below)
      int lo = 0, hi = 8 * bytes;   // smallest v with #{d <= v} > kth lies in [lo, hi]
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        int cnt = 0;
        for (int j0 = i + 1; j0 < N; j0 += 64) {
          const int j = j0 + lane;
          bool le = false;
          if (j < N) {
            uint32_t dj[NW], mj[NW];
            const uint32_t* rj = rowp(desc, j);
#pragma unroll
            for (int k = 0; k < NW; k++) dj[k] = rj[k];
            if (MASKED) {
              const uint32_t* rmj = rowp(masks, j);
#pragma unroll
              for (int k = 0; k < NW; k++) mj[k] = rmj[k];
            }
            le = row_dist<NW, MASKED>(di, dj, mi, mj) <= mid;
          }
          cnt += __popcll(__ballot(le));
        }
        if (cnt > kth) hi = mid; else lo = mid + 1;
      }
      if (lo < bmed) { bmed = lo; bi = i; }
    }
  }
  if (lane == 0) best[p] = bi;
  if (out_desc && lane < NW) {
    reinterpret_cast<uint32_t*>(out_desc + (int64_t)p * bytes)[lane] = rowp(desc, bi)[lane];
    if (MASKED && out_mask)
      reinterpret_cast<uint32_t*>(out_mask + (int64_t)p * bytes)[lane] = rowp(masks, bi)[lane];
  }
}

// cv::norm of a Vec3d: sqrt of the in-order sum of squares (normL2Sqr)
__device__ __forceinline__ double norm3(double x, double y, double z) {
  double s = 0.0;
  s = __dadd_rn(s, __dmul_rn(x, x));
  s = __dadd_rn(s, __dmul_rn(y, y));
  s = __dadd_rn(s, __dmul_rn(z, z));
  return __dsqrt_rn(s);
}

// one thread per point, the reference's cv::Vec3d arithmetic: v / a is v * (1. / a)
// (Vec operator/ -> Matx_ScaleOp), sums in observation order
__global__ __launch_bounds__(256) void k_normal_depth(const double* __restrict__ pts, int n,
                                                      const int32_t* __restrict__ obs_ptr,
                                                      const int32_t* __restrict__ obs_kf,
                                                      const double* __restrict__ kf_c,
                                                      const int32_t* __restrict__ ref_kf,
                                                      const int32_t* __restrict__ ref_level,
                                                      const double* __restrict__ scale, int nlev,
                                                      double* __restrict__ normal,
                                                      double* __restrict__ dmin,
                                                      double* __restrict__ dmax) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= n) return;
  const int q0 = obs_ptr[p], q1 = obs_ptr[p + 1];
  if (q1 <= q0) return;
  const double X = pts[3 * p], Y = pts[3 * p + 1], Z = pts[3 * p + 2];
  double nx = 0.0, ny = 0.0, nz = 0.0;
  int cnt = 0;
  for (int q = q0; q < q1; q++) {
    const double* O = kf_c + 3 * (int64_t)obs_kf[q];
    const double ax = __dsub_rn(X, O[0]), ay = __dsub_rn(Y, O[1]), az = __dsub_rn(Z, O[2]);
    const double ia = __ddiv_rn(1.0, norm3(ax, ay, az));
    nx = __dadd_rn(nx, __dmul_rn(ax, ia));
    ny = __dadd_rn(ny, __dmul_rn(ay, ia));
    nz = __dadd_rn(nz, __dmul_rn(az, ia));
    ++cnt;
  }
  const double* R = kf_c + 3 * (int64_t)ref_kf[p];
  const double dist = norm3(__dsub_rn(X, R[0]), __dsub_rn(Y, R[1]), __dsub_rn(Z, R[2]));
  int level = ref_level[p];
  if (level < 0) level = 1;
  const double sf = scale[level];
  dmin[p] = __ddiv_rn(__dmul_rn(__ddiv_rn(1.0, sf), dist), sf);
  dmax[p] = __dmul_rn(__dmul_rn(sf, dist), scale[nlev - 1 - level]);
  const double in = __ddiv_rn(1.0, (double)cnt);
  normal[3 * p] = __dmul_rn(nx, in);
  normal[3 * p + 1] = __dmul_rn(ny, in);
  normal[3 * p + 2] = __dmul_rn(nz, in);
}

template <int NW>
void launch_distinctive(bool masked, dim3 g, hipStream_t st, const uint8_t* desc,
                        const uint8_t* masks, const int32_t* ptr, const int32_t* row, int n,
                        int32_t* best, uint8_t* od, uint8_t* om) {
  if (masked)
    hipLaunchKernelGGL((k_distinctive<NW, true>), g, dim3(256), 0, st, desc, masks, ptr, row, n,
                       best, od, om);
  else
    hipLaunchKernelGGL((k_distinctive<NW, false>), g, dim3(256), 0, st, desc, masks, ptr, row, n,
                       best, od, om);
}

}  // namespace
}  // namespace mcs

extern "C" {

int mcs_distinctive_descriptors_device(const uint8_t* d_desc, const uint8_t* d_masks, int32_t bytes,
                                       const int32_t* d_obs_ptr, const int32_t* d_obs_row,
                                       int32_t n_points, int32_t* d_best, uint8_t* d_out_desc,
                                       uint8_t* d_out_mask, void* stream) {
  if (n_points < 0) {
    mcs::set_error("distinctive descriptors: n_points must be >= 0");
    return MCS_ERR_ARG;
  }
  if (bytes != 16 && bytes != 32 && bytes != 64) {
    mcs::set_error("distinctive descriptors: bytes must be 16, 32 or 64");
    return MCS_ERR_ARG;
  }
  if (n_points == 0) return MCS_OK;
  if (!d_desc || !d_obs_ptr || !d_obs_row || !d_best) {
    mcs::set_error("distinctive descriptors: null device pointer");
    return MCS_ERR_ARG;
  }
  const dim3 g((unsigned)((n_points + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
  const bool m = d_masks != nullptr;
  if (bytes == 16) mcs::launch_distinctive<4>(m, g, st, d_desc, d_masks, d_obs_ptr, d_obs_row, n_points, d_best, d_out_desc, d_out_mask);
  else if (bytes == 32) mcs::launch_distinctive<8>(m, g, st, d_desc, d_masks, d_obs_ptr, d_obs_row, n_points, d_best, d_out_desc, d_out_mask);
  else mcs::launch_distinctive<16>(m, g, st, d_desc, d_masks, d_obs_ptr, d_obs_row, n_points, d_best, d_out_desc, d_out_mask);
  MCS_HIP_CHECK(hipGetLastError());
  return MCS_OK;
}

int mcs_update_normal_depth_device(const double* d_points, int32_t n_points,
                                   const int32_t* d_obs_ptr, const int32_t* d_obs_kf,
                                   const double* d_kf_center, const int32_t* d_ref_kf,
                                   const int32_t* d_ref_level, const double* d_scale,
                                   int32_t n_levels, double* d_normal, double* d_min_dist,
                                   double* d_max_dist, void* stream) {
  if (n_points < 0) {
    mcs::set_error("update normal/depth: n_points must be >= 0");
    return MCS_ERR_ARG;
  }
  if (n_levels < 2) {
    mcs::set_error("update normal/depth: n_levels must be >= 2");
    return MCS_ERR_ARG;
  }
  if (n_points == 0) return MCS_OK;
  if (!d_points || !d_obs_ptr || !d_obs_kf || !d_kf_center || !d_ref_kf || !d_ref_level ||
      !d_scale || !d_normal || !d_min_dist || !d_max_dist) {
    mcs::set_error("update normal/depth: null device pointer");
    return MCS_ERR_ARG;
  }
  hipLaunchKernelGGL(mcs::k_normal_depth, dim3((unsigned)((n_points + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, d_points, n_points, d_obs_ptr, d_obs_kf, d_kf_center,
                     d_ref_kf, d_ref_level, d_scale, n_levels, d_normal, d_min_dist, d_max_dist);
  MCS_HIP_CHECK(hipGetLastError());
  return MCS_OK;
}

}  // extern "C"
