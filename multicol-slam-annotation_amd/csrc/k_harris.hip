// HarrisResponses (src/mdBRIEFextractorOct.cpp:86-132), opt-in: the reference defines it and
// stores scoreType (HARRIS_SCORE = 0) but ComputeKeyPointsOctTree never calls it (responses
// stay FAST scores).  Exposed as its own device entry point for callers that want Harris
// responses for keypoints in level coordinates.
//
// One lane per keypoint: blockSize^2 3x3 Sobel taps accumulated in int32 (a = sum Ix^2,
// b = sum Iy^2, c = sum Ix*Iy; |Ix|, |Iy| <= 1020 so 49 * 1020^2 < 2^31), then the reference's
// float expression in its evaluation order with round-to-nearest intrinsics (no contraction).
// The reference reads the 25 px BORDER_REFLECT_101-padded level (:1185-1197); pixels outside
// the level are read from their reflect-101 mirror here.
#include "common.hpp"
#include "../../include/mcs_extractor.h"

namespace mcs {

__device__ __forceinline__ int harris_refl(int p, int n) {
  p = p < 0 ? -p : p;
  return p >= n ? 2 * n - 2 - p : p;
}

__global__ __launch_bounds__(256) void k_harris(const uint64_t* __restrict__ level_ptrs,
                                                const int32_t* __restrict__ geom, int n_levels,
                                                const mcs_keypoint* __restrict__ kps, int n,
                                                int bs, float k, float scale_sq_sq,
                                                float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const mcs_keypoint kp = kps[i];
  const int z = min(max(kp.octave, 0), n_levels - 1);
  const uint8_t* img = reinterpret_cast<const uint8_t*>(level_ptrs[z]);
  const int w = geom[3 * z], h = geom[3 * z + 1], pitch = geom[3 * z + 2];
  const int x0 = (int)rintf(kp.x), y0 = (int)rintf(kp.y);   // cvRound
  const int r = bs / 2;
  auto px = [&](int y, int x) -> int {
    return img[(int64_t)harris_refl(y, h) * pitch + harris_refl(x, w)];
  };
  int a = 0, b = 0, c = 0;
  for (int dy = 0; dy < bs; dy++) {
    const int y = y0 - r + dy;
    for (int dx = 0; dx < bs; dx++) {
      const int x = x0 - r + dx;
      const int ix = (px(y, x + 1) - px(y, x - 1)) * 2 + (px(y - 1, x + 1) - px(y - 1, x - 1)) +
                     (px(y + 1, x + 1) - px(y + 1, x - 1));
      const int iy = (px(y + 1, x) - px(y - 1, x)) * 2 + (px(y + 1, x - 1) - px(y - 1, x - 1)) +
                     (px(y + 1, x + 1) - px(y - 1, x + 1));
      a += ix * ix;
      b += iy * iy;
      c += ix * iy;
    }
  }
  // ((float)a * b - (float)c * c - harris_k * ((float)a + b) * ((float)a + b)) * scale_sq_sq
  const float fa = (float)a, fb = (float)b, fc = (float)c;
  const float apb = __fadd_rn(fa, fb);
  const float t = __fsub_rn(__fsub_rn(__fmul_rn(fa, fb), __fmul_rn(fc, fc)),
                            __fmul_rn(__fmul_rn(k, apb), apb));
  out[i] = __fmul_rn(t, scale_sq_sq);
}

}  // namespace mcs

using namespace mcs;

extern "C" int mcs_harris_responses_device(const uint64_t* d_level_ptrs, const int32_t* d_level_geom,
                                           int32_t n_levels, const mcs_keypoint* d_kps, int32_t n,
                                           int32_t block_size, float harris_k, float* d_response,
                                           void* stream) {
  // CV_Assert(blockSize * blockSize <= 2048) (:92); the int32 sums need blockSize <= 45
  if (n < 0 || n_levels < 1 || block_size < 1 || block_size > 45 ||
      (n > 0 && (!d_level_ptrs || !d_level_geom || !d_kps || !d_response))) {
    set_error("mcs_harris_responses_device: bad argument");
    return MCS_ERR_ARG;
  }
  if (n == 0) return MCS_OK;
  // float scale = 1.f / ((1 << 2) * blockSize * 255.f); scale_sq_sq = scale^4 (left to right)
  const float scale = 1.f / ((float)((1 << 2) * block_size) * 255.f);
  const float s4 = ((scale * scale) * scale) * scale;
  hipLaunchKernelGGL(k_harris, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     d_level_ptrs, d_level_geom, n_levels, d_kps, n, block_size, harris_k, s4,
                     d_response);
  MCS_HIP_CHECK(hipGetLastError());
  return MCS_OK;
}
