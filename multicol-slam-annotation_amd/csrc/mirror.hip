// Mirror-mask pyramid of the omni camera model (include/mcs_cammodel.h).
// Reference: CreateMirrorMask src/cam_model_omni.cpp:183-222, isPointInMirrorMask :165-180.
//
// One launch writes every level: grid.y = level, each lane produces 4 consecutive bytes of a
// row (one dword store; HBM-bound, 1 B written per pixel, nothing read). The per-pixel test
// keeps the reference's float/double mix: (float)pow(i - u0, 2) squares the float difference
// in double (exact) and rounds to float, the sum and sqrt are float (correctly rounded).
#include "common.hpp"
#include "../../include/mcs_cammodel.h"

namespace mcs {
namespace {

constexpr int kMaxMirrorLevels = 4;
constexpr float kMirrorOffset[kMaxMirrorLevels] = {22.0f, 10.0f, 5.0f, 1.0f};  // :195

struct MirrorLevels {
  int w[kMaxMirrorLevels], h[kMaxMirrorLevels];
  long long off[kMaxMirrorLevels];
  float rc[kMaxMirrorLevels], cc[kMaxMirrorLevels], thr[kMaxMirrorLevels];
};

__global__ __launch_bounds__(256) void k_mirror_mask(MirrorLevels L, uint8_t* __restrict__ out) {
  const int l = blockIdx.y;
  const int w = L.w[l], h = L.h[l];
  const int quads = (w + 3) >> 2;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)quads * h) return;
  const int i = (int)(t / quads), j0 = (int)(t % quads) * 4;
  const float rc = L.rc[l], cc = L.cc[l], thr = L.thr[l];
  const double di = (double)((float)i - rc);
  const float a = (float)(di * di);
  uint8_t v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double dj = (double)((float)(j0 + k) - cc);
    const float ans = __fsqrt_rn(a + (float)(dj * dj));
    v[k] = ans < thr ? 255 : 0;
  }
  uint8_t* row = out + L.off[l] + (long long)i * w;
  if (j0 + 4 <= w && (((uintptr_t)(row + j0)) & 3) == 0) {
    *reinterpret_cast<uint32_t*>(row + j0) =
        (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16) | ((uint32_t)v[3] << 24);
  } else {
    for (int k = 0; k < 4 && j0 + k < w; ++k) row[j0 + k] = v[k];
  }
}

int layout(int32_t width, int32_t height, int32_t levels, MirrorLevels* L, long long* total) {
  if (width <= 0 || height <= 0 || levels < 1 || levels > kMaxMirrorLevels) {
    set_error("mirror mask: need width, height > 0 and 1 <= levels <= 4");
    return MCS_ERR_ARG;
  }
  long long off = 0;
  int w = width, h = height;
  for (int l = 0; l < levels; ++l) {
    if (l) { w = (w + 1) / 2; h = (h + 1) / 2; }  // cv::buildPyramid / pyrDown sizes
    L->w[l] = w; L->h[l] = h; L->off[l] = off;
    off += (long long)w * h;
  }
  *total = off;
  return MCS_OK;
}

}  // namespace
}  // namespace mcs

using namespace mcs;

extern "C" {

int mcs_mirror_mask_layout(int32_t width, int32_t height, int32_t levels, int32_t* widths,
                           int32_t* heights, int64_t* offsets, int64_t* total_bytes) {
  MirrorLevels L{};
  long long total = 0;
  int rc = layout(width, height, levels, &L, &total);
  if (rc) return rc;
  for (int l = 0; l < levels; ++l) {
    if (widths) widths[l] = L.w[l];
    if (heights) heights[l] = L.h[l];
    if (offsets) offsets[l] = L.off[l];
  }
  if (total_bytes) *total_bytes = total;
  return MCS_OK;
}

int mcs_create_mirror_mask_device(double cam_u0, double cam_v0, int32_t width, int32_t height,
                                  int32_t levels, uint8_t* d_masks, void* stream) {
  MirrorLevels L{};
  long long total = 0;
  int rc = layout(width, height, levels, &L, &total);
  if (rc) return rc;
  if (!d_masks) { set_error("mirror mask: null output"); return MCS_ERR_ARG; }
  // src/cam_model_omni.cpp:189-190 (u0 <- v0, v0 <- u0) and :204-205 (ceil of the half)
  float r = (float)cam_v0, c = (float)cam_u0;
  int max_items = 0;
  for (int l = 0; l < levels; ++l) {
    if (l) { r = std::ceil(r / 2.0f); c = std::ceil(c / 2.0f); }
    L.rc[l] = r; L.cc[l] = c; L.thr[l] = r + kMirrorOffset[l];
    const int items = ((L.w[l] + 3) / 4) * L.h[l];
    if (items > max_items) max_items = items;
  }
  hipLaunchKernelGGL(k_mirror_mask, dim3((max_items + 255) / 256, levels), dim3(256), 0,
                     (hipStream_t)stream, L, d_masks);
  MCS_HIP_CHECK(hipGetLastError());
  return MCS_OK;
}

int mcs_is_point_in_mirror_mask(const uint8_t* mask, int32_t cols, int32_t rows, double u,
                                double v) {
  if (!mask) return 0;
  const int ur = cv_round(u), vr = cv_round(v);  // :170-171
  if (ur >= cols || ur <= 0 || vr >= rows || vr <= 0) return 0;  // :173-175
  return mask[(long long)vr * cols + ur] > 0 ? 1 : 0;  // :177
}

}  // extern "C"
