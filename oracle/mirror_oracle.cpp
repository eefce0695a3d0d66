// TEST INFRASTRUCTURE ONLY (checker, never the product path): CPU restatement of the omni
// camera's mirror masks for the parity tests of csrc/mirror.hip.
//   oracle_create_mirror_mask   ~ CreateMirrorMask   reference src/cam_model_omni.cpp:183-222
//   oracle_is_point_in_mirror_mask ~ isPointInMirrorMask  src/cam_model_omni.cpp:165-180
// Written as the reference's literal pixel loop (std::pow in double, float sum, std::sqrt of a
// float); cv::buildPyramid level sizes are ((w+1)/2, (h+1)/2). Pinned by the reference's own
// Lafida calibration (tests/golden/lafida_settings.json: u0/v0/Iw/Ih) and by the geometric
// property checks in tests/test_mirror.py; OpenCV itself is absent, so the level-size rule
// is restated from pyrDown's documented dst size.
#include <cmath>
#include <cstdint>

extern "C" int oracle_create_mirror_mask(double cam_u0, double cam_v0, int width, int height,
                                         int levels, uint8_t* out) {
  if (width <= 0 || height <= 0 || levels < 1 || levels > 4 || !out) return -1;
  int w = width, h = height;
  float u0 = (float)cam_v0;  // :189 (swapped as in the reference)
  float v0 = (float)cam_u0;  // :190
  const float offset[4] = {22.0f, 10.0f, 5.0f, 1.0f};
  long long off = 0;
  for (int mIdx = 0; mIdx < levels; mIdx++) {
    if (mIdx != 0) {
      w = (w + 1) / 2;
      h = (h + 1) / 2;
      u0 = std::ceil(u0 / 2.0f);
      v0 = std::ceil(v0 / 2.0f);
    }
    for (int i = 0; i < h; ++i)
      for (int j = 0; j < w; ++j) {
        float ans = std::sqrt((float)std::pow(i - u0, 2) + (float)std::pow(j - v0, 2));
        out[off + (long long)i * w + j] = ans < (u0 + offset[mIdx]) ? 255 : 0;
      }
    off += (long long)w * h;
  }
  return 0;
}

extern "C" int oracle_is_point_in_mirror_mask(const uint8_t* mask, int cols, int rows, double u,
                                              double v) {
  const int ur = (int)std::lrint(u), vr = (int)std::lrint(v);
  if (ur >= cols || ur <= 0 || vr >= rows || vr <= 0) return 0;
  return mask[(long long)vr * cols + ur] > 0 ? 1 : 0;
}
