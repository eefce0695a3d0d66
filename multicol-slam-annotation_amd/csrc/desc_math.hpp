// Single-precision sin / cos of the keypoint angle for k_orient_desc's rotated-BRIEF fast path
// (compiled for the device and, by tests/cpp/sincos_f32_bound.cpp, for the host: the same IEEE
// operations, every multiply-add an explicit fma, so both evaluate bit for bit alike).
//
// The reference rotates the pattern with cos / sin of the double angle (rotatePattern,
// src/mdBRIEFextractorOct.cpp:285-301, angle = (double)(kp.angle * DEG2RADf), :313-316) and
// rounds x c - y s, x s + y c with cvRound.  The kernel rotates in float with these values and
// takes the double path (cos / sin in double, then the reference's double products) for every
// round in which some rotated value lies within kNearHalf of a half-integer: outside that
// band the float value and the double one round alike.  Bound: |x|, |y| <= 15 (the ORB
// pattern), |c_f - cos| and |s_f - sin| <= kSinCosErr, so |float value - exact| <= 30
// kSinCosErr + 1.5e-6 (half an ulp of |y s| <= 15 and of the fma's |value| <= 21.3) < kNearHalf.
// tests/test_desc_sincos.py checks kSinCosErr over EVERY float angle in [0, 2 pi + 1e-3].
#pragma once
#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define MCS_HD __host__ __device__
#else
#define MCS_HD
#endif
#include <cmath>

namespace mcs {

constexpr float kSinCosErr = 2.0e-7f;                     // max |error| of sincos_f32 (measured 7.2e-8)
constexpr float kNearHalf = 30.0f * kSinCosErr + 2.5e-6f;  // 8.5e-6

// sin / cos of t in [0, 2 pi + 1e-3] (the range of DEG2RADf * fastAtan2's [0, 360]):
// quadrant k = rint(t 2 / pi), r = t - k pi/2 (two-part Cody-Waite constant, |r| <= pi / 4 +
// 1e-6), Taylor polynomials of degree 9 (sin) and 10 (cos) on r, then the quadrant's swap / sign.
MCS_HD inline void sincos_f32(float t, float& s, float& c) {
  const float k = std::rint(t * 0.636619772f);
  float r = std::fma(-k, 1.57079637050628662109375f, t);   // pi/2 rounded to float
  r = std::fma(k, 4.37113900018624283e-8f, r);             // pi/2 - float(pi/2) = -4.37e-8
  const float r2 = r * r;
  float ps = std::fma(r2, 2.75573192e-6f, -1.98412698e-4f);
  ps = std::fma(ps, r2, 8.33333333e-3f);
  ps = std::fma(ps, r2, -1.66666667e-1f);
  const float sn = std::fma(ps * r2, r, r);                // r + r^3 ps(r^2)
  float pc = std::fma(r2, -2.75573192e-7f, 2.48015873e-5f);
  pc = std::fma(pc, r2, -1.38888889e-3f);
  pc = std::fma(pc, r2, 4.16666667e-2f);
  pc = std::fma(pc, r2, -0.5f);
  const float cs = std::fma(pc, r2, 1.0f);                 // 1 + r^2 pc(r^2)
  const int q = (int)k & 3;                                // sin / cos of r + q pi / 2
  float sv = (q & 1) ? cs : sn, cv = (q & 1) ? sn : cs;
  if (q & 2) sv = -sv;
  if ((q + 1) & 2) cv = -cv;
  s = sv;
  c = cv;
}

}  // namespace mcs
