// Pixel arithmetic of the pyramid kernels (k_pyramid.hip): the
// BORDER_REFLECT_101 index, the INTER_LINEAR vertical pass in both OpenCV 3.1 forms and the
// rounding of the normalised 5x5 box filter.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace mcs {

__device__ __forceinline__ int refl101(int p, int n) {
  p = p < 0 ? -p : p;
  return p >= n ? 2 * n - 2 - p : p;
}

// Vertical pass of cv::resize INTER_LINEAR.  Operand ranges: s = p0*a0 + p1*a1
// with p <= 255 and a0 + a1 = 2048 (each in [0, 2048]) so 0 <= s <= 522240 < 2^23, and
// b0, b1 in [0, 2048]: every product fits v_mul_i32_i24 exactly (< 2^31).
//   SSE2 form (VResizeLinearVec_32s8u): x0 = s0 >> 4 <= 32640, (x0*b0 >> 16) + (y0*b1 >> 16)
//   <= 1020, so the int16 saturations of the reference are no-ops and only the final u8
//   clamp remains; the caller passes x0 = s0 >> 4, y0 = s1 >> 4 (computed once per row).
//   scalar tail (FixedPtCast<int,uchar,22>): (s0*b0 + s1*b1 + 2^21) >> 22.
// The bit-field extracts below are exact for these ranges; they only tell the compiler the
// operand widths so that it emits v_mul_u32_u24 instead of the quarter-rate v_mul_lo_u32.
__device__ __forceinline__ uint32_t sse_x(int s) { return __builtin_amdgcn_ubfe((uint32_t)s, 4, 15); }
__device__ __forceinline__ int vres_sse(uint32_t x0, uint32_t y0, int b0, int b1) {
  const uint32_t t = ((x0 * ((uint32_t)b0 & 0xFFFu)) >> 16) + ((y0 * ((uint32_t)b1 & 0xFFFu)) >> 16);
  return (int)min(255u, (t + 2u) >> 2);
}
// The SSE2 form with both products as one v_mul_hi_u32_u24 each: with X = x0 << 8 (< 2^24 for
// x0 <= 32640) and B = b << 8 (<= 2^19), X * B >> 32 = x0 * b >> 16 exactly; the sum of the two
// terms is <= 1020, so (t + 2) >> 2 <= 255 and the u8 clamp is a no-op.
// (written as the instruction: left to the 64-bit pattern, a loop-carried operand whose range
// the compiler cannot see becomes v_mul_lo_u32 + v_mul_hi_u32 + v_mad_u64_u32, quarter rate)
__device__ __forceinline__ uint32_t mulhi_u24(uint32_t a_vgpr, uint32_t b_sgpr) {
  uint32_t d;
  asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(d) : "s"(b_sgpr), "v"(a_vgpr));
  return d;
}
__device__ __forceinline__ uint32_t sse_vres8(uint32_t X0, uint32_t Y0, uint32_t B0, uint32_t B1) {
  return (mulhi_u24(X0, B0) + mulhi_u24(Y0, B1) + 2u) >> 2;
}
__device__ __forceinline__ int vres_fixed(int s0, int s1, int b0, int b1) {
  const uint32_t u0 = __builtin_amdgcn_ubfe((uint32_t)s0, 0, 20), u1 = __builtin_amdgcn_ubfe((uint32_t)s1, 0, 20);
  return (int)min(255u, (u0 * ((uint32_t)b0 & 0xFFFu) + u1 * ((uint32_t)b1 & 0xFFFu) + (1u << 21)) >> 22);
}
__device__ __forceinline__ int vres(int s0, int s1, int b0, int b1, bool simd) {
  return simd ? vres_sse(sse_x(s0), sse_x(s1), b0, b1) : vres_fixed(s0, s1, b0, b1);
}

// (2s + 25) / 50 for 2s + 25 <= 12775 (s = 5x5 sum of u8) by multiply-shift;
// exact: 20972 / 2^20 - 1/50 < 4.6e-7 and 12775 * 4.6e-7 < 1/50 (checked on the host too)
__device__ __forceinline__ uint32_t div50(uint32_t n) { return (n * 20972u) >> 20; }

}  // namespace mcs
