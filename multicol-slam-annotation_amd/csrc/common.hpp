// Shared host/device helpers for libmcs_amd (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cmath>
#include "../../include/mcs_common.h"

namespace mcs {

void set_error(const char* msg);
void set_hip_error(hipError_t e, const char* expr, const char* file, int line);

// host cvRound/cvFloor with OpenCV semantics (round half to even via lrint)
inline int cv_round(double v) { return (int)std::lrint(v); }
inline int cv_roundf(float v) { return (int)std::lrintf(v); }
inline int cv_floor(double v) { int i = (int)v; return i - (i > v); }
inline int cv_floorf(float v) { int i = (int)v; return i - (i > v); }

}  // namespace mcs

#define MCS_HIP_CHECK(expr)                                          \
  do {                                                               \
    hipError_t e_ = (expr);                                          \
    if (e_ != hipSuccess) {                                          \
      mcs::set_hip_error(e_, #expr, __FILE__, __LINE__);             \
      return MCS_ERR_HIP;                                            \
    }                                                                \
  } while (0)

// ---- device helpers -------------------------------------------------------
namespace mcs {
namespace dev {

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Round a byte pointer down to its dword.  Pointer arithmetic (not an integer round trip)
// keeps the global address space, so loads stay global_load (a flat_load also counts on
// lgkmcnt and every LDS wait would then wait for it).
// a wave-uniform pointer moved to SGPRs: stores / loads through it + a 32-bit lane offset use
// the saddr form (no 64-bit address arithmetic per lane)
// (rebuilt as a global-address-space pointer: from a plain integer the compiler would treat it
// as generic and emit flat instructions, which also count against lgkmcnt)
template <typename T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  typedef __attribute__((address_space(1))) T GT;
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  GT* g = (GT*)(((uint64_t)hi << 32) | lo);
  return (T*)g;
}
__device__ __forceinline__ const uint32_t* align_down4(const uint8_t* p) {
  return reinterpret_cast<const uint32_t*>(p - ((uintptr_t)p & 3));
}

// LDS ordering between lanes of ONE wave (no cross-wave barrier)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int wave_incl_scan(int v) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int t = __shfl_up(v, o, 64);
    if (lane_id() >= o) v += t;
  }
  return v;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ uint64_t lanemask_lt() {
  const int l = lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// Exclusive scan across a block of NT threads (NT multiple of 64, <= 1024).
// s_tmp needs NT/64 + 1 ints.  Returns exclusive prefix, *total = block sum.
template <int NT>
__device__ __forceinline__ int block_excl_scan(int v, int* s_tmp, int* total) {
  const int w = threadIdx.x >> 6, l = lane_id();
  int inc = wave_incl_scan(v);
  if (l == 63) s_tmp[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int i = 0; i < NT / 64; i++) { int t = s_tmp[i]; s_tmp[i] = acc; acc += t; }
    s_tmp[NT / 64] = acc;
  }
  __syncthreads();
  int r = s_tmp[w] + inc - v;
  *total = s_tmp[NT / 64];
  __syncthreads();
  return r;
}

}  // namespace dev
}  // namespace mcs
