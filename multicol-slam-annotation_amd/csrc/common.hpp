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

// inclusive prefix sum over the 64 lanes on DPP (integer adds: any order is exact): within each
// row of 16 the sums of the 1, 2, 3 lanes below, then 4 back (banks 1-3) and 8 back (banks 2-3);
// then row 15's total into rows 1 and 3 (row_bcast:15) and lane 31's into rows 2 and 3
// (row_bcast:31).  Seven DPP adds instead of six ds_bpermute round trips with their address
// arithmetic.  Disabled rows / banks and out-of-row sources contribute the 0 of update_dpp.
__device__ __forceinline__ int wave_incl_scan(int v) {
  int x = v + __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);   // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);          // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, v, 0x113, 0xF, 0xF, true);          // row_shr:3
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xE, true);          // row_shr:4, banks 1-3
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xC, true);          // row_shr:8, banks 2-3
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);         // row_bcast:15, rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);         // row_bcast:31, rows 2, 3
  return x;
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

// The same with one barrier: the wave totals alternate between two halves of s_tmp2 (2 NT/64
// ints; `parity` is a per-thread counter every thread of the block advances alike), so a scan's
// writes never meet the previous scan's reads (those precede the previous scan's barrier in
// program order) and the two trailing barriers of block_excl_scan go.  Callers that relied on
// a scan as a block-wide barrier for their own data must not use this form.
template <int NT>
__device__ __forceinline__ int block_excl_scan1(int v, int* s_tmp2, int& parity, int* total) {
  constexpr int NW = NT / 64;
  const int w = threadIdx.x >> 6, l = lane_id();
  const int inc = wave_incl_scan(v);
  int* const t = s_tmp2 + parity * NW;
  parity ^= 1;
  if (l == 63) t[w] = inc;
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NW; i++) {
    const int x = t[i];
    pre += (i < w) ? x : 0;
    tot += x;
  }
  *total = tot;
  return pre + inc - v;
}

}  // namespace dev
}  // namespace mcs
