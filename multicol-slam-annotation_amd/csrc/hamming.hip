// Hamming matching on gfx950: XOR + v_bcnt_u32_b32 popcount-accumulate, trains staged in
// LDS and broadcast to a wave of 64 queries (one query per lane, descriptor in VGPRs).
//
// Reference: DescriptorDistance64 / ...Masked   src/cORBmatcher.cpp:2443-2477
//            SearchForTriangulationRaw          src/cORBmatcher.cpp:968-1156
//            best/second-best scans             src/cORBmatcher.cpp:67-163, 326-475
#include "common.hpp"
#include <map>
#include <mutex>
#include "../../include/mcs_matcher.h"
#include "ldlt.hpp"
#include <cstring>
#include <rocprim/rocprim.hpp>
#include <algorithm>
#include <new>
#include <vector>

namespace mcs {

constexpr int kHamThreads = 256;
constexpr int kHamTile = 256;      // train rows per LDS tile

template <int W>
__device__ __forceinline__ int ham_dist_v(const uint32_t (&q)[W], const uint4* t4) {
  int d = 0;
#pragma unroll
  for (int w4 = 0; w4 < W / 4; w4++) {
    const uint4 v = t4[w4];
    d += __popc(q[4 * w4 + 0] ^ v.x);
    d += __popc(q[4 * w4 + 1] ^ v.y);
    d += __popc(q[4 * w4 + 2] ^ v.z);
    d += __popc(q[4 * w4 + 3] ^ v.w);
  }
  return d;
}

// Top-2 over one (query set, train set) pair; blockIdx.x = query tile, blockIdx.y = pair.
// Each lane owns kQPT queries (descriptors in VGPRs) so one LDS broadcast read of a train
// row feeds kQPT distances.  The running best/second-best are kept as packed keys
// (dist << 16 | train index): trains are scanned in index order, so the strict-< rule of the
// reference scans (first minimum wins, :2447) equals "two smallest keys", maintained with
// v_min_u32 + v_med3_u32 (best <= second always).
constexpr int kQPT = 2;

__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// popcount-accumulate as one v_bcnt_u32_b32 (the compiler otherwise reassociates the sum
// into bcnt(x, 0) + v_add3 chains, 25 % more VALU)
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
  uint32_t r;
  asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
  return r;
}

template <int W>
__global__ __launch_bounds__(kHamThreads) void k_top2(
    const uint8_t* __restrict__ qbase, const uint8_t* __restrict__ tbase,
    const int32_t* __restrict__ counts, const int32_t* __restrict__ pairs, int64_t set_stride,
    int nq_fixed, int nt_fixed, int cap_out, int32_t* __restrict__ best_idx,
    int32_t* __restrict__ best_dist, int32_t* __restrict__ second_idx,
    int32_t* __restrict__ second_dist) {
  __shared__ uint4 tile[kHamTile * (W / 4)];
  const int p = blockIdx.y;
  const uint8_t* Q;
  const uint8_t* T;
  int nq, nt;
  if (pairs) {
    const int qs = pairs[2 * p], ts = pairs[2 * p + 1];
    Q = qbase + (int64_t)qs * set_stride;
    T = tbase + (int64_t)ts * set_stride;
    nq = counts[qs];
    nt = counts[ts];
  } else {
    Q = qbase; T = tbase; nq = nq_fixed; nt = nt_fixed;
  }
  const int q0 = blockIdx.x * (kHamThreads * kQPT);
  if (q0 >= nq) return;  // uniform per block
  uint32_t q[kQPT][W];
#pragma unroll
  for (int k = 0; k < kQPT; k++) {
    const int qi = q0 + k * kHamThreads + threadIdx.x;
    if (qi < nq) {
      const uint4* qp = reinterpret_cast<const uint4*>(Q + (int64_t)qi * W * 4);
#pragma unroll
      for (int w4 = 0; w4 < W / 4; w4++) {
        const uint4 v = qp[w4];
        q[k][4 * w4] = v.x; q[k][4 * w4 + 1] = v.y; q[k][4 * w4 + 2] = v.z; q[k][4 * w4 + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int w = 0; w < W; w++) q[k][w] = 0;
    }
  }
  uint32_t k1[kQPT], k2[kQPT];
#pragma unroll
  for (int k = 0; k < kQPT; k++) { k1[k] = 0xFFFFFFFFu; k2[k] = 0xFFFFFFFFu; }
  for (int t0 = 0; t0 < nt; t0 += kHamTile) {
    const int nt_tile = min(kHamTile, nt - t0);
    __syncthreads();
    const uint4* src = reinterpret_cast<const uint4*>(T + (int64_t)t0 * W * 4);
    for (int i = threadIdx.x; i < nt_tile * (W / 4); i += kHamThreads) tile[i] = src[i];
    __syncthreads();
    auto body = [&](int j) {
      const uint4* tr = &tile[j * (W / 4)];
      const uint32_t idx = (uint32_t)(t0 + j);
      uint32_t d[kQPT];
#pragma unroll
      for (int k = 0; k < kQPT; k++) d[k] = 0;
#pragma unroll
      for (int w4 = 0; w4 < W / 4; w4++) {
        const uint4 v = tr[w4];
#pragma unroll
        for (int k = 0; k < kQPT; k++) {
          d[k] = bcnt_acc(q[k][4 * w4 + 0] ^ v.x, d[k]);
          d[k] = bcnt_acc(q[k][4 * w4 + 1] ^ v.y, d[k]);
          d[k] = bcnt_acc(q[k][4 * w4 + 2] ^ v.z, d[k]);
          d[k] = bcnt_acc(q[k][4 * w4 + 3] ^ v.w, d[k]);
        }
      }
#pragma unroll
      for (int k = 0; k < kQPT; k++) {
        const uint32_t key = (d[k] << 16) | idx;
        k2[k] = med3_u32(k1[k], key, k2[k]);
        k1[k] = min(k1[k], key);
      }
    };
    int j = 0;
    for (; j + 4 <= nt_tile; j += 4) { body(j); body(j + 1); body(j + 2); body(j + 3); }
    for (; j < nt_tile; j++) body(j);
  }
  const int none = 8 * 4 * W + 1;
#pragma unroll
  for (int k = 0; k < kQPT; k++) {
    const int qi = q0 + k * kHamThreads + threadIdx.x;
    if (qi < nq) {
      const int64_t o = (int64_t)p * cap_out + qi;
      const bool h1 = k1[k] != 0xFFFFFFFFu, h2 = k2[k] != 0xFFFFFFFFu;
      best_idx[o] = h1 ? (int)(k1[k] & 0xFFFF) : -1;
      best_dist[o] = h1 ? (int)(k1[k] >> 16) : none;
      second_idx[o] = h2 ? (int)(k2[k] & 0xFFFF) : -1;
      second_dist[o] = h2 ? (int)(k2[k] >> 16) : none;
    }
  }
}

// ---------------------------------------------------------------------------
// 32-byte descriptors on the int8 matrix cores: with bits mapped to +-1 bytes,
// dot(a, b) = 256 - 2 * Hamming(a, b), exactly (i32 accumulation of +-1 products).
// v_mfma_i32_32x32x32_i8: A = 32 train rows, B = 32 query columns, K = 32 bits per
// instruction, 8 instructions per 256-bit descriptor.  A workgroup (4 waves) owns 256
// queries of one pair; each wave keeps the expanded bits of its 64 queries in registers
// (B operands of both 32-column groups) and streams 64-train tiles, expanded once per
// workgroup into LDS.  The accumulator puts one query column on each lane and 16 train rows
// in its registers, so the running best/second-best keys (dist << 16 | train) are updated
// lane-locally; the two lane halves (different train rows) are merged at the end.
// ---------------------------------------------------------------------------
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// 4 bits -> 4 bytes of +1 (bit set) / -1 (bit clear)
__device__ __forceinline__ uint32_t expand4(uint32_t nib) {
  const uint32_t m = (nib * 0x00204081u) & 0x01010101u;
  return ~(m * 0xFEu);
}
// 16 bits -> 16 bytes (element j <-> bit j)
__device__ __forceinline__ v4i expand16(uint32_t bits) {
  v4i r;
  r.x = (int)expand4(bits & 0xF);
  r.y = (int)expand4((bits >> 4) & 0xF);
  r.z = (int)expand4((bits >> 8) & 0xF);
  r.w = (int)expand4((bits >> 12) & 0xF);
  return r;
}

// KEYED form (every train index < 2^13): the matrix cores produce the top-2 key up to the
// train index.  Train bits map to -64 (set) / +64 (clear), query bits to +64 (set) / -64
// (clear), so the product sum is -4096 (256 - 2 Hamming) = 2^13 Hamming - 2^20, and
// key = sum + (2^20 + tile base) + the row's offset (one v_add3, the offset an inline constant)
// = 2^13 Hamming + train index, ordered as (Hamming, train index) by min / med3 (< 2^22).
__device__ __forceinline__ uint32_t expand4_64(uint32_t nib) {   // set -> 0xC0, clear -> 0x40
  const uint32_t m = (nib * 0x00204081u) & 0x01010101u;
  return (m << 7) | 0x40404040u;
}
__device__ __forceinline__ v4i expand16_64(uint32_t bits) {
  v4i r;
  r.x = (int)expand4_64(bits & 0xF);
  r.y = (int)expand4_64((bits >> 4) & 0xF);
  r.z = (int)expand4_64((bits >> 8) & 0xF);
  r.w = (int)expand4_64((bits >> 12) & 0xF);
  return r;
}
constexpr int kKeyBits = 13;

constexpr int kMfTileT = 64;            // trains per LDS tile
constexpr int kMfPitch = 256 + 16;      // expanded train row (bytes), padded against bank conflicts

#ifndef MCS_TOP2_MINB
#define MCS_TOP2_MINB 4   // 128 VGPRs, accumulators in VGPRs (no AGPR reads); measured 0.47 -> 0.44 ms
#endif
template <bool KEYED>
__global__ __launch_bounds__(256, MCS_TOP2_MINB) void k_top2_mfma32(
    const uint8_t* __restrict__ qbase, const uint8_t* __restrict__ tbase,
    const int32_t* __restrict__ counts, const int32_t* __restrict__ pairs, int64_t set_stride,
    int nq_fixed, int nt_fixed, int cap_out, int32_t* __restrict__ best_idx,
    int32_t* __restrict__ best_dist, int32_t* __restrict__ second_idx,
    int32_t* __restrict__ second_dist) {
  __shared__ __attribute__((aligned(16))) uint8_t s_t[kMfTileT * kMfPitch];
  const int p = blockIdx.y;
  const uint8_t* Q;
  const uint8_t* T;
  int nq, nt;
  if (pairs) {
    const int qs = pairs[2 * p], ts = pairs[2 * p + 1];
    Q = qbase + (int64_t)qs * set_stride;
    T = tbase + (int64_t)ts * set_stride;
    nq = counts[qs];
    nt = counts[ts];
  } else {
    Q = qbase; T = tbase; nq = nq_fixed; nt = nt_fixed;
  }
  const int q_blk = blockIdx.x * 256;
  if (q_blk >= nq) return;   // uniform per block
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int h = lane >> 5, col = lane & 31;
  // ---- B operands: this wave's 64 queries (2 column groups x 8 k-steps)
  v4i bq[2][8];
#pragma unroll
  for (int c = 0; c < 2; c++) {
    const int qi = q_blk + wv * 64 + c * 32 + col;
    const uint32_t* qd = reinterpret_cast<const uint32_t*>(Q + (int64_t)min(qi, max(nq - 1, 0)) * 32);
    uint32_t w[8];
#pragma unroll
    for (int s = 0; s < 8; s++) w[s] = qd[s];
#pragma unroll
    for (int s = 0; s < 8; s++)   // KEYED: query set -> +64, i.e. the train map of ~bits
      bq[c][s] = KEYED ? expand16_64(~(w[s] >> (16 * h)) & 0xFFFF) : expand16((w[s] >> (16 * h)) & 0xFFFF);
  }
  uint32_t k1[2] = {0xFFFFFFFFu, 0xFFFFFFFFu}, k2[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
  // train tile bits, one tile ahead: the next tile's loads are in flight while this one is
  // expanded and multiplied (each thread 2 dwords of 64 trains x 8 dwords)
  uint32_t nb[2];
  auto fetch = [&](int t0n) {
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const int e = tid + 256 * r;
      const int tr = e >> 3, dw = e & 7;
      nb[r] = t0n + tr < nt ? reinterpret_cast<const uint32_t*>(T + (int64_t)(t0n + tr) * 32)[dw] : 0u;
    }
  };
  fetch(0);
  for (int t0 = 0; t0 < nt; t0 += kMfTileT) {
    const int ntile = min(kMfTileT, nt - t0);
    const uint32_t cb[2] = {nb[0], nb[1]};
    if (t0 + kMfTileT < nt) fetch(t0 + kMfTileT);
    __syncthreads();
    // ---- expand the tile: 64 trains x 8 dwords; each thread 2 dwords -> 2 x 32 bytes
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const int e = tid + 256 * r;          // 0..511
      const int tr = e >> 3, dw = e & 7;
      const uint32_t bits = cb[r];
      uint8_t* dst = s_t + tr * kMfPitch + dw * 32;
      const v4i lo = KEYED ? expand16_64(bits & 0xFFFF) : expand16(bits & 0xFFFF);
      const v4i hi = KEYED ? expand16_64(bits >> 16) : expand16(bits >> 16);
      *reinterpret_cast<v4i*>(dst) = lo;
      *reinterpret_cast<v4i*>(dst + 16) = hi;
    }
    __syncthreads();
    // ---- two 32-train sub-tiles
#pragma unroll
    for (int st = 0; st < 2; st++) {
      if (st * 32 >= ntile) break;
      const int tb = t0 + st * 32 + 4 * h;
      // KEYED: both accumulators start from the rows' key offsets (2^20 + tile base + the row's
      // offset), one set shared by the two query groups, so the MFMA result is the key itself
      v16i cinit = {0};
      if (KEYED) {
        const uint32_t tbk = (uint32_t)tb + (1u << 20);
#pragma unroll
        for (int r = 0; r < 16; r++) cinit[r] = (int)(tbk + (uint32_t)((r & 3) + 8 * (r >> 2)));
      }
      v16i acc0 = cinit, acc1 = cinit;
      const uint8_t* arow = s_t + (st * 32 + col) * kMfPitch + 16 * h;
#pragma unroll
      for (int s = 0; s < 8; s++) {
        const v4i a = *reinterpret_cast<const v4i*>(arow + 32 * s);
        acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bq[0][s], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bq[1][s], acc1, 0, 0, 0);
      }
      const bool full = st * 32 + 32 <= ntile;
      if (KEYED) {
        uint32_t key0[16], key1[16];
#pragma unroll
        for (int r = 0; r < 16; r++) {
          key0[r] = (uint32_t)acc0[r];
          key1[r] = (uint32_t)acc1[r];
        }
        if (!full) {   // the last, partial tile (a scalar branch: no selects in full tiles)
          asm volatile("" ::: "memory");
#pragma unroll
          for (int r = 0; r < 16; r++)
            if (tb + (r & 3) + 8 * (r >> 2) >= nt) { key0[r] = 0xFFFFFFFFu; key1[r] = 0xFFFFFFFFu; }
        }
#pragma unroll
        for (int r = 0; r < 16; r++) {
          k2[0] = med3_u32(k1[0], key0[r], k2[0]);
          k1[0] = min(k1[0], key0[r]);
          k2[1] = med3_u32(k1[1], key1[r], k2[1]);
          k1[1] = min(k1[1], key1[r]);
        }
        continue;
      }
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int trow = tb + (r & 3) + 8 * (r >> 2);
        const uint32_t d0 = (uint32_t)(256 - acc0[r]) >> 1, d1 = (uint32_t)(256 - acc1[r]) >> 1;
        uint32_t key0 = (d0 << 16) | (uint32_t)trow, key1 = (d1 << 16) | (uint32_t)trow;
        if (!full && trow >= nt) { key0 = 0xFFFFFFFFu; key1 = 0xFFFFFFFFu; }
        k2[0] = med3_u32(k1[0], key0, k2[0]);
        k1[0] = min(k1[0], key0);
        k2[1] = med3_u32(k1[1], key1, k2[1]);
        k1[1] = min(k1[1], key1);
      }
    }
  }
  // ---- merge the two lane halves (same query, disjoint train rows) and write
  const int none = 8 * 32 + 1;
#pragma unroll
  for (int c = 0; c < 2; c++) {
    const uint32_t o1 = __shfl_xor(k1[c], 32), o2 = __shfl_xor(k2[c], 32);
    const uint32_t b1 = min(k1[c], o1), b2 = min(max(k1[c], o1), min(k2[c], o2));
    const int qi = q_blk + wv * 64 + c * 32 + col;
    if (h == 0 && qi < nq) {
      const int64_t o = (int64_t)p * cap_out + qi;
      const bool h1 = b1 != 0xFFFFFFFFu, h2 = b2 != 0xFFFFFFFFu;
      constexpr int kIb = KEYED ? kKeyBits : 16;
      constexpr uint32_t kIm = (1u << kIb) - 1u;
      best_idx[o] = h1 ? (int)(b1 & kIm) : -1;
      best_dist[o] = h1 ? (int)(b1 >> kIb) : none;
      second_idx[o] = h2 ? (int)(b2 & kIm) : -1;
      second_dist[o] = h2 ? (int)(b2 >> kIb) : none;
    }
  }
}

template <int W>
__global__ __launch_bounds__(kHamThreads) void k_dense(const uint8_t* __restrict__ A, int na,
                                                       const uint8_t* __restrict__ B, int nb,
                                                       uint16_t* __restrict__ D) {
  __shared__ uint4 tile[kHamTile * (W / 4)];
  const int qi = blockIdx.x * kHamThreads + threadIdx.x;
  const int t0 = blockIdx.y * kHamTile;
  const int nt_tile = min(kHamTile, nb - t0);
  const uint4* src = reinterpret_cast<const uint4*>(B + (int64_t)t0 * W * 4);
  for (int i = threadIdx.x; i < nt_tile * (W / 4); i += kHamThreads) tile[i] = src[i];
  __syncthreads();
  if (qi >= na) return;
  uint32_t q[W];
  const uint4* qp = reinterpret_cast<const uint4*>(A + (int64_t)qi * W * 4);
#pragma unroll
  for (int w4 = 0; w4 < W / 4; w4++) {
    const uint4 v = qp[w4];
    q[4 * w4] = v.x; q[4 * w4 + 1] = v.y; q[4 * w4 + 2] = v.z; q[4 * w4 + 3] = v.w;
  }
  for (int j = 0; j < nt_tile; j++) D[(int64_t)qi * nb + t0 + j] = (uint16_t)ham_dist_v<W>(q, &tile[j * (W / 4)]);
}

// DescriptorDistance64Masked (src/cORBmatcher.cpp:2457-2477): (sum popc(x & m1) +
// sum popc(x & m2)) / 2 over the whole descriptor, integer division of the total.
template <int W>
__device__ __forceinline__ int ham_dist_masked_v(const uint32_t (&q)[W], const uint32_t (&qm)[W],
                                                 const uint4* t4, const uint4* m4) {
  int d = 0;
#pragma unroll
  for (int w4 = 0; w4 < W / 4; w4++) {
    const uint4 v = t4[w4], m = m4[w4];
    const uint32_t x0 = q[4 * w4 + 0] ^ v.x, x1 = q[4 * w4 + 1] ^ v.y;
    const uint32_t x2 = q[4 * w4 + 2] ^ v.z, x3 = q[4 * w4 + 3] ^ v.w;
    d += __popc(x0 & qm[4 * w4 + 0]) + __popc(x0 & m.x);
    d += __popc(x1 & qm[4 * w4 + 1]) + __popc(x1 & m.y);
    d += __popc(x2 & qm[4 * w4 + 2]) + __popc(x2 & m.z);
    d += __popc(x3 & qm[4 * w4 + 3]) + __popc(x3 & m.w);
  }
  return d >> 1;
}

template <int W>
__device__ __forceinline__ void load_desc_row(uint32_t (&q)[W], const uint8_t* row) {
  const uint4* qp = reinterpret_cast<const uint4*>(row);
#pragma unroll
  for (int w4 = 0; w4 < W / 4; w4++) {
    const uint4 v = qp[w4];
    q[4 * w4] = v.x; q[4 * w4 + 1] = v.y; q[4 * w4 + 2] = v.z; q[4 * w4 + 3] = v.w;
  }
}

static int check_bytes(int bytes) {
  if (bytes != 16 && bytes != 32 && bytes != 64) {
    set_error("descriptor bytes must be 16, 32 or 64");
    return MCS_ERR_ARG;
  }
  return MCS_OK;
}

#define MCS_DISPATCH_W(bytes, KERNEL, ...)                                                  \
  do {                                                                                     \
    if ((bytes) == 16) hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__);                         \
    else if ((bytes) == 32) hipLaunchKernelGGL(KERNEL<8>, __VA_ARGS__);                    \
    else hipLaunchKernelGGL(KERNEL<16>, __VA_ARGS__);                                      \
  } while (0)

}  // namespace mcs

using namespace mcs;

extern "C" {

int mcs_descriptor_distance64(const uint64_t* d1, const uint64_t* d2, int32_t dim) {
  uint64_t dist = 0;
  for (int d = 0; d < dim / 8; ++d) dist += (uint64_t)__builtin_popcountll(d1[d] ^ d2[d]);
  return (int)dist;
}

int mcs_descriptor_distance64_masked(const uint64_t* d1, const uint64_t* d2, const uint64_t* m1,
                                     const uint64_t* m2, int32_t dim) {
  uint64_t dist = 0;
  for (int i = 0; i < dim / 8; ++i) {
    const uint64_t x = d1[i] ^ d2[i];
    dist += (uint64_t)__builtin_popcountll(x & m1[i]) + (uint64_t)__builtin_popcountll(x & m2[i]);
  }
  return (int)(dist / 2);
}

int mcs_hamming_dense_device(const uint8_t* d_a, int32_t na, const uint8_t* d_b, int32_t nb,
                             int32_t bytes, uint16_t* d_dist, void* stream) {
  int rc = check_bytes(bytes);
  if (rc) return rc;
  if (na <= 0 || nb <= 0) return MCS_OK;
  dim3 g((na + kHamThreads - 1) / kHamThreads, (nb + kHamTile - 1) / kHamTile);
  MCS_DISPATCH_W(bytes, k_dense, g, dim3(kHamThreads), 0, (hipStream_t)stream, d_a, na, d_b, nb,
                 d_dist);
  MCS_HIP_CHECK(hipGetLastError());
  return MCS_OK;
}

int mcs_hamming_top2_device(const uint8_t* d_q, int32_t nq, const uint8_t* d_t, int32_t nt,
                            int32_t bytes, int32_t* d_best_idx, int32_t* d_best_dist,
                            int32_t* d_second_idx, int32_t* d_second_dist, void* stream) {
  int rc = check_bytes(bytes);
  if (rc) return rc;
  if (nq <= 0) return MCS_OK;
  if (nt > 65535) { set_error("top2: at most 65535 train descriptors"); return MCS_ERR_ARG; }
  if (bytes == 32) {
    auto* kfn = nt <= (1 << kKeyBits) ? k_top2_mfma32<true> : k_top2_mfma32<false>;
    hipLaunchKernelGGL(kfn, dim3((nq + 255) / 256, 1), dim3(256), 0, (hipStream_t)stream,
                       d_q, d_t, (const int32_t*)nullptr, (const int32_t*)nullptr, (int64_t)0, nq,
                       nt, nq, d_best_idx, d_best_dist, d_second_idx, d_second_dist);
    MCS_HIP_CHECK(hipGetLastError());
    return MCS_OK;
  }
  dim3 g((nq + kHamThreads * kQPT - 1) / (kHamThreads * kQPT), 1);
  MCS_DISPATCH_W(bytes, k_top2, g, dim3(kHamThreads), 0, (hipStream_t)stream, d_q, d_t,
                 (const int32_t*)nullptr, (const int32_t*)nullptr, (int64_t)0, nq, nt, nq,
                 d_best_idx, d_best_dist, d_second_idx, d_second_dist);
  MCS_HIP_CHECK(hipGetLastError());
  return MCS_OK;
}

int mcs_hamming_top2_batch_device(const uint8_t* d_desc, const int32_t* d_counts,
                                  const int32_t* d_pairs, int32_t n_pairs, int32_t cap,
                                  int32_t bytes, int32_t* d_best_idx, int32_t* d_best_dist,
                                  int32_t* d_second_idx, int32_t* d_second_dist, void* stream) {
  int rc = check_bytes(bytes);
  if (rc) return rc;
  if (n_pairs <= 0) return MCS_OK;
  if (!d_desc || !d_counts || !d_pairs || cap <= 0) return MCS_ERR_ARG;
  if (cap > 65535) { set_error("top2: capacity above 65535"); return MCS_ERR_ARG; }
  if (bytes == 32) {   // a pair's train count is <= cap
    auto* kfn = cap <= (1 << kKeyBits) ? k_top2_mfma32<true> : k_top2_mfma32<false>;
    hipLaunchKernelGGL(kfn, dim3((cap + 255) / 256, n_pairs), dim3(256), 0,
                       (hipStream_t)stream, d_desc, d_desc, d_counts, d_pairs,
                       (int64_t)cap * bytes, 0, 0, cap, d_best_idx, d_best_dist, d_second_idx,
                       d_second_dist);
    MCS_HIP_CHECK(hipGetLastError());
    return MCS_OK;
  }
  dim3 g((cap + kHamThreads * kQPT - 1) / (kHamThreads * kQPT), n_pairs);
  MCS_DISPATCH_W(bytes, k_top2, g, dim3(kHamThreads), 0, (hipStream_t)stream, d_desc, d_desc,
                 d_counts, d_pairs, (int64_t)cap * bytes, 0, 0, cap, d_best_idx, d_best_dist,
                 d_second_idx, d_second_dist);
  MCS_HIP_CHECK(hipGetLastError());
  return MCS_OK;
}

}  // extern "C"

namespace mcs {

// CheckDistEpipolarLine (src/misc.cpp:54-70).  nom = (ray2^T E12) ray1 evaluated left to right
// as cv::Matx does; (ray2^T E12)_c = sum_r ray2_r E_rc is exactly Etx2_c, so nom = Etx2 . ray1.
// One definition for the host entry and the device search (same operation order, no FMA
// contraction on either side: -ffp-contract=off), so both give the same verdict bit for bit.
__host__ __device__ __forceinline__ bool epi_check(const double* r1, const double* r2,
                                                   const double* Em, double thresh) {
  double Ex1[3], Etx2[3];
  for (int r = 0; r < 3; r++) {
    Ex1[r] = Em[3 * r] * r1[0] + Em[3 * r + 1] * r1[1] + Em[3 * r + 2] * r1[2];
    Etx2[r] = r2[0] * Em[r] + r2[1] * Em[3 + r] + r2[2] * Em[6 + r];
  }
  const double nom = Etx2[0] * r1[0] + Etx2[1] * r1[1] + Etx2[2] * r1[2];
  const double den = Ex1[0] * Ex1[0] + Ex1[1] * Ex1[1] + Ex1[2] * Ex1[2] + Etx2[0] * Etx2[0] +
                     Etx2[1] * Etx2[1] + Etx2[2] * Etx2[2];
  if (den == 0.0) return false;
  return (nom * nom) / den < thresh;
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}

// ---- SearchForTriangulationRaw on the device (src/cORBmatcher.cpp:1016-1089)
// The reference walks KF1's keypoints in index order; for each it sorts the (dist, idx2) list of
// unmatched same-camera KF2 keypoints with dist <= TH_LOW, takes best = the first list entry,
// and accepts the first entry with dist <= cvRound(2 best) that passes CheckDistEpipolarLine,
// marking it in vbMatched2.  With keys (dist << 20 | idx2) the sorted order is key order.  The
// only state between queries is vbMatched2, and KF2 keypoint i2 can only be taken by a query
// that lists it AND passes the epipolar check with it.  Kernels (stream-ordered):
//   k_tri_radius  (query tiles x train segments): each (query, segment) thread appends its
//                 candidate keys to its own kTriSub slots (no returning atomics in the loop),
//                 counts how many queries list each KF2 keypoint, flags slot overflow
//   k_tri_pass    (one thread per query and segment): the epipolar verdict of every stored
//                 candidate into bit 30, and how many queries pass with each KF2 keypoint
//   k_tri_private (one thread per query): a query none of whose candidates another query could
//                 take, and none of whose passing candidates another query lists, decides alone
//                 (its outcome neither depends on nor changes anyone's vbMatched2 view); the
//                 others are marked -2 and flagged for the ordered pass.  After any overflow the
//                 pass counts are incomplete, so every query goes to the ordered pass.
//   two exclusive scans (rocPRIM) give each flagged query its place and key offset
//   k_tri_gather  (one wave per flagged query): its keys sorted into one flat array, flagged
//                 queries in index order
//   k_tri_seq     (one wave per camera): the flagged queries in index order against an LDS
//                 vbMatched2 bitmap, streaming the flat keys through two LDS windows with the
//                 next window prefetched; per query a ballot finds the first unmatched key
//                 (best) and a second the first unmatched passing key with dist <= 2 best.  A
//                 query whose candidates overflowed a slot rescans KF2 on the fly (exact, rare).
constexpr int kTriSeg = 16;                 // train segments of k_tri_radius (grid.y)
constexpr int kTriSub = 96;                 // candidate slots per (query, segment)
constexpr int kTriCap = kTriSeg * kTriSub;  // per query
constexpr int kTriWin = 1024;    // keys per k_tri_seq LDS window (16 per lane)
constexpr uint32_t kTriPass = 1u << 30, kTriKey = kTriPass - 1;

template <int W, bool MASKED>
__global__ __launch_bounds__(kHamThreads) void k_tri_radius(
    const uint8_t* __restrict__ A, const uint8_t* __restrict__ MA, const int32_t* __restrict__ camA,
    const uint8_t* __restrict__ hasA, int na, const uint8_t* __restrict__ B,
    const uint8_t* __restrict__ MB, const int32_t* __restrict__ camB,
    const uint8_t* __restrict__ hasB, int nb, int ncams, int th, uint32_t* __restrict__ cand,
    int32_t* __restrict__ cnt, int32_t* __restrict__ ref_all, int32_t* __restrict__ overflow) {
  __shared__ uint4 tile[kHamTile * (W / 4)];
  __shared__ uint4 mtile[MASKED ? kHamTile * (W / 4) : 1];
  __shared__ int tcam[kHamTile];
  const int qi = blockIdx.x * kHamThreads + threadIdx.x;
  const int seg = blockIdx.y;
  uint32_t q[W], qm[W];
  int qc = -1;
#pragma unroll
  for (int w = 0; w < W; w++) { q[w] = 0; qm[w] = 0; }
  if (qi < na) {
    qc = camA[qi];
    if (hasA[qi] || qc < 0 || qc >= ncams) qc = -1;   // inactive: no candidates
  }
  if (qc >= 0) {
    load_desc_row<W>(q, A + (int64_t)qi * W * 4);
    if (MASKED) load_desc_row<W>(qm, MA + (int64_t)qi * W * 4);
  }
  uint32_t* const out = cand + ((int64_t)(qi < na ? qi : 0) * kTriSeg + seg) * kTriSub;
  int n = 0;
  const int per = ((nb + kTriSeg - 1) / kTriSeg + kHamTile - 1) / kHamTile * kHamTile;
  const int tb = seg * per, te = min(nb, tb + per);
  for (int t0 = tb; t0 < te; t0 += kHamTile) {
    const int nt_tile = min(kHamTile, te - t0);
    __syncthreads();
    const uint4* src = reinterpret_cast<const uint4*>(B + (int64_t)t0 * W * 4);
    for (int i = threadIdx.x; i < nt_tile * (W / 4); i += kHamThreads) tile[i] = src[i];
    if (MASKED) {
      const uint4* msrc = reinterpret_cast<const uint4*>(MB + (int64_t)t0 * W * 4);
      for (int i = threadIdx.x; i < nt_tile * (W / 4); i += kHamThreads) mtile[i] = msrc[i];
    }
    for (int i = threadIdx.x; i < nt_tile; i += kHamThreads)
      tcam[i] = hasB[t0 + i] ? -2 : camB[t0 + i];
    __syncthreads();
    if (qc < 0) continue;
    for (int j = 0; j < nt_tile; j++) {
      if (tcam[j] != qc) continue;
      const int d = MASKED ? ham_dist_masked_v<W>(q, qm, &tile[j * (W / 4)], &mtile[j * (W / 4)])
                           : ham_dist_v<W>(q, &tile[j * (W / 4)]);
      if (d <= th) {
        const int i2 = t0 + j;
        if (n < kTriSub) out[n] = ((uint32_t)d << 20) | (uint32_t)i2;
        n++;
        atomicAdd(ref_all + i2, 1);
      }
    }
  }
  if (qi < na) {
    cnt[(int64_t)qi * kTriSeg + seg] = n;
    if (n > kTriSub) atomicOr(overflow, 1);
  }
}

__global__ __launch_bounds__(256) void k_tri_pass(const int32_t* __restrict__ camA,
                                                  const double* __restrict__ raysA, int na,
                                                  const double* __restrict__ raysB, int ncams,
                                                  const double* __restrict__ E, double thresh,
                                                  uint32_t* __restrict__ cand,
                                                  const int32_t* __restrict__ cnt,
                                                  int32_t* __restrict__ ref_pass) {
  const int gt = blockIdx.x * 256 + threadIdx.x;
  if (gt >= na * kTriSeg) return;
  const int n = min(cnt[gt], kTriSub);
  if (n == 0) return;
  const int qi = gt / kTriSeg, qc = camA[qi];
  double r1[3], Em[9];
  for (int k = 0; k < 3; k++) r1[k] = raysA[3 * (int64_t)qi + k];
  // same camera only (:1040-1041): E[cam1][cam2] with cam2 == cam1
  for (int k = 0; k < 9; k++) Em[k] = E[9 * ((int64_t)qc * ncams + qc) + k];
  uint32_t* const ks = cand + (int64_t)gt * kTriSub;
  for (int i = 0; i < n; i++) {
    const uint32_t key = ks[i];
    const int i2 = (int)(key & 0xFFFFFu);
    if (epi_check(r1, raysB + 3 * (int64_t)i2, Em, thresh)) {
      ks[i] = key | kTriPass;
      atomicAdd(ref_pass + i2, 1);
    }
  }
}

__global__ __launch_bounds__(256) void k_tri_private(const uint32_t* __restrict__ cand,
                                                     const int32_t* __restrict__ cnt_in,
                                                     const int32_t* __restrict__ ref_all,
                                                     const int32_t* __restrict__ ref_pass,
                                                     const int32_t* __restrict__ overflow, int na,
                                                     int32_t* __restrict__ m12,
                                                     int32_t* __restrict__ n_matches,
                                                     int32_t* __restrict__ flag,
                                                     int32_t* __restrict__ len) {
  const int qi = blockIdx.x * 256 + threadIdx.x;
  int won = 0;
  if (qi < na) {
    int c = 0;
    bool over = false;
    for (int sg = 0; sg < kTriSeg; sg++) {
      const int n = cnt_in[(int64_t)qi * kTriSeg + sg];
      over = over || n > kTriSub;
      c += n;
    }
    over = over || c > kTriWin;   // k_tri_seq keeps a query's keys inside two LDS windows
    int r = -1, fl = 0, ln = 0;
    if (over) {
      r = -2; fl = 1;   // ln = 0: k_tri_seq rescans
    } else if (c > 0) {
      bool alone = *overflow == 0;
      uint32_t best = 0xFFFFFFFFu;
      for (int sg = 0; sg < kTriSeg; sg++) {
        const uint32_t* k = cand + ((int64_t)qi * kTriSeg + sg) * kTriSub;
        const int n = cnt_in[(int64_t)qi * kTriSeg + sg];
        for (int i = 0; i < n; i++) {
          const uint32_t key = k[i];
          const int i2 = (int)(key & 0xFFFFFu), own = (key & kTriPass) ? 1 : 0;
          best = min(best, key & kTriKey);
          if (own && ref_all[i2] > 1) alone = false;       // it could take a key another lists
          if (ref_pass[i2] - own > 0) alone = false;      // another could take one of its keys
        }
      }
      if (!alone) {
        r = -2; fl = 1; ln = c;
      } else {
        const uint32_t th = 2u * (best >> 20);   // cvRound(2 * bestDist), integer distance
        uint32_t win = 0xFFFFFFFFu;
        for (int sg = 0; sg < kTriSeg; sg++) {
          const uint32_t* k = cand + ((int64_t)qi * kTriSeg + sg) * kTriSub;
          const int n = cnt_in[(int64_t)qi * kTriSeg + sg];
          for (int i = 0; i < n; i++) {
            const uint32_t key = k[i];
            if ((key & kTriPass) && ((key & kTriKey) >> 20) <= th) win = min(win, key & kTriKey);
          }
        }
        if (win != 0xFFFFFFFFu) { r = (int)(win & 0xFFFFFu); won = 1; }
      }
    }
    m12[qi] = r;
    flag[qi] = fl;
    len[qi] = ln;
  } else if (qi == na) {   // the scans' total slot
    flag[qi] = 0;
    len[qi] = 0;
  }
  const int s = dev::wave_sum(won);
  if ((threadIdx.x & 63) == 0 && s) atomicAdd(n_matches, s);
}

// one wave per flagged query: its keys (the segments' lists), ascending by (dist, idx2), to
// flat[koff[q] ...); the entry (q, offset, count, camera) at its place pos[q] of the ordered list
__global__ __launch_bounds__(256) void k_tri_gather(const uint32_t* __restrict__ cand,
                                                    const int32_t* __restrict__ cnt_in,
                                                    const int32_t* __restrict__ cam,
                                                    const int32_t* __restrict__ flag,
                                                    const int32_t* __restrict__ len,
                                                    const int32_t* __restrict__ pos,
                                                    const int32_t* __restrict__ koff, int na,
                                                    uint32_t* __restrict__ flat,
                                                    int4* __restrict__ entries) {
  __shared__ uint32_t sk[4][kTriCap];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int q = blockIdx.x * 4 + wv;
  if (q >= na || !flag[q]) return;
  const int c = len[q], o = koff[q];
  if (lane == 0) entries[pos[q]] = make_int4(q, o, c, cam[q]);
  int at = 0;
  for (int sg = 0; sg < kTriSeg && c > 0; sg++) {
    const int n = cnt_in[(int64_t)q * kTriSeg + sg];
    const uint32_t* src = cand + ((int64_t)q * kTriSeg + sg) * kTriSub;
    for (int i = lane; i < n; i += 64) sk[wv][at + i] = src[i];
    at += n;
  }
  dev::wave_sync();
  for (int i = lane; i < c; i += 64) {   // rank by counting (keys are distinct: idx2 differs)
    const uint32_t key = sk[wv][i], kk = key & kTriKey;
    int rank = 0;
    for (int j = 0; j < c; j++) rank += (sk[wv][j] & kTriKey) < kk;
    flat[o + rank] = key;
  }
}

__device__ __forceinline__ int first_lane(uint64_t m) { return (int)__builtin_ctzll(m); }

// One wave per camera (a query's candidates are KF2 keypoints of its own camera, so cameras
// never share vbMatched2 bits): the wave walks the ordered flagged list, takes its camera's
// entries, and streams their keys through two LDS windows of its own.
template <int W, bool MASKED>
__global__ __launch_bounds__(512) void k_tri_seq(
    const uint8_t* __restrict__ A, const uint8_t* __restrict__ MA, const int32_t* __restrict__ camA,
    const double* __restrict__ raysA, const uint8_t* __restrict__ B,
    const uint8_t* __restrict__ MB, const int32_t* __restrict__ camB,
    const uint8_t* __restrict__ hasB, const double* __restrict__ raysB, int na, int nb, int ncams,
    const double* __restrict__ E, int th_low, double thresh, const uint32_t* __restrict__ flat,
    const int4* __restrict__ entries, const int32_t* __restrict__ pos,
    int32_t* __restrict__ m12, int32_t* __restrict__ n_matches) {
  extern __shared__ uint32_t smem[];
  const int cam = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  uint32_t* const matched2 = smem;                                 // vbMatched2 bitmap, nb bits
  const int nwords = (nb + 31) >> 5;
  uint32_t* const win = smem + ((nwords + 3) & ~3) + cam * 2 * kTriWin;   // this wave's windows
  for (int i = threadIdx.x; i < nwords; i += blockDim.x) matched2[i] = 0u;
  __syncthreads();
  if (cam >= ncams) return;
  const int ns = pos[na];                         // flagged queries
  auto is_matched = [&](uint32_t i2) { return (matched2[i2 >> 5] >> (i2 & 31)) & 1u; };
  constexpr int R = kTriWin / 64;
  uint32_t pre[R];
  auto load_win = [&](int wj, uint32_t (&v)[R]) {
#pragma unroll
    for (int k = 0; k < R; k++) v[k] = flat[(int64_t)wj * kTriWin + 64 * k + lane];
  };
  auto store_win = [&](int wj, const uint32_t (&v)[R]) {
#pragma unroll
    for (int k = 0; k < R; k++) win[(wj & 1) * kTriWin + 64 * k + lane] = v[k];
  };
  // windows cw, cw + 1 are in LDS (slots cw & 1, (cw + 1) & 1), window cw + 2 in flight; the
  // flat array is padded by three windows (workspace), so whole-window loads stay inside it
  int cw = -8;
  auto ensure = [&](int o) {
    const int w0 = o / kTriWin;
    if (w0 == cw) return;
    if (w0 == cw + 1) {
      store_win(cw + 2, pre);
      cw++;
    } else {
      uint32_t v0[R], v1[R];
      load_win(w0, v0);
      load_win(w0 + 1, v1);
      store_win(w0, v0);
      store_win(w0 + 1, v1);
      cw = w0;
    }
    load_win(cw + 2, pre);
    dev::wave_sync();
  };
  auto key_at = [&](int g) { return win[((g / kTriWin) & 1) * kTriWin + (g % kTriWin)]; };
  int nm = 0;
  int4 ent = lane < ns ? entries[lane] : make_int4(0, 0, 0, -1);
  for (int base = 0; base < ns; base += 64) {
    const int4 cur = ent;
    if (base + 64 + lane < ns) ent = entries[base + 64 + lane];   // next chunk's entries
    uint64_t todo = __ballot(base + lane < ns && cur.w == cam);
    while (todo) {
      const int i = first_lane(todo);
      todo &= todo - 1;
      const int q = __builtin_amdgcn_readlane(cur.x, i);
      const int o = __builtin_amdgcn_readlane(cur.y, i);
      const int c = __builtin_amdgcn_readlane(cur.z, i);
      // Two short queries at once, one per 32-lane half, from one key read and one vbMatched2
      // read: the second decides on the first's state plus the first's winner (its bit is
      // cleared from the second's unmatched keys before its own best is taken), which is the
      // sequential order.  Both must lie in the two resident windows.
      if (todo && c > 0 && c <= 32) {
        const int j = first_lane(todo);
        const int c2 = __builtin_amdgcn_readlane(cur.z, j);
        const int o2 = __builtin_amdgcn_readlane(cur.y, j);
        if (c2 > 0 && c2 <= 32 && o2 + c2 - o <= kTriWin) {
          todo &= todo - 1;
          const int q2 = __builtin_amdgcn_readlane(cur.x, j);
          ensure(o);
          const bool hi = lane >= 32;
          const int li = lane & 31;
          const bool valid = li < (hi ? c2 : c);
          const uint32_t key = valid ? key_at((hi ? o2 : o) + li) : 0u;
          const uint32_t kid = key & 0xFFFFFu;
          const bool unm = valid && !is_matched(kid);
          const uint64_t bu = __ballot(unm);
          uint32_t w1 = 0xFFFFFFFFu, w2 = 0xFFFFFFFFu;
          const uint64_t b1 = bu & 0xFFFFFFFFull;
          if (b1) {
            const uint32_t best = (uint32_t)__builtin_amdgcn_readlane((int)key, first_lane(b1)) & kTriKey;
            const uint32_t th = 2u * (best >> 20);
            const uint64_t bo = __ballot(!hi && unm && (key & kTriPass) && ((key & kTriKey) >> 20) <= th);
            if (bo) w1 = (uint32_t)__builtin_amdgcn_readlane((int)key, first_lane(bo)) & kTriKey;
          }
          const uint32_t r1k = w1 != 0xFFFFFFFFu ? (w1 & 0xFFFFFu) : 0xFFFFFFFFu;
          const bool unm2 = hi && unm && kid != r1k;
          const uint64_t b2 = __ballot(unm2);
          if (b2) {
            const uint32_t best = (uint32_t)__builtin_amdgcn_readlane((int)key, first_lane(b2)) & kTriKey;
            const uint32_t th = 2u * (best >> 20);
            const uint64_t bo = __ballot(unm2 && (key & kTriPass) && ((key & kTriKey) >> 20) <= th);
            if (bo) w2 = (uint32_t)__builtin_amdgcn_readlane((int)key, first_lane(bo)) & kTriKey;
          }
          const int r1 = w1 != 0xFFFFFFFFu ? (int)(w1 & 0xFFFFFu) : -1;
          const int r2 = w2 != 0xFFFFFFFFu ? (int)(w2 & 0xFFFFFu) : -1;
          if (lane == 0) {
            m12[q] = r1;
            m12[q2] = r2;
            if (r1 >= 0) atomicOr(&matched2[r1 >> 5], 1u << (r1 & 31));
            if (r2 >= 0) atomicOr(&matched2[r2 >> 5], 1u << (r2 & 31));
          }
          nm += (r1 >= 0) + (r2 >= 0);
          continue;
        }
      }
      uint32_t wkey = 0xFFFFFFFFu;
      if (c > 0) {
        ensure(o);
        if (c <= 64) {   // one round: best and winner from the same reads
          const bool valid = lane < c;
          const uint32_t key = valid ? key_at(o + lane) : 0u;
          const bool unm = valid && !is_matched(key & 0xFFFFFu);
          const uint64_t bu = __ballot(unm);
          if (bu) {
            const uint32_t best = (uint32_t)__builtin_amdgcn_readlane((int)key, first_lane(bu)) & kTriKey;
            const uint32_t th = 2u * (best >> 20);
            const uint64_t bo = __ballot(unm && (key & kTriPass) && ((key & kTriKey) >> 20) <= th);
            if (bo) wkey = (uint32_t)__builtin_amdgcn_readlane((int)key, first_lane(bo)) & kTriKey;
          }
        } else {
          int rb = -1;
          uint32_t best = 0;
          for (int r = 0; r * 64 < c; r++) {
            const bool valid = r * 64 + lane < c;
            const uint32_t key = valid ? key_at(o + r * 64 + lane) : 0u;
            const uint64_t b = __ballot(valid && !is_matched(key & 0xFFFFFu));
            if (b) { best = (uint32_t)__builtin_amdgcn_readlane((int)key, first_lane(b)) & kTriKey; rb = r; break; }
          }
          if (rb >= 0) {
            const uint32_t th = 2u * (best >> 20);
            for (int r = rb; r * 64 < c; r++) {
              const bool valid = r * 64 + lane < c;
              const uint32_t key = valid ? key_at(o + r * 64 + lane) : 0xFFFFFFFFu;
              const uint32_t d = (key & kTriKey) >> 20;
              const uint64_t b = __ballot(valid && (key & kTriPass) && d <= th && !is_matched(key & 0xFFFFFu));
              if (b) { wkey = (uint32_t)__builtin_amdgcn_readlane((int)key, first_lane(b)) & kTriKey; break; }
              // keys ascend: once a round's last key is past the threshold, no later key qualifies
              if ((((uint32_t)__builtin_amdgcn_readlane((int)key, 63) & kTriKey) >> 20) > th) break;
            }
          }
        }
      } else {
        // more candidates than a slot holds: rescan KF2 for this query (same filters)
        const int qc = camA[q];
        uint32_t qd[W], qmk[W];
        load_desc_row<W>(qd, A + (int64_t)q * W * 4);
        if (MASKED) load_desc_row<W>(qmk, MA + (int64_t)q * W * 4);
        else
          for (int w = 0; w < W; w++) qmk[w] = 0;
        auto dist_to = [&](int i2) {
          uint32_t t[W], tm[W];
          load_desc_row<W>(t, B + (int64_t)i2 * W * 4);
          int d = 0;
          if (MASKED) {
            load_desc_row<W>(tm, MB + (int64_t)i2 * W * 4);
            for (int w = 0; w < W; w++) {
              const uint32_t x = qd[w] ^ t[w];
              d += __popc(x & qmk[w]) + __popc(x & tm[w]);
            }
            d /= 2;
          } else {
            for (int w = 0; w < W; w++) d += __popc(qd[w] ^ t[w]);
          }
          return d;
        };
        uint32_t lbest = 0xFFFFFFFFu;
        for (int i2 = lane; i2 < nb; i2 += 64) {
          if (camB[i2] != qc || hasB[i2] || is_matched((uint32_t)i2)) continue;
          const int d = dist_to(i2);
          if (d <= th_low) lbest = min(lbest, ((uint32_t)d << 20) | (uint32_t)i2);
        }
        const uint32_t best = wave_min_u32(lbest);
        if (best != 0xFFFFFFFFu) {
          const int th = 2 * (int)(best >> 20);
          double r1[3], Em[9];
          for (int k = 0; k < 3; k++) r1[k] = raysA[3 * (int64_t)q + k];
          for (int k = 0; k < 9; k++) Em[k] = E[9 * ((int64_t)qc * ncams + qc) + k];
          uint32_t lw = 0xFFFFFFFFu;
          for (int i2 = lane; i2 < nb; i2 += 64) {
            if (camB[i2] != qc || hasB[i2] || is_matched((uint32_t)i2)) continue;
            const int d = dist_to(i2);
            if (d <= th_low && d <= th && epi_check(r1, raysB + 3 * (int64_t)i2, Em, thresh))
              lw = min(lw, ((uint32_t)d << 20) | (uint32_t)i2);
          }
          wkey = wave_min_u32(lw);
        }
      }
      const int r = wkey != 0xFFFFFFFFu ? (int)(wkey & 0xFFFFFu) : -1;
      if (lane == 0) {
        m12[q] = r;
        // LDS atomics of one wave execute in order with its later LDS reads
        if (r >= 0) atomicOr(&matched2[r >> 5], 1u << (r & 31));
      }
      nm += r >= 0;
    }
  }
  if (lane == 0 && nm) atomicAdd(n_matches, nm);
}

// ---- ComputeE per camera pair (src/misc.cpp:72-86) as SearchForTriangulationRaw builds its
// Es table (src/cORBmatcher.cpp:985-998): Es[i][j] = ComputeE(KF1.Get_MtMc_inv(i),
// KF2.Get_MtMc(j)), with MtMc = cayley2hom(M_t) * cayley2hom(M_c) and MtMc_inv =
// cConverter::invMat(MtMc) (cMultiCamSys_::Set_M_t_from_min, src/cam_system_omni.cpp:170-183).
// Every product accumulates s = 0; s += a(i,k) b(k,j) in k order (cv::Matx), `t12 /= norm`
// multiplies by 1./norm (cv::Vec::operator/=), norm = sqrt of the in-order sum of squares.
// Tiny 3x3 / 4x4 host math: nothing here is worth a device launch.
static void host_matmul(const double* a, const double* b, double* c, int m, int l, int n) {
  for (int i = 0; i < m; i++)
    for (int j = 0; j < n; j++) {
      double s = 0;
      for (int k = 0; k < l; k++) s += a[i * l + k] * b[k * n + j];
      c[i * n + j] = s;
    }
}

static void host_cayley2hom(const double* p, double* T) {  // include/misc.h:134-162, 213-226
  const double c1 = p[0], c2 = p[1], c3 = p[2];
  const double c1s = c1 * c1, c2s = c2 * c2, c3s = c3 * c3;
  const double scale = 1.0 + c1s + c2s + c3s;
  const double R[9] = {1 + c1s - c2s - c3s, 2 * (c1 * c2 - c3), 2 * (c1 * c3 + c2),
                       2 * (c1 * c2 + c3), 1 - c1s + c2s - c3s, 2 * (c2 * c3 - c1),
                       2 * (c1 * c3 - c2), 2 * (c2 * c3 + c1), 1 - c1s - c2s + c3s};
  const double inv = 1 / scale;  // R = (1 / scale) * R
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) T[4 * i + j] = R[3 * i + j] * inv;
    T[4 * i + 3] = p[3 + i];
  }
  T[12] = T[13] = T[14] = 0.0;
  T[15] = 1.0;
}

static void host_inv_mat(const double* M, double* O) {  // src/cConverter.cpp:31-44
  double Rt[9], t[3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) Rt[3 * i + j] = M[4 * j + i];
  for (int i = 0; i < 3; i++) {  // t = -R * t
    double s = 0;
    for (int k = 0; k < 3; k++) s += (Rt[3 * i + k] * -1.0) * M[4 * k + 3];
    t[i] = s;
  }
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) O[4 * i + j] = Rt[3 * i + j];
    O[4 * i + 3] = t[i];
  }
  O[12] = O[13] = O[14] = 0.0;
  O[15] = 1.0;
}

static void host_compute_e(const double* T1, const double* T2, double* E) {  // misc.cpp:72-86
  double R1w[9], R2wt[9], nR1w[9], R12[9], A[9], t12[3], t1w[3], t2w[3];
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) {
      R1w[3 * i + j] = T1[4 * i + j];
      nR1w[3 * i + j] = T1[4 * i + j] * -1.0;
      R2wt[3 * i + j] = T2[4 * j + i];
    }
    t1w[i] = T1[4 * i + 3];
    t2w[i] = T2[4 * i + 3];
  }
  host_matmul(R1w, R2wt, R12, 3, 3, 3);   // R12 = R1w * R2w.t()
  host_matmul(nR1w, R2wt, A, 3, 3, 3);    // t12 = -R1w * R2w.t() * t2w + t1w
  host_matmul(A, t2w, t12, 3, 3, 1);
  for (int i = 0; i < 3; i++) t12[i] = t12[i] + t1w[i];
  double ss = 0;
  for (int i = 0; i < 3; i++) ss += t12[i] * t12[i];
  const double ialpha = 1. / std::sqrt(ss);  // t12 /= cv::norm(t12)
  for (int i = 0; i < 3; i++) t12[i] = t12[i] * ialpha;
  const double S[9] = {0.0, -t12[2], t12[1], t12[2], 0.0, -t12[0], -t12[1], t12[0], 0.0};  // Skew
  host_matmul(S, R12, E, 3, 3, 3);        // t12x * R12
}

}  // namespace mcs

// Workspace of the device search (sized at creation; reused call after call on one stream).
struct mcs_tri_workspace {
  int device = 0, max_n1 = 0, max_n2 = 0;
  uint32_t* cand = nullptr;     // [max_n1][kTriCap] candidate keys
  uint32_t* flat = nullptr;     // [max_n1 * kTriCap + 3 kTriWin] sorted keys of flagged queries
  int4* entries = nullptr;      // [max_n1] (query, key offset, count)
  int32_t* cnt = nullptr;       // [max_n1][kTriSeg]
  int32_t* overflow = nullptr;  // [1] a (query, segment) overflowed its slots
  int32_t* flag = nullptr;      // [max_n1 + 1]
  int32_t* len = nullptr;       // [max_n1 + 1]
  int32_t* pos = nullptr;       // [max_n1 + 1]
  int32_t* koff = nullptr;      // [max_n1 + 1]
  int32_t* ref_all = nullptr;   // [max_n2]
  int32_t* ref_pass = nullptr;  // [max_n2]
  void* scan_tmp = nullptr; size_t scan_bytes = 0;
};

namespace mcs {

static size_t tri_lds_bytes(int n2, int ncams) {
  return (size_t)ncams * 2 * kTriWin * 4 + (size_t)(((n2 + 31) / 32 + 3) & ~3) * 4;
}

// Device pipeline on device buffers (stream-ordered; no host synchronisation).
static hipError_t tri_run(mcs_tri_workspace* ws, const uint8_t* dA, const uint8_t* dmA, const int32_t* dcA,
                          const uint8_t* dhA, const double* drA, int n1, const uint8_t* dB, const uint8_t* dmB,
                          const int32_t* dcB, const uint8_t* dhB, const double* drB, int n2, int ncams,
                          const double* dE, int bytes, int th_low, double thresh, int32_t* m12,
                          int32_t* nmatch, hipStream_t st) {
  hipError_t e = hipMemsetAsync(nmatch, 0, sizeof(int32_t), st);
  if (e == hipSuccess) e = hipMemsetAsync(ws->overflow, 0, sizeof(int32_t), st);
  if (e == hipSuccess) e = hipMemsetAsync(ws->ref_all, 0, sizeof(int32_t) * (size_t)n2, st);
  if (e == hipSuccess) e = hipMemsetAsync(ws->ref_pass, 0, sizeof(int32_t) * (size_t)n2, st);
  if (e != hipSuccess) return e;
  const bool masked = dmA != nullptr;
  const dim3 g((n1 + kHamThreads - 1) / kHamThreads, kTriSeg);
#define MCS_TRI_RADIUS(WW, MM)                                                                   \
  hipLaunchKernelGGL((k_tri_radius<WW, MM>), g, dim3(kHamThreads), 0, st, dA, dmA, dcA, dhA, n1, dB,  \
                     dmB, dcB, dhB, n2, ncams, th_low, ws->cand, ws->cnt, ws->ref_all, ws->overflow)
  if (bytes == 16) { if (masked) MCS_TRI_RADIUS(4, true); else MCS_TRI_RADIUS(4, false); }
  else if (bytes == 32) { if (masked) MCS_TRI_RADIUS(8, true); else MCS_TRI_RADIUS(8, false); }
  else { if (masked) MCS_TRI_RADIUS(16, true); else MCS_TRI_RADIUS(16, false); }
#undef MCS_TRI_RADIUS
  hipLaunchKernelGGL(k_tri_pass, dim3((n1 * kTriSeg + 255) / 256), dim3(256), 0, st, dcA, drA, n1, drB, ncams, dE,
                     thresh, ws->cand, ws->cnt, ws->ref_pass);
  hipLaunchKernelGGL(k_tri_private, dim3((n1 + 1 + 255) / 256), dim3(256), 0, st, ws->cand, ws->cnt, ws->ref_all,
                     ws->ref_pass, ws->overflow, n1, m12, nmatch, ws->flag, ws->len);
  auto plus = rocprim::plus<int32_t>();
  size_t b1 = ws->scan_bytes;
  if ((e = rocprim::exclusive_scan(ws->scan_tmp, b1, ws->flag, ws->pos, 0, (size_t)n1 + 1, plus, st)) != hipSuccess)
    return e;
  b1 = ws->scan_bytes;
  if ((e = rocprim::exclusive_scan(ws->scan_tmp, b1, ws->len, ws->koff, 0, (size_t)n1 + 1, plus, st)) != hipSuccess)
    return e;
  hipLaunchKernelGGL(k_tri_gather, dim3((n1 + 3) / 4), dim3(256), 0, st, ws->cand, ws->cnt, dcA, ws->flag, ws->len, ws->pos,
                     ws->koff, n1, ws->flat, ws->entries);
  const int lds = (int)tri_lds_bytes(n2, ncams);
  if (ncams > 8 || lds > 160 * 1024) return hipErrorInvalidValue;   // entry points check first
  const void* fn = nullptr;
#define MCS_TRI_SEQ_FN(WW, MM) fn = (const void*)&k_tri_seq<WW, MM>
  if (bytes == 16) { if (masked) MCS_TRI_SEQ_FN(4, true); else MCS_TRI_SEQ_FN(4, false); }
  else if (bytes == 32) { if (masked) MCS_TRI_SEQ_FN(8, true); else MCS_TRI_SEQ_FN(8, false); }
  else { if (masked) MCS_TRI_SEQ_FN(16, true); else MCS_TRI_SEQ_FN(16, false); }
#undef MCS_TRI_SEQ_FN
  if (lds > 64 * 1024 && (e = ldlt::set_lds_limit(fn, lds)) != hipSuccess) return e;
#define MCS_TRI_SEQ(WW, MM)                                                                       \
  hipLaunchKernelGGL((k_tri_seq<WW, MM>), dim3(1), dim3(64 * ncams), lds, st, dA, dmA, dcA, drA, dB, dmB, dcB, \
                     dhB, drB, n1, n2, ncams, dE, th_low, thresh, ws->flat, ws->entries, ws->pos, m12, \
                     nmatch)
  if (bytes == 16) { if (masked) MCS_TRI_SEQ(4, true); else MCS_TRI_SEQ(4, false); }
  else if (bytes == 32) { if (masked) MCS_TRI_SEQ(8, true); else MCS_TRI_SEQ(8, false); }
  else { if (masked) MCS_TRI_SEQ(16, true); else MCS_TRI_SEQ(16, false); }
#undef MCS_TRI_SEQ
  return hipGetLastError();
}

static int search_for_triangulation(const uint8_t* desc1, const uint8_t* mask1,
                                    const int32_t* cam1, const uint8_t* has_mp1,
                                    const double* rays1, int32_t n1, const uint8_t* desc2,
                                    const uint8_t* mask2, const int32_t* cam2,
                                    const uint8_t* has_mp2, const double* rays2, int32_t n2,
                                    int32_t ncams, const double* E, int32_t bytes, int32_t th_low,
                                    double epi_thresh, int32_t* matches12, int32_t* n_matches) {
  int rc = check_bytes(bytes);
  if (rc) return rc;
  if (!n_matches || (n1 > 0 && !matches12)) return MCS_ERR_ARG;
  *n_matches = 0;
  for (int i = 0; i < n1; i++) matches12[i] = -1;
  if (n1 <= 0 || n2 <= 0) return MCS_OK;
  // candidates are packed (dist << 20 | idx2): train index must fit 20 bits
  if (n2 >= (1 << 19)) { set_error("triangulation: at most 2^19 - 1 keypoints in KF2"); return MCS_ERR_ARG; }
  if (!desc1 || !desc2 || !cam1 || !cam2 || !has_mp1 || !has_mp2 || !rays1 || !rays2 || !E ||
      ncams <= 0)
    return MCS_ERR_ARG;
  if (ncams > 8) { set_error("triangulation: at most 8 cameras (one ordered-pass wave each)"); return MCS_ERR_UNSUPPORTED; }
  const bool masked = mask1 != nullptr;
  if (masked != (mask2 != nullptr)) { set_error("triangulation: masks for both keyframes or none"); return MCS_ERR_ARG; }
  for (int i = 0; i < n1; i++)
    if (cam1[i] < 0 || cam1[i] >= ncams) { set_error("triangulation: cam1 out of range"); return MCS_ERR_ARG; }
  for (int i = 0; i < n2; i++)
    if (cam2[i] < 0 || cam2[i] >= ncams) { set_error("triangulation: cam2 out of range"); return MCS_ERR_ARG; }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    set_error("no HIP device visible (no CPU fallback)");
    return MCS_ERR_NO_DEVICE;
  }
  // host entry: upload, run the device search, download (one synchronisation)
  uint8_t *dA = nullptr, *dB = nullptr, *dmA = nullptr, *dmB = nullptr, *dhA = nullptr,
          *dhB = nullptr;
  int32_t *dcA = nullptr, *dcB = nullptr, *dm12 = nullptr, *dn = nullptr;
  double *drA = nullptr, *drB = nullptr, *dE = nullptr;
  hipError_t e = hipSuccess;
  auto chk = [&](hipError_t x) { if (e == hipSuccess) e = x; };
  chk(hipMalloc((void**)&dA, (size_t)n1 * bytes));
  chk(hipMalloc((void**)&dB, (size_t)n2 * bytes));
  if (masked) {
    chk(hipMalloc((void**)&dmA, (size_t)n1 * bytes));
    chk(hipMalloc((void**)&dmB, (size_t)n2 * bytes));
    chk(hipMemcpy(dmA, mask1, (size_t)n1 * bytes, hipMemcpyHostToDevice));
    chk(hipMemcpy(dmB, mask2, (size_t)n2 * bytes, hipMemcpyHostToDevice));
  }
  chk(hipMalloc((void**)&dhA, n1));
  chk(hipMalloc((void**)&dhB, n2));
  chk(hipMalloc((void**)&dcA, 4 * (size_t)n1));
  chk(hipMalloc((void**)&dcB, 4 * (size_t)n2));
  chk(hipMalloc((void**)&drA, 24 * (size_t)n1));
  chk(hipMalloc((void**)&drB, 24 * (size_t)n2));
  chk(hipMalloc((void**)&dE, 72 * (size_t)ncams * ncams));
  chk(hipMalloc((void**)&dm12, 4 * (size_t)n1));
  chk(hipMalloc((void**)&dn, 4));
  chk(hipMemcpy(dA, desc1, (size_t)n1 * bytes, hipMemcpyHostToDevice));
  chk(hipMemcpy(dB, desc2, (size_t)n2 * bytes, hipMemcpyHostToDevice));
  chk(hipMemcpy(dhA, has_mp1, n1, hipMemcpyHostToDevice));
  chk(hipMemcpy(dhB, has_mp2, n2, hipMemcpyHostToDevice));
  chk(hipMemcpy(dcA, cam1, 4 * (size_t)n1, hipMemcpyHostToDevice));
  chk(hipMemcpy(dcB, cam2, 4 * (size_t)n2, hipMemcpyHostToDevice));
  chk(hipMemcpy(drA, rays1, 24 * (size_t)n1, hipMemcpyHostToDevice));
  chk(hipMemcpy(drB, rays2, 24 * (size_t)n2, hipMemcpyHostToDevice));
  chk(hipMemcpy(dE, E, 72 * (size_t)ncams * ncams, hipMemcpyHostToDevice));
  int dev = 0;
  chk(hipGetDevice(&dev));
  {
    // one workspace per device, kept for the process and grown on demand (a call holds the
    // lock for its whole run: calls on one device share the buffers)
    static std::mutex mu;
    static std::map<int, mcs_tri_workspace*> cache;
    std::lock_guard<std::mutex> g(mu);
    mcs_tri_workspace*& ws = cache[dev];
    if (e == hipSuccess && (!ws || ws->max_n1 < n1 || ws->max_n2 < n2)) {
      const int32_t g1 = ws ? std::max(ws->max_n1, n1) : n1, g2 = ws ? std::max(ws->max_n2, n2) : n2;
      if (ws) { mcs_tri_workspace_destroy(ws); ws = nullptr; }
      if ((rc = mcs_tri_workspace_create(dev, g1, g2, &ws)) != MCS_OK) { ws = nullptr; e = hipErrorOutOfMemory; }
    }
    if (e == hipSuccess)
      e = tri_run(ws, dA, dmA, dcA, dhA, drA, n1, dB, dmB, dcB, dhB, drB, n2, ncams, dE, bytes, th_low,
                  epi_thresh, dm12, dn, nullptr);
    chk(hipMemcpy(matches12, dm12, 4 * (size_t)n1, hipMemcpyDeviceToHost));
    chk(hipMemcpy(n_matches, dn, 4, hipMemcpyDeviceToHost));
  }
  void* bufs[] = {dA, dB, dmA, dmB, dhA, dhB, dcA, dcB, drA, drB, dE, dm12, dn};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  if (e != hipSuccess) {
    for (int i = 0; i < n1; i++) matches12[i] = -1;
    *n_matches = 0;
    set_hip_error(e, "triangulation search", __FILE__, __LINE__);
    return MCS_ERR_HIP;
  }
  return MCS_OK;
}

}  // namespace mcs

extern "C" {

int mcs_search_for_triangulation_raw(const uint8_t* desc1, const int32_t* cam1,
                                     const uint8_t* has_mp1, const double* rays1, int32_t n1,
                                     const uint8_t* desc2, const int32_t* cam2,
                                     const uint8_t* has_mp2, const double* rays2, int32_t n2,
                                     int32_t ncams, const double* E, int32_t bytes,
                                     int32_t th_low, double epi_thresh, int32_t* matches12,
                                     int32_t* n_matches) {
  return search_for_triangulation(desc1, nullptr, cam1, has_mp1, rays1, n1, desc2, nullptr, cam2,
                                  has_mp2, rays2, n2, ncams, E, bytes, th_low, epi_thresh,
                                  matches12, n_matches);
}

int mcs_search_for_triangulation_raw_masked(const uint8_t* desc1, const uint8_t* mask1,
                                            const int32_t* cam1, const uint8_t* has_mp1,
                                            const double* rays1, int32_t n1,
                                            const uint8_t* desc2, const uint8_t* mask2,
                                            const int32_t* cam2, const uint8_t* has_mp2,
                                            const double* rays2, int32_t n2, int32_t ncams,
                                            const double* E, int32_t bytes, int32_t th_low,
                                            double epi_thresh, int32_t* matches12,
                                            int32_t* n_matches) {
  if (!mask1 || !mask2) { set_error("triangulation: masked entry needs both masks"); return MCS_ERR_ARG; }
  return search_for_triangulation(desc1, mask1, cam1, has_mp1, rays1, n1, desc2, mask2, cam2,
                                  has_mp2, rays2, n2, ncams, E, bytes, th_low, epi_thresh,
                                  matches12, n_matches);
}

int mcs_tri_workspace_create(int32_t device, int32_t max_n1, int32_t max_n2, mcs_tri_workspace** out) {
  if (!out || max_n1 < 1 || max_n2 < 1 || max_n2 >= (1 << 19)) {
    set_error("tri workspace: need max_n1 >= 1 and 1 <= max_n2 < 2^19");
    return MCS_ERR_ARG;
  }
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) { set_error("no HIP device visible (no CPU fallback)"); return MCS_ERR_NO_DEVICE; }
  if (device < 0 || device >= ndev) { set_error("bad device ordinal"); return MCS_ERR_ARG; }
  MCS_HIP_CHECK(hipSetDevice(device));
  auto* w = new (std::nothrow) mcs_tri_workspace();
  if (!w) return MCS_ERR_ARG;
  w->device = device; w->max_n1 = max_n1; w->max_n2 = max_n2;
  const size_t n1 = (size_t)max_n1, n2 = (size_t)max_n2;
  hipError_t e = hipMalloc((void**)&w->cand, 4 * n1 * kTriCap);
  if (e == hipSuccess) e = hipMalloc((void**)&w->flat, 4 * (n1 * kTriCap + 3 * kTriWin));
  if (e == hipSuccess) e = hipMalloc((void**)&w->entries, sizeof(int4) * n1);
  if (e == hipSuccess) e = hipMalloc((void**)&w->cnt, 4 * n1 * kTriSeg);
  if (e == hipSuccess) e = hipMalloc((void**)&w->overflow, 4);
  if (e == hipSuccess) e = hipMalloc((void**)&w->flag, 4 * (n1 + 1));
  if (e == hipSuccess) e = hipMalloc((void**)&w->len, 4 * (n1 + 1));
  if (e == hipSuccess) e = hipMalloc((void**)&w->pos, 4 * (n1 + 1));
  if (e == hipSuccess) e = hipMalloc((void**)&w->koff, 4 * (n1 + 1));
  if (e == hipSuccess) e = hipMalloc((void**)&w->ref_all, 4 * n2);
  if (e == hipSuccess) e = hipMalloc((void**)&w->ref_pass, 4 * n2);
  if (e == hipSuccess)
    e = rocprim::exclusive_scan(nullptr, w->scan_bytes, w->flag, w->pos, 0, n1 + 1, rocprim::plus<int32_t>(),
                                (hipStream_t)0);
  if (e == hipSuccess) e = hipMalloc(&w->scan_tmp, std::max<size_t>(16, w->scan_bytes));
  if (e != hipSuccess) {
    mcs_tri_workspace_destroy(w);
    set_hip_error(e, "tri workspace", __FILE__, __LINE__);
    return MCS_ERR_HIP;
  }
  *out = w;
  return MCS_OK;
}

void mcs_tri_workspace_destroy(mcs_tri_workspace* w) {
  if (!w) return;
  (void)hipSetDevice(w->device);
  void* bufs[] = {w->cand, w->flat, w->entries, w->cnt, w->overflow, w->flag, w->len, w->pos, w->koff, w->ref_all,
                  w->ref_pass, w->scan_tmp};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  delete w;
}

int mcs_search_for_triangulation_raw_device(mcs_tri_workspace* ws, const uint8_t* d_desc1,
                                            const uint8_t* d_mask1, const int32_t* d_cam1,
                                            const uint8_t* d_has_mp1, const double* d_rays1,
                                            int32_t n1, const uint8_t* d_desc2,
                                            const uint8_t* d_mask2, const int32_t* d_cam2,
                                            const uint8_t* d_has_mp2, const double* d_rays2,
                                            int32_t n2, int32_t ncams, const double* d_E,
                                            int32_t bytes, int32_t th_low, double epi_thresh,
                                            int32_t* d_matches12, int32_t* d_n_matches,
                                            void* stream) {
  int rc = check_bytes(bytes);
  if (rc) return rc;
  if (!ws || !d_n_matches || n1 < 0 || n2 < 0 || ncams <= 0) { set_error("triangulation: bad arguments"); return MCS_ERR_ARG; }
  if (n1 > ws->max_n1 || n2 > ws->max_n2) { set_error("triangulation: n1 / n2 above the workspace capacity"); return MCS_ERR_CAPACITY; }
  if (ncams > 8) { set_error("triangulation: at most 8 cameras (one ordered-pass wave each)"); return MCS_ERR_UNSUPPORTED; }
  if ((d_mask1 != nullptr) != (d_mask2 != nullptr)) { set_error("triangulation: masks for both keyframes or none"); return MCS_ERR_ARG; }
  MCS_HIP_CHECK(hipSetDevice(ws->device));
  hipStream_t st = (hipStream_t)stream;
  if (n1 == 0 || n2 == 0) {
    if (n1 > 0) MCS_HIP_CHECK(hipMemsetAsync(d_matches12, 0xFF, 4 * (size_t)n1, st));   // -1
    MCS_HIP_CHECK(hipMemsetAsync(d_n_matches, 0, 4, st));
    return MCS_OK;
  }
  if (!d_desc1 || !d_desc2 || !d_cam1 || !d_cam2 || !d_has_mp1 || !d_has_mp2 || !d_rays1 ||
      !d_rays2 || !d_E || !d_matches12) {
    set_error("triangulation: null device buffer");
    return MCS_ERR_ARG;
  }
  const hipError_t e = tri_run(ws, d_desc1, d_mask1, d_cam1, d_has_mp1, d_rays1, n1, d_desc2, d_mask2, d_cam2,
                               d_has_mp2, d_rays2, n2, ncams, d_E, bytes, th_low, epi_thresh, d_matches12,
                               d_n_matches, st);
  if (e != hipSuccess) { set_hip_error(e, "triangulation search", __FILE__, __LINE__); return MCS_ERR_HIP; }
  return MCS_OK;
}

int mcs_compute_e_rig(const double* mt1, const double* mt2, const double* mc, int32_t ncams,
                      double* E) {
  if (!mt1 || !mt2 || !mc || !E || ncams <= 0) { set_error("compute_e_rig: bad arguments"); return MCS_ERR_ARG; }
  double T1[16], T2[16], Mc[16], M[16], inv1[16];
  host_cayley2hom(mt1, T1);
  host_cayley2hom(mt2, T2);
  for (int i = 0; i < ncams; i++) {
    host_cayley2hom(mc + 6 * i, Mc);
    host_matmul(T1, Mc, M, 4, 4, 4);
    host_inv_mat(M, inv1);
    for (int j = 0; j < ncams; j++) {
      host_cayley2hom(mc + 6 * j, Mc);
      host_matmul(T2, Mc, M, 4, 4, 4);
      host_compute_e(inv1, M, E + 9 * ((size_t)i * ncams + j));
    }
  }
  return MCS_OK;
}

int mcs_check_dist_epipolar_line(const double* ray1, const double* ray2, const double* E12,
                                 double thresh) {
  if (!ray1 || !ray2 || !E12) { set_error("check_dist_epipolar_line: null argument"); return MCS_ERR_ARG; }
  return epi_check(ray1, ray2, E12, thresh) ? 1 : 0;
}

}  // extern "C"
