// K4 + K6: intensity-centroid orientation (unblurred level) and rotated BRIEF (blurred
// level), one wave per keypoint; all keypoints of a frame run on one XCD so the frame's
// level images stay in that XCD's L2.
//
// Reference: IC_Angle src/mdBRIEFextractorOct.cpp:221-248 (+ fastAtan2),
// compute_ORB / rotatePattern :285-354, keypoint finalisation :959-970,
// :1326-1335.  Compiled with -ffp-contract=off; the float/double ops below are additionally
// spelled with _rn intrinsics so no FMA contraction can change a rounding.
#include "common.hpp"
#include "desc_math.hpp"
#include "extractor_kernels.hpp"
#include <algorithm>

namespace mcs {

__constant__ int c_pattern[2048] = {
#include "pattern_orb64.inc"
};
// IC_Angle's circular r=16 patch (inside <=> |u| <= umax[|v|]) per staged raw-patch dword (33 rows x 9 dwords, byte k of dword (r, cw) is
// u = 4cw + k - 16, v = r - 16): packed u8 weights (u+16 inside, 0 outside) and inside flags,
// so the moments are two v_dot4_u32_u8 per dword:  m10 = sum (u+16) I - 16 S, m01 = sum (v+16) I
// - 16 S, S = sum I (exact integers, identical to the reference's loops).
__constant__ uint32_t c_icw[2][33 * 9];
// pattern as doubles (the rotation runs in double, :290-300)
__constant__ double c_pattern_d[2048];
// the same per test t as packed int8 (x0, y0, x1, y1): k_orient_desc stages it in LDS
__constant__ uint32_t c_pattern_i8[512];

int upload_desc_constants() {
  int umax[kHalfPatch + 1];
  int v, v0, vmax = (int)std::floor(kHalfPatch * std::sqrt(2.f) / 2 + 1);  // ctor :187-202
  int vmin = (int)std::ceil(kHalfPatch * std::sqrt(2.f) / 2);
  const double hp2 = kHalfPatch * kHalfPatch;
  for (v = 0; v <= vmax; ++v) umax[v] = cv_round(std::sqrt(hp2 - v * v));
  for (v = kHalfPatch, v0 = 0; v >= vmin; --v) {
    while (umax[v0] == umax[v0 + 1]) ++v0;
    umax[v] = v0;
    ++v0;
  }
  uint32_t icw[2][33 * 9];
  for (int q = 0; q < 33 * 9; q++) {
    const int r = q / 9, cw = q % 9;
    uint32_t W = 0, M = 0;
    for (int k = 0; k < 4; k++) {
      const int c = 4 * cw + k, uu = c - kHalfPatch, vv = r - kHalfPatch;
      const bool in = c < 33 && std::abs(uu) <= umax[std::abs(vv)];
      W |= (uint32_t)(in ? c : 0) << (8 * k);
      M |= (uint32_t)(in ? 1 : 0) << (8 * k);
    }
    icw[0][q] = W;
    icw[1][q] = M;
  }
  MCS_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_icw), icw, sizeof(icw)));
  static const int pat[2048] = {
#include "pattern_orb64.inc"
  };
  double patd[2048];
  for (int i = 0; i < 2048; i++) patd[i] = (double)pat[i];
  MCS_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_pattern_d), patd, sizeof(patd)));
  uint32_t pat8[512];
  for (int t = 0; t < 512; t++)
    pat8[t] = (uint32_t)(uint8_t)(int8_t)pat[4 * t] | (uint32_t)(uint8_t)(int8_t)pat[4 * t + 1] << 8 |
              (uint32_t)(uint8_t)(int8_t)pat[4 * t + 2] << 16 | (uint32_t)(uint8_t)(int8_t)pat[4 * t + 3] << 24;
  MCS_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_pattern_i8), pat8, sizeof(pat8)));
  return MCS_OK;
}

__device__ __forceinline__ float fast_atan2_dev(float y, float x) {
  // OpenCV fastAtan2
  const float k = (float)(180 / 3.14159265358979323846);
  const float p1 = __fmul_rn(0.9997878412794807f, k), p3 = __fmul_rn(-0.3258083974640975f, k);
  const float p5 = __fmul_rn(0.1555786518463281f, k), p7 = __fmul_rn(-0.04432655554792128f, k);
  const float ax = fabsf(x), ay = fabsf(y);
  const float eps = (float)2.220446049250313080847e-16;
  // both branches of the reference as one: the operands are selected first, so a wave whose
  // lanes disagree runs one division instead of two (the same operations on the same values)
  const bool xs = ax >= ay;
  const float c = __fdiv_rn(xs ? ay : ax, __fadd_rn(xs ? ax : ay, eps));
  const float c2 = __fmul_rn(c, c);
  const float pa = __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1), c);
  float a = xs ? pa : __fsub_rn(90.f, pa);
  if (x < 0) a = __fsub_rn(180.f, a);
  if (y < 0) a = __fsub_rn(360.f, a);
  return a;
}

// signed byte B of v as a float: v_cvt_f32_i32 on an SDWA operand (sign-extended byte select)
template <int B>
__device__ __forceinline__ float sbyte_f32(uint32_t v) {
  float f;
  if constexpr (B == 0)
    asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0" : "=v"(f) : "v"(v));
  else if constexpr (B == 1)
    asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1" : "=v"(f) : "v"(v));
  else if constexpr (B == 2)
    asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2" : "=v"(f) : "v"(v));
  else
    asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3" : "=v"(f) : "v"(v));
  return f;
}

__device__ __forceinline__ int rot_round(double px, double py, double ca, double sa, bool xaxis) {
  // cvRound(x*cos - y*sin) / cvRound(x*sin + y*cos), double, round-half-even
  return xaxis ? (int)rint(__dsub_rn(__dmul_rn(px, ca), __dmul_rn(py, sa)))
               : (int)rint(__dadd_rn(__dmul_rn(px, sa), __dmul_rn(py, ca)));
}
// the same rounding as one add: for |v| < 2^51, v + 1.5 * 2^52 rounds v to an integer in the
// current (nearest-even) mode, and that integer, two's complement, is the low word of the sum
__device__ __forceinline__ int rint_magic(double v) {
  return (int)__double2loint(__dadd_rn(v, 6755399441055744.0));
}
__device__ __forceinline__ int rot_x(double px, double py, double ca, double sa) {
  return rint_magic(__dsub_rn(__dmul_rn(px, ca), __dmul_rn(py, sa)));
}
__device__ __forceinline__ int rot_y(double px, double py, double ca, double sa) {
  return rint_magic(__dadd_rn(__dmul_rn(px, sa), __dmul_rn(py, ca)));
}

// Both patches (raw r=16 for the moments, blurred r=21 for the rotated pattern) are staged
// into LDS with aligned dword loads right after the keypoint is known, so a keypoint costs
// two dependent memory round trips (selection entry, then both patches) instead of one per
// gather batch.
constexpr int kRawW = 9;    // dwords per raw patch row (33 bytes + alignment -> 36)
constexpr int kRawH = 33;
constexpr int kBlrH = 43;

__device__ __forceinline__ uint32_t load_aligned_dword(const uint8_t* g) {
  const uint32_t* ap = dev::align_down4(g);
  return __builtin_amdgcn_alignbyte(ap[1], ap[0], (uint32_t)((uintptr_t)g & 3));
}

// Blurred patch (+-21 around the keypoint) staged in LDS rows of kBlrRow bytes, one 16-byte
// chunk per load.  Default (round 6): the chunks start at the dword below the patch (mis =
// (cx - 21) & 3; global loads need dword alignment only), so 3 chunks cover a row's 43 + 3
// bytes: 48-byte LDS rows, 129 chunks per keypoint (5 loads per lane), 2064 B per keypoint.
// MCS_DESC_ROW64 (the round-2..5 layout): 16-byte aligned chunks (mis = (cx - 21) & 15), 4
// per row, 64-byte rows, 172 chunks (6 loads per lane), 2752 B per keypoint.  A/B in round 6:
// 0.575 (48-byte rows: 20.9 KB per workgroup, 7 per CU) against 0.577 ms (26.4 KB, 6 per CU).
// (Measured slower in round 2: 12 dword loads per 48-byte row, 1.11 vs 0.89 ms.)
#ifdef MCS_DESC_ROW64
constexpr int kBlrRow = 64, kBlrAlign = 15;
#else
constexpr int kBlrRow = 48, kBlrAlign = 3;
#endif
constexpr int kBlrChunks = kBlrRow / 16;   // 16-byte chunks per row

// sum over each 32-lane half of the wave (exact integers, any order): xor 1 and 2 (quad_perm),
// the 8- and 16-lane mirrors (DPP, fused into the adds), then lane ^ 16 (ds_swizzle, bit-mask
// mode); every lane of a half receives its half's sum
__device__ __forceinline__ int half_sum32(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
  v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
  v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false);   // row_half_mirror
  v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false);   // row_mirror
  return v + __builtin_amdgcn_ds_swizzle(v, 0x401F);                // swap 16
}

// IC moments of the raw patch (see c_icw); one half-wave (32 lanes) per keypoint: lane hl
// holds patch dwords q = hl + 32k in registers (each dword is used by one lane only, so the
// raw patch needs no LDS), sums reduced within the half (xor offsets < 32 never cross halves)
__device__ __forceinline__ float ic_angle_regs(const uint32_t (&raw)[10], int hl,
                                               const uint32_t* icw0 = c_icw[0],
                                               const uint32_t* icw1 = c_icw[1]) {
  uint32_t a10 = 0, aS = 0, a01 = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    const int q = hl + 32 * k;
    if (q < kRawH * kRawW) {
      const uint32_t px = raw[k];
      const uint32_t d1 = __builtin_amdgcn_udot4(icw0[q], px, 0u, false);
      const uint32_t d0 = __builtin_amdgcn_udot4(icw1[q], px, 0u, false);
      a10 += d1;
      aS += d0;
      a01 += (uint32_t)(q / kRawW) * d0;
    }
  }
  const int S = half_sum32((int)aS);
  int m10 = half_sum32((int)a10), m01 = half_sum32((int)a01);
  m10 -= kHalfPatch * S;
  m01 -= kHalfPatch * S;
  return fast_atan2_dev((float)m01, (float)m10);
}

// same from a raw patch staged in LDS (dBRIEF path)
__device__ __forceinline__ float ic_angle_lds(const uint32_t* rawp, int hl) {
  uint32_t raw[10];
#pragma unroll
  for (int k = 0; k < 10; k++) {
    const int q = hl + 32 * k;
    raw[k] = (q < kRawH * kRawW) ? rawp[q] : 0u;
  }
  return ic_angle_regs(raw, hl);
}

// Two keypoints per wave, one per 32-lane half: the per-keypoint scalar work (level lookup,
// fastAtan2, double sincos, keypoint record) runs once for both, the 8-32 test words of a
// descriptor come from one 64-bit ballot per 32 tests (low half / high half).
#ifndef MCS_DESC_WAVES
#define MCS_DESC_WAVES 4
#endif
constexpr int kDescWaves = MCS_DESC_WAVES;   // waves per workgroup (the tables are staged once per workgroup)
__global__ __launch_bounds__(64 * kDescWaves) void k_orient_desc(DescArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t s_blr[2 * kDescWaves][kBlrH * kBlrRow];
  // the IC weight tables and the packed pattern, staged once per workgroup: read per lane at
  // lane-dependent indices, from constant memory they were L2 round trips inside the compute
  // (one per test round) instead of LDS reads
  __shared__ uint32_t s_icw[2][kRawH * kRawW];
  __shared__ uint32_t s_pat[512];
  typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
  // wave index as a scalar: the pair, its level and counts are wave-uniform
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int half = lane >> 5, hl = lane & 31, slot = 2 * wv + half;
  int f, item;
  const int pairs = (a.sel_per_frame + 1) / 2;
  if (!xcd_frame_map(blockIdx.x, a.nframes, (pairs + kDescWaves - 1) / kDescWaves, &f, &item)) return;
  // The tables are staged after this wave's keypoint and patch loads are issued, and one
  // barrier covers both: a wave waits on two dependent memory round trips (selection entry, then
  // the patches, with the table loads beside them) instead of three.  A wave without keypoints
  // stages its share and meets the barrier on its own (wave-uniform branch: every wave reaches
  // exactly one s_barrier).
  static_assert(kDescWaves == 4, "table staging assumes 256 threads");
  const int tid = threadIdx.x;
  uint32_t tw[6];   // this thread's table words: icw[0][tid (+256)], icw[1][tid (+256)], pat[tid (+256)]
  auto load_tables = [&]() {
    const int t2 = min(tid + 256, kRawH * kRawW - 1);
    tw[0] = c_icw[0][tid]; tw[1] = c_icw[0][t2];
    tw[2] = c_icw[1][tid]; tw[3] = c_icw[1][t2];
    tw[4] = c_pattern_i8[tid]; tw[5] = c_pattern_i8[tid + 256];
  };
  auto store_tables = [&]() {
    s_icw[0][tid] = tw[0];
    s_icw[1][tid] = tw[2];
    if (tid + 256 < kRawH * kRawW) {
      s_icw[0][tid + 256] = tw[1];
      s_icw[1][tid + 256] = tw[3];
    }
    s_pat[tid] = tw[4];
    s_pat[tid + 256] = tw[5];
  };
  auto stage_tables = [&]() {
    load_tables();
    store_tables();
  };
  // even j0: both keypoints on one level (every level's sel_off is even, build_plan)
  const int j0 = 2 * (item * kDescWaves + wv);
  if (j0 >= a.sel_per_frame) {
    stage_tables();
    __syncthreads();
    return;
  }
  int l = 0;
  while (l + 1 < a.nlevels && j0 >= a.lv[l + 1].sel_off) l++;
  const LevelPlan& L = a.lv[l];
  const int32_t* scount = a.sel_count + (int64_t)f * a.nlevels;
  const int cnt = scount[l];
  const int i0 = j0 - L.sel_off;
  if (i0 >= cnt) {                             // both halves past the level's selection
    stage_tables();
    __syncthreads();
    return;
  }
  const bool valid = i0 + half < cnt;          // else: recompute keypoint i0, write nothing
  int outIdx = i0 + (valid ? half : 0);
  for (int t = 0; t < l; t++) outIdx += scount[t];
  const uint32_t pk = a.sel[(int64_t)f * a.sel_fstride + j0 + (valid ? half : 0)];
  const int cx = (int)(pk & 0xFFF) + kMinBorder, cy = (int)((pk >> 12) & 0xFFF) + kMinBorder;
  const int score = (int)(pk >> 24);
  const int pitch = L.pitch, bp = L.bpitch;
  // frame / level bases are wave-uniform (both keypoints of a wave share frame and level):
  // SGPR bases + 32-bit lane offsets, no 64-bit address arithmetic per load
  const uint8_t* const img = dev::uniform_ptr(
      (l == 0) ? a.img0 + (int64_t)f * a.img0_fstride : a.pyr + (int64_t)f * a.pyr_fstride + L.pyr_off);
  const uint8_t* const blr = dev::uniform_ptr(a.blur + (int64_t)f * a.blur_fstride + L.img_off);
  // ---- raw patch: dword q = hl + 32k (row q / 9, column q % 9) of the 33 x 9 dwords per
  // lane, consecutive lanes on consecutive dwords (coalesced), kept in registers; blurred patch
  // into LDS (independent loads, issued together), 32-bit offsets from the uniform bases
  const int mis = (cx - 21) & kBlrAlign;
  uint32_t raw[10];
  uint32_t rq[10];
  {
    // dword q = hl + 32k of the patch: row r = q / 9 = (57 q) >> 9 (exact for q < 320), byte
    // offset r (pitch - 36) + 4 q + origin = r (pitch - 36) + (origin & ~3) + 4 hl + 128 k +
    // (origin & 3): one 24-bit multiply-add per dword (128 k is the load's immediate offset), and
    // the misalignment origin & 3 is the wave's (every row shares it: pitches are multiples of 4)
    const uint32_t org = (uint32_t)((cy - kHalfPatch) * pitch + (cx - kHalfPatch));
    const uint32_t al = org & 3u;
    const uint32_t ob4 = (org & ~3u) + 4u * (uint32_t)hl;
    const uint32_t pm = (uint32_t)(pitch - 4 * kRawW);
    const uint32_t h57 = __umul24((uint32_t)hl, 57u);
#pragma unroll
    // every load is unconditional (lanes past the patch re-read its last dword, unused): a
    // register loaded on one path only would be merged after a wait for all loads in flight
    for (int k = 0; k < 10; k++) {
      uint32_t r, o;
      if (k < 9) {            // q <= 31 + 256 < 297
        r = (h57 + 1824u * k) >> 9;
        o = __umul24(r, pm) + ob4 + 128u * k;
      } else {                // q = min(hl + 288, 296)
        const uint32_t hc = min((uint32_t)hl, 8u);
        r = (__umul24(hc, 57u) + 1824u * k) >> 9;
        o = __umul24(r, pm) + (org & ~3u) + 4u * (hc + 32u * k);
      }
      rq[k] = r;
      const uint32_t* ap = reinterpret_cast<const uint32_t*>(img + o);
      raw[k] = __builtin_amdgcn_alignbyte(ap[1], ap[0], al);
    }
    // blurred patch: chunk q = hl + 32k is row q / kBlrChunks, chunk q % kBlrChunks, at byte
    // q (16 rows-worth) of the wave's LDS patch (rows of kBlrChunks chunks: LDS offset 16 q) and
    // at r (bp - kBlrRow) + 16 q + origin in the level (r = q / 3 = (171 q) >> 9, exact for
    // q < 512)
    constexpr int NQ = kBlrH * kBlrChunks;              // 129 (172)
    constexpr int NK = NQ / 32;                         // full loads per lane: 4 (5)
    const uint32_t bo0 = (uint32_t)((cy - 21) * bp + (cx - 21 - mis));
    const uint32_t bpm = (uint32_t)(bp - kBlrRow);
    const uint32_t bl = bo0 + 16u * (uint32_t)hl;
    auto chunk_row = [&](uint32_t q) -> uint32_t {
      return kBlrChunks == 4 ? (q >> 2) : ((q * 171u) >> 9);
    };
    const uint32_t h171 = __umul24((uint32_t)hl, 171u);
    u32x4a bv[NK];
#pragma unroll
    for (int k = 0; k < NK; k++) {
      const uint32_t r = kBlrChunks == 4 ? (((uint32_t)hl >> 2) + 8u * k) : ((h171 + 5472u * k) >> 9);
      bv[k] = *reinterpret_cast<const u32x4a*>(blr + (__umul24(r, bpm) + bl + 512u * k));
    }
    // the last NQ - 32 NK chunks; lanes past them re-read the last chunk (unused)
    const uint32_t qt = min((uint32_t)hl + 32u * NK, (uint32_t)NQ - 1u);
    const u32x4a bt = *reinterpret_cast<const u32x4a*>(blr + (__umul24(chunk_row(qt), bpm) + bo0 + 16u * qt));
    load_tables();   // beside the patch loads
    uint8_t* const sb = &s_blr[slot][16 * hl];
#pragma unroll
    for (int k = 0; k < NK; k++) *reinterpret_cast<u32x4a*>(sb + 512 * k) = bv[k];
    if (hl < NQ - 32 * NK) *reinterpret_cast<u32x4a*>(sb + 512 * NK) = bt;
  }
  store_tables();
  __syncthreads();
  // ---- IC_Angle: integer moments over the circular r=16 patch (see c_icw; exact integer
  // sums): m10 = sum (u+16) I - 16 S, m01 = sum (v+16) I - 16 S with v + 16 = the row
  float angle;
  {
    uint32_t a10 = 0, aS = 0, a01 = 0;
#pragma unroll
    for (int k = 0; k < 10; k++) {
      const int q = hl + 32 * k;
      if (q < kRawH * kRawW) {
        a10 = __builtin_amdgcn_udot4(s_icw[0][q], raw[k], a10, false);
        const uint32_t d0 = __builtin_amdgcn_udot4(s_icw[1][q], raw[k], 0u, false);
        aS += d0;
        a01 += __umul24(rq[k], d0);   // row < 33, d0 <= 1020
      }
    }
    int S = (int)aS, m10 = (int)a10, m01 = (int)a01;
    S = half_sum32(S);
    m10 = half_sum32(m10);
    m01 = half_sum32(m01);
    m10 -= kHalfPatch * S;
    m01 -= kHalfPatch * S;
    angle = fast_atan2_dev((float)m01, (float)m10);
  }
  // ---- rotated BRIEF on the blurred patch
  const float DEG2RADf = (float)3.14159265358979323846 / 180.f;
  const float thf = __fmul_rn(angle, DEG2RADf);  // the reference's angle, (double)(angle * DEG2RADf)
  // cos / sin: in float (desc_math.hpp, |error| <= kSinCosErr) for the float rotation; in double
  // only for a wave whose rounds reach the near-half band (after the rounds, see `redo`)
  float saf, caf;
  sincos_f32(thf, saf, caf);
  const int nw = a.desc_size / 4;               // 32-test words: 4 / 8 / 16
  const uint8_t* bc = &s_blr[slot][21 * kBlrRow + 21 + mis];
  uint32_t w = 0u;   // lane hl keeps test word hl of its half's descriptor
  // The rotated coordinates are cvRound of double products (rot_x / rot_y).  They are first
  // taken in float, with cos / sin in float (sincos_f32): the float value is within kNearHalf of
  // the double one (desc_math.hpp), so both round alike unless the float value lies within
  // kNearHalf of a half-integer.  A round where any lane of the wave is that close is marked
  // and taken again after the loop in the double form for every lane (rare; the double cos /
  // sin are formed only then), so every test word is the double form's, bit for bit.
  // Round 6: the double sincos (~150 VALU per wave) left the common path, the pattern bytes
  // convert to float with SDWA operands, both points' x and y rotate as packed pairs, the LDS
  // addresses come out of one packed fma and the near-half test is branch-free: 36 -> ~25 VALU
  // per round; the double form's constants no longer occupy registers inside the loop.
  // (Measured slower in round 4/5: software-pipelining several pairs per wave, 0.71 -> 0.94-1.13
  // ms per step; OCML sincosf in place of the double sincos, 0.72 -> 0.77 ms.)
  // LDS byte address of the patch centre as a float (exact: < 2^24), so a sample's address is
  // one fma + one conversion: (ry * row + rx) + centre, all small integers
  const uint32_t bc_lds = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)bc;
  const float bcf = (float)bc_lds;
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  uint32_t redo = 0u;   // wave-uniform: rounds to take again in double
  // (Measured slower in round 6: the pattern words from global memory, a pair of rounds ahead,
  // without s_pat: 18.9 KB and 60 VGPRs allow 8 waves per SIMD, but 0.575 -> 0.61 ms.)
  auto patw = [&](int r) -> uint32_t { return s_pat[r * 32 + hl]; };
  auto round = [&](const int r, const uint32_t pw) {
    // the four signed pattern bytes straight to float (v_cvt_f32_i32 with a sign-extended byte
    // operand: one instruction each instead of a bit-field extract and a conversion)
    const float fx0 = sbyte_f32<0>(pw), fy0 = sbyte_f32<1>(pw), fx1 = sbyte_f32<2>(pw), fy1 = sbyte_f32<3>(pw);
    // both points' x and both points' y as packed pairs: X = (xa, xb) = fma((x0, x1), c,
    // (y0, y1) * -s), Y = (ya, yb) = fma((x0, x1), s, (y0, y1) * c) -- per lane the same
    // roundings as xa = fma(x0, c, -(y0 s)), ya = fma(x0, s, y0 c), in four packed instructions
    const f32x2 px = {fx0, fx1}, py = {fy0, fy1};
    const f32x2 X = __builtin_elementwise_fma(px, (f32x2){caf, caf}, py * (f32x2){-saf, -saf});
    const f32x2 Y = __builtin_elementwise_fma(px, (f32x2){saf, saf}, py * (f32x2){caf, caf});
    const f32x2 RX = {__builtin_rintf(X.x), __builtin_rintf(X.y)};
    const f32x2 RY = {__builtin_rintf(Y.x), __builtin_rintf(Y.y)};
    // LDS addresses (ry * row + rx) + centre of both points, packed, then converted
    const f32x2 A = __builtin_elementwise_fma(RY, (f32x2){(float)kBlrRow, (float)kBlrRow}, RX + (f32x2){bcf, bcf});
    // the largest distance of the four values from their rounding, branch-free
    const f32x2 DX = X - RX, DY = Y - RY;
    const float dm = fmaxf(fmaxf(fabsf(DX.x), fabsf(DX.y)), fmaxf(fabsf(DY.x), fabsf(DY.y)));
    if (__ballot(dm > 0.5f - kNearHalf)) redo |= 1u << r;
    const auto* p0 = (const __attribute__((address_space(3))) uint8_t*)(uintptr_t)(uint32_t)A.x;
    const auto* p1 = (const __attribute__((address_space(3))) uint8_t*)(uintptr_t)(uint32_t)A.y;
    const uint64_t b = __ballot(*p0 < *p1);
    if (hl == r) w = half ? (uint32_t)(b >> 32) : (uint32_t)b;
  };
  // nw is 4, 8 or 16: rounds in pairs (the convergent ballots keep the compiler from unrolling a
  // loop of unknown count), so the next round's pattern read is in flight
  for (int r = 0; r < nw; r += 2) {
    round(r, patw(r));
    round(r + 1, patw(r + 1));
  }
  if (redo) {
    double sa, ca;
    sincos((double)thf, &sa, &ca);
    do {
      const int r = __builtin_ctz(redo);
      redo &= redo - 1u;
      const uint32_t pw = patw(r);
      const double px0 = (double)sbyte_f32<0>(pw), py0 = (double)sbyte_f32<1>(pw);
      const double px1 = (double)sbyte_f32<2>(pw), py1 = (double)sbyte_f32<3>(pw);
      const uint32_t a0 = bc_lds + (uint32_t)(rot_y(px0, py0, ca, sa) * kBlrRow + rot_x(px0, py0, ca, sa));
      const uint32_t a1 = bc_lds + (uint32_t)(rot_y(px1, py1, ca, sa) * kBlrRow + rot_x(px1, py1, ca, sa));
      const auto* p0 = (const __attribute__((address_space(3))) uint8_t*)(uintptr_t)a0;
      const auto* p1 = (const __attribute__((address_space(3))) uint8_t*)(uintptr_t)a1;
      const uint64_t b = __ballot(*p0 < *p1);
      if (hl == r) w = half ? (uint32_t)(b >> 32) : (uint32_t)b;
    } while (redo);
  }
  if (valid && hl < nw)
    reinterpret_cast<uint32_t*>(a.desc + ((int64_t)f * a.cap + outIdx) * a.desc_size)[hl] = w;
  if (valid && hl == 0) {
    mcs_keypoint kp;
    kp.x = (float)cx; kp.y = (float)cy;
    if (l != 0) { kp.x = __fmul_rn((float)cx, L.scale); kp.y = __fmul_rn((float)cy, L.scale); }
    kp.size = (float)L.patch_size_scaled;
    kp.angle = angle;
    kp.response = (float)score;
    kp.octave = l;
    kp.class_id = -1;
    a.kps[(int64_t)f * a.cap + outIdx] = kp;
  }
}

// ===========================================================================
// dBRIEF / mdBRIEF (src/mdBRIEFextractorOct.cpp:250-283 rotateAndDistortPattern, :356-408
// compute_dBRIEF, :410-554 compute_mdBRIEF; keypoint undistortion :1304-1316) on the
// Scaramuzza model (src/cam_model_omni.cpp:49-163).  One wave per keypoint: every lane
// distorts npoints/64 pattern points in double precision (ImgToWorld / WorldToImg with the
// reference's operation order, no FMA), the pattern mean is summed by one lane in point
// order (the reference's sequential sum), and the tests sample the padded level buffer the
// reference reads (blurred ROI, raw reflect-101 border of 25 px, linear wrap beyond).
// ===========================================================================
__device__ __forceinline__ double horner_d(const double* c, int s, double x) {
  double r = 0.0;
  for (int i = s - 1; i >= 0; i--) r = __dadd_rn(__dmul_rn(r, x), c[i]);
  return r;
}

__device__ void img_to_world_d(const mcs_cam_model& m, double u, double v, double& x, double& y,
                               double& z) {
  const double invAffine = __dsub_rn(m.c, __dmul_rn(m.d, m.e));
  const double u_t = __dsub_rn(u, m.u0), v_t = __dsub_rn(v, m.v0);
  x = __ddiv_rn(__dsub_rn(u_t, __dmul_rn(m.d, v_t)), invAffine);
  y = __ddiv_rn(__dadd_rn(__dmul_rn(-m.e, u_t), __dmul_rn(m.c, v_t)), invAffine);
  const double X2 = __dmul_rn(x, x), Y2 = __dmul_rn(y, y);
  z = -horner_d(m.p, m.p_deg, __dsqrt_rn(__dadd_rn(X2, Y2)));
  const double norm = __dsqrt_rn(__dadd_rn(__dadd_rn(X2, Y2), __dmul_rn(z, z)));
  x = __ddiv_rn(x, norm); y = __ddiv_rn(y, norm); z = __ddiv_rn(z, norm);
}

__device__ void world_to_img_d(const mcs_cam_model& m, double x, double y, double z, double& u,
                               double& v) {
  double norm = __dsqrt_rn(__dadd_rn(__dmul_rn(x, x), __dmul_rn(y, y)));
  if (norm == 0.0) norm = 1e-14;
  const double theta = atan(__ddiv_rn(-z, norm));
  const double rho = horner_d(m.invp, m.invp_deg, theta);
  const double uu = __dmul_rn(__ddiv_rn(x, norm), rho), vv = __dmul_rn(__ddiv_rn(y, norm), rho);
  u = __dadd_rn(__dadd_rn(__dmul_rn(uu, m.c), __dmul_rn(vv, m.d)), m.u0);
  v = __dadd_rn(__dadd_rn(__dmul_rn(uu, m.e), vv), m.v0);
}

__device__ __forceinline__ int refl101_d(int p, int n) {
  if (n == 1) return 0;
  while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
  return p;
}

// image.ptr(y)[x] of the reference's padded level buffer (see oracle padded_at)
__device__ __forceinline__ int padded_at_dev(const uint8_t* blr, int bp, const uint8_t* raw, int rp,
                                             int w, int h, int y, int x) {
  if ((unsigned)y < (unsigned)h && (unsigned)x < (unsigned)w) return blr[(int64_t)y * bp + x];
  int py = y, px = x;
  if (x < -kEdgeThreshold || x >= w + kEdgeThreshold || y < -kEdgeThreshold ||
      y >= h + kEdgeThreshold) {
    const int64_t W2 = w + 2 * kEdgeThreshold, H2 = h + 2 * kEdgeThreshold;
    int64_t L = (int64_t)(y + kEdgeThreshold) * W2 + (x + kEdgeThreshold);
    L = L < 0 ? 0 : (L >= W2 * H2 ? W2 * H2 - 1 : L);
    py = (int)(L / W2) - kEdgeThreshold;
    px = (int)(L - (int64_t)(py + kEdgeThreshold) * W2) - kEdgeThreshold;
    if ((unsigned)py < (unsigned)h && (unsigned)px < (unsigned)w) return blr[(int64_t)py * bp + px];
  }
  return raw[(int64_t)refl101_d(py, h) * rp + refl101_d(px, w)];
}

template <bool LEARN>
__global__ __launch_bounds__(256) void k_dbrief(DescArgs a, int wave_lds) {
  extern __shared__ __attribute__((aligned(16))) uint8_t dlds[];
  const int wpb = blockDim.x >> 6;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int npts = 16 * a.desc_size;
  double* xs = reinterpret_cast<double*>(dlds + (size_t)wv * wave_lds);
  double* ys = xs + npts;
  int32_t* offs = reinterpret_cast<int32_t*>(ys + npts);   // [LEARN ? 3 : 1][npts]
  int f, item;
  const int chunks = (a.sel_per_frame + wpb - 1) / wpb;
  if (!xcd_frame_map(blockIdx.x, a.nframes, chunks, &f, &item)) return;
  const int j = item * wpb + wv;
  if (j >= a.sel_per_frame) return;
  int l = 0;
  while (l + 1 < a.nlevels && j >= a.lv[l + 1].sel_off) l++;
  const LevelPlan& L = a.lv[l];
  const int i = j - L.sel_off;
  const int32_t* scount = a.sel_count + (int64_t)f * a.nlevels;
  if (i >= scount[l]) return;
  int outIdx = i;
  for (int t = 0; t < l; t++) outIdx += scount[t];
  const uint32_t pk = a.sel[(int64_t)f * a.sel_fstride + j];
  const int cx = (int)(pk & 0xFFF) + kMinBorder, cy = (int)((pk >> 12) & 0xFFF) + kMinBorder;
  const int score = (int)(pk >> 24);
  const int pitch = L.pitch, bp = L.bpitch;
  const uint8_t* img = (l == 0) ? a.img0 + (int64_t)f * a.img0_fstride
                                : a.pyr + (int64_t)f * a.pyr_fstride + L.pyr_off;
  const uint8_t* blr = a.blur + (int64_t)f * a.blur_fstride + L.img_off;
  // ---- IC_Angle on the raw patch, staged in the (not yet used) xs area
  {
    uint32_t* rawp = reinterpret_cast<uint32_t*>(xs);
    const uint8_t* r0 = img + (int64_t)(cy - kHalfPatch) * pitch + (cx - kHalfPatch);
    for (int q = lane; q < kRawH * kRawW; q += 64) {
      const int r = q / kRawW, c = q - r * kRawW;
      rawp[q] = load_aligned_dword(r0 + (int64_t)r * pitch + 4 * c);
    }
  }
  dev::wave_sync();
  const float angle = ic_angle_lds(reinterpret_cast<const uint32_t*>(xs), lane & 31);
  dev::wave_sync();
  // ---- undistorted keypoint (zero unless do_dBrief, :1304-1316)
  const mcs_cam_model& m = a.cams[a.cam_index ? a.cam_index[f] : 0];
  double ux = 0.0, uy = 0.0;
  if (a.do_dbrief) {
    const float fx = (l != 0) ? __fmul_rn((float)cx, L.scale) : (float)cx;
    const float fy = (l != 0) ? __fmul_rn((float)cy, L.scale) : (float)cy;
    double x, y, z;
    img_to_world_d(m, (double)fx, (double)fy, x, y, z);
    ux = __dmul_rn(__ddiv_rn(-x, z), m.p[0]);
    uy = __dmul_rn(__ddiv_rn(-y, z), m.p[0]);
  }
  // ---- rotateAndDistortPattern
  auto build = [&](double ang, int32_t* out) {
    double ax, ay;
    sincos(ang, &ay, &ax);
    for (int p = lane; p < npts; p += 64) {
      const double px = c_pattern_d[2 * p], py = c_pattern_d[2 * p + 1];
      const double xr = __dadd_rn(__dsub_rn(__dmul_rn(px, ax), __dmul_rn(py, ay)), ux);
      const double yr = __dadd_rn(__dadd_rn(__dmul_rn(px, ay), __dmul_rn(py, ax)), uy);
      double u, v;
      world_to_img_d(m, xr, yr, -m.p[0], u, v);
      xs[p] = u;
      ys[p] = v;
    }
    dev::wave_sync();
    double sx = 0.0, sy = 0.0;
    if (lane == 0) {   // the reference's running sum, in point order
      for (int p = 0; p < npts; p++) { sx = __dadd_rn(sx, xs[p]); sy = __dadd_rn(sy, ys[p]); }
    }
    sx = __shfl(sx, 0);
    sy = __shfl(sy, 0);
    const double mx = __ddiv_rn(sx, (double)npts), my = __ddiv_rn(sy, (double)npts);
    for (int p = lane; p < npts; p += 64) {
      const int ox = (int)rint(__dsub_rn(xs[p], mx)), oy = (int)rint(__dsub_rn(ys[p], my));
      out[p] = (ox & 0xFFFF) | (oy << 16);
    }
    dev::wave_sync();
  };
  if (LEARN) {
    const float RHOf = 180.0f / 3.1415926535897932384626f;
    const double RHOd = 180.0 / 3.1415926535897932384626433832795028841971693993;
    const double rot = 20.0 / RHOd;
    const double ang = (double)__fdiv_rn(angle, RHOf);
    build(ang, offs);
    build(__dadd_rn(ang, rot), offs + npts);
    build(__dsub_rn(ang, rot), offs + 2 * npts);
  } else {
    const float DEG2RADf = (float)3.14159265358979323846 / 180.f;
    build((double)__fmul_rn(angle, DEG2RADf), offs);
  }
  // ---- tests
  auto sample = [&](int32_t o) {
    const int ox = (int)(int16_t)(o & 0xFFFF), oy = o >> 16;
    return padded_at_dev(blr, bp, img, pitch, L.w, L.h, cy + oy, cx + ox);
  };
  const int nwords = a.desc_size / 8;
  uint64_t words[8], mwords[8];
#pragma unroll
  for (int r = 0; r < 8; r++) {
    words[r] = mwords[r] = 0;
    if (r < nwords) {
      const int t = r * 64 + lane;
      const int bit = sample(offs[2 * t]) < sample(offs[2 * t + 1]);
      words[r] = __ballot(bit);
      if (LEARN) {
        const int s1 = (sample(offs[npts + 2 * t]) < sample(offs[npts + 2 * t + 1])) ^ bit;
        const int s2 = (sample(offs[2 * npts + 2 * t]) < sample(offs[2 * npts + 2 * t + 1])) ^ bit;
        mwords[r] = __ballot(s1 + s2 == 0);
      }
    }
  }
  uint8_t* dptr = a.desc + ((int64_t)f * a.cap + outIdx) * a.desc_size;
  if (lane < nwords) {
    uint64_t w = words[0], mw = mwords[0];
#pragma unroll
    for (int r = 1; r < 8; r++)
      if (lane == r) { w = words[r]; mw = mwords[r]; }
    reinterpret_cast<uint64_t*>(dptr)[lane] = w;
    if (a.desc_masks)
      reinterpret_cast<uint64_t*>(a.desc_masks + ((int64_t)f * a.cap + outIdx) * a.desc_size)[lane] = mw;
  }
  if (lane == 0) {
    mcs_keypoint kp;
    kp.x = (float)cx; kp.y = (float)cy;
    if (l != 0) { kp.x = __fmul_rn((float)cx, L.scale); kp.y = __fmul_rn((float)cy, L.scale); }
    kp.size = (float)L.patch_size_scaled;
    kp.angle = angle;
    kp.response = (float)score;
    kp.octave = l;
    kp.class_id = -1;
    a.kps[(int64_t)f * a.cap + outIdx] = kp;
  }
}

void launch_orient_desc(const DescArgs& a, hipStream_t st) {
  if (a.mode == 0) {
    const unsigned g = xcd_grid(a.nframes, ((a.sel_per_frame + 1) / 2 + kDescWaves - 1) / kDescWaves);
    hipLaunchKernelGGL(k_orient_desc, dim3(g), dim3(64 * kDescWaves), 0, st, a);
    return;
  }
  const int npts = 16 * a.desc_size;
  const int npat = a.mode == 2 ? 3 : 1;
  const int wave_lds = (npts * 16 + npat * npts * 4 + 15) & ~15;
  const int wpb = std::max(1, std::min(4, 65536 / wave_lds));
  const unsigned g = xcd_grid(a.nframes, (a.sel_per_frame + wpb - 1) / wpb);
  if (a.mode == 2)
    hipLaunchKernelGGL(k_dbrief<true>, dim3(g), dim3(64 * wpb), (size_t)wpb * wave_lds, st, a, wave_lds);
  else
    hipLaunchKernelGGL(k_dbrief<false>, dim3(g), dim3(64 * wpb), (size_t)wpb * wave_lds, st, a, wave_lds);
}

}  // namespace mcs
