// K1 + K5 fused: one pyramid level = cv::resize(INTER_LINEAR) of level l-1 and
// the 5x5 normalised box blur of level l, in one row stream per wave.
//
// Reference: ComputePyramid src/mdBRIEFextractorOct.cpp:1158-1201 (resize chain) and the
// in-place boxFilter of operator() :1298-1301.  The reference pads every level by 25 px of
// BORDER_REFLECT_101 (:1185-1197) only so that later stages may read outside it; nothing
// downstream reads outside a level except the blur, which reflects explicitly here.
#include "common.hpp"
#include "extractor_kernels.hpp"
#include "pyr_math.hpp"
#include <type_traits>

namespace mcs {

// Row-streaming pyramid level: one wave owns a strip of `core` (<= 244) output columns and a
// segment of `seg_rows` rows.  Lane L holds 4 consecutive pixels [xs-4+4L, xs+4L); lane 0 and
// the lane after the core are the +-2 px halo of the blur.  A pixel outside the level holds
// the value of its BORDER_REFLECT_101 mirror (computed from the mirror's own coordinates),
// so the horizontal 5-sum needs no border cases.  Rows are produced top to bottom with a
// 2-row halo above and below the segment:
//   RESIZE: every source row the segment needs is streamed once per wave with aligned dword
//           loads (kPF rows in flight), staged in wave-private LDS, and horizontally resized
//           per lane (coefficients in registers, v_dot2_u32_u16); an output row combines the
//           last two;
//   level 0: the input row is streamed the same way.
// Each raw row is written out (RESIZE); its horizontal 5-sums (lane neighbours by DPP)
// enter a 5-row register window; once row r+2 exists the blurred row r is written.
// No workgroup barriers: every wave works alone.  Everything derived from the work unit is
// wave-uniform and kept scalar (readfirstlane of the wave index and of table reads).
constexpr int kStageDW = 192;    // staged source row (dwords), scale <= 2.2
#ifndef MCS_PYR_KPF
#define MCS_PYR_KPF 6
#endif
// source rows in flight per wave: 6 (end of round 6: pyramid 0.632-0.633 -> 0.622-0.626 ms per
// step over three A/B runs; 2 and 8 measured 0.671 and 0.80 ms)
constexpr int kPF = MCS_PYR_KPF;

typedef unsigned short us2 __attribute__((ext_vector_type(2)));

// NDW = staged dwords per lane per source row: 1 (level 0), 2 (scale <= 1.5), 3 (scale <= 2.2)
#ifndef MCS_PYR_OCC
#define MCS_PYR_OCC 1
#endif
template <bool RESIZE, int NDW>
__global__ __launch_bounds__(256, MCS_PYR_OCC) void k_pyr_rows(PyrArgs a) {
  __shared__ uint32_t lds_stage[4][kStageDW];
  // wave index as a scalar: everything derived from the work unit is wave-uniform, and the
  // compiler must know it (SGPRs, scalar branches) or it keeps all of it in VGPRs
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  uint32_t* const stage = lds_stage[wv];
  const uint8_t* const stb = reinterpret_cast<const uint8_t*>(stage);
  int f, item;
  const int units = a.tiles_x * a.tiles_y;
  if (!xcd_frame_map(blockIdx.x, a.nframes, (units + 3) / 4, &f, &item)) return;
  const int unit = item * 4 + wv;
  if (unit >= units) return;
  const int strip = unit % a.tiles_x, seg = unit / a.tiles_x;
  const int dw = a.dw, dh = a.dh, core = a.core;
  const int xs = strip * core;
  const int xcore1 = min(xs + core, dw);           // core px [xs, xcore1)
  const int seg0 = seg * a.seg_rows, seg1 = min(dh, seg0 + a.seg_rows);
  const int r_begin = max(0, seg0 - 2), r_end = min(dh, seg1 + 2);
  const int xb = xs - 4 + 4 * lane;                // lane's first pixel
  const bool core_lane = xb >= xs && xb < xcore1;
  const uint8_t* S = a.src + (int64_t)f * a.src_fstride;
  const int sh = RESIZE ? a.sh : dh;

  // staged source columns [c_lo, c_hi]: the mirrors of the strip's pixels stay inside
  // [xs-4, xs+core+4) clamped to the level; per pixel: the (mirrored) column it reads
  int c_lo, c_hi;
  int sx[4];
  uint32_t aa[4];     // alpha0 | alpha1 << 16 (v_dot2_u32_u16 operand)
  int simd = 0;       // bit k: pixel k uses the SSE2 vertical form
  if (RESIZE) {
    c_lo = __builtin_amdgcn_readfirstlane(a.xofs[max(xs - 4, 0)]);
    c_hi = min(__builtin_amdgcn_readfirstlane(a.xofs[min(xs + core + 3, dw - 1)]) + 1, a.sw - 1);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int p = min(max(refl101(xb + k, dw), 0), dw - 1);
      // the right neighbour is read at sx + 1 even where resize clamps it to sx (the last
      // source column): alpha1 is 0 there, and sx + 1 stays inside the staged LDS row
      sx[k] = min(max(a.xofs[p] - c_lo, 0), c_hi - c_lo);
      // alpha << 4 (alpha <= 2048, so <= 32768 still fits u16): the dot product is s << 4
      aa[k] = ((uint32_t)(uint16_t)a.alpha[2 * p] | ((uint32_t)(uint16_t)a.alpha[2 * p + 1] << 16)) << 4;
      simd |= (p < a.simd_end) << k;
    }
  } else {
    c_lo = max(xs - 4, 0);
    c_hi = min(xs + core + 3, dw - 1);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      sx[k] = min(max(min(max(refl101(xb + k, dw), 0), dw - 1) - c_lo, 0), c_hi - c_lo);
      aa[k] = 0;
    }
  }
  const int nbytes0 = c_hi - c_lo + 1;

  // ---- streamed source rows: aligned dwords covering [c_lo, c_hi]
  auto row_base = [&](int sr) -> const uint8_t* { return S + (int64_t)sr * a.spitch; };
  // Every dword is loaded whole, also the last one of the last row of a frame buffer: an
  // aligned dword that holds a valid byte lies in that byte's page, so it cannot fault, and
  // its bytes past the row end are never consumed.  No conditional tail: a register written
  // on two paths would have to be merged, and that merge waits for every load in flight.
  auto load_row = [&](int sr, uint32_t (&v)[NDW]) {
    const uint8_t* st = row_base(sr) + c_lo;
    const uint32_t* ap = dev::align_down4(st);
    const int ndw = ((int)((uintptr_t)st & 3) + nbytes0 + 3) >> 2;
#pragma unroll
    for (int m = 0; m < NDW; m++) v[m] = ap[min(lane + 64 * m, ndw - 1)];
  };
  // stage a row and read this lane's 4 (mirrored) source bytes / resized values
  auto stage_and_gather = [&](int sr, const uint32_t (&v)[NDW], int (&h)[4]) {
    const int shft = (int)((uintptr_t)(row_base(sr) + c_lo) & 3);
#pragma unroll
    for (int m = 0; m < NDW; m++) stage[lane + 64 * m] = v[m];
    dev::wave_sync();
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (RESIZE) {
        const uint32_t pp = (uint32_t)stb[shft + sx[k]] | ((uint32_t)stb[shft + sx[k] + 1] << 16);
        h[k] = (int)__builtin_amdgcn_udot2(__builtin_bit_cast(us2, pp), __builtin_bit_cast(us2, aa[k]), 0u, false);
      } else {
        h[k] = stb[shft + sx[k]];
      }
    }
    dev::wave_sync();
  };

  // ---- raw row -> store, horizontal 5-sums, 5-row window, blurred rows out
  uint8_t* const dstf = RESIZE ? a.dst + (int64_t)f * a.dst_fstride : nullptr;
  uint8_t* const blrf = a.blur + (int64_t)f * a.blur_fstride;
  uint32_t win[5][2];   // packed u16 5-sums of raw rows r-4..r (win[4] = newest)
#pragma unroll
  for (int i = 0; i < 5; i++) win[i][0] = win[i][1] = 0;
  // blurred row y from the window sums: (2s + 25) / 50 = (s * 671090 + 8388625) >> 24 for
  // s <= 25 * 255 (exhaustively checked, tests/test_oracle_cpu.py), the quotient is the top
  // byte, and v_perm packs the four top bytes
  auto store_blur = [&](int y, uint32_t s01, uint32_t s23) {
    if (core_lane) {
      const uint32_t q0 = (s01 & 0xFFFFu) * 671090u + 8388625u, q1 = (s01 >> 16) * 671090u + 8388625u;
      const uint32_t q2 = (s23 & 0xFFFFu) * 671090u + 8388625u, q3 = (s23 >> 16) * 671090u + 8388625u;
      const uint32_t o = __builtin_amdgcn_perm(q1, q0, 0x0C0C0703u) | __builtin_amdgcn_perm(q3, q2, 0x07030C0Cu);
      *reinterpret_cast<uint32_t*>(dev::uniform_ptr(blrf + (int64_t)y * a.bpitch) + (uint32_t)xb) = o;
    }
  };
  // interior row y = r - 2 (2 <= y <= dh - 3): plain 5-row sum of the window
  auto emit_interior = [&](int y) {
    store_blur(y, (win[0][0] + win[1][0] + win[2][0]) + (win[3][0] + win[4][0]),
               (win[0][1] + win[1][1] + win[2][1]) + (win[3][1] + win[4][1]));
  };
  // the two top / bottom rows: BORDER_REFLECT_101 folds mirrored rows into window weights
  // (2 bits each, row r-4 first; row -1 = row 1, row -2 = row 2, row dh = row dh-2,
  // row dh+1 = row dh-3); weight * sum by selects and a shift (no 32-bit multiply)
  auto emit_border = [&](int y) {
    const uint32_t wts = y == 0 ? 0x22100u                          // rows 2 1 0 1 2
                       : y == 1 ? 0x11210u                          // rows 1 0 1 2 3
                       : y == dh - 2 ? 0x12110u                     // rows dh-4..dh-1, dh-2
                       : 0x12200u;                                  // dh-3 dh-2 dh-1 dh-2 dh-3
    uint32_t s01 = 0, s23 = 0;
#pragma unroll
    for (int i = 0; i < 5; i++) {
      const uint32_t wi = (wts >> (4 * i)) & 15u;   // 0, 1 or 2
      s01 += (wi & 1u ? win[i][0] : 0u) + (wi & 2u ? win[i][0] << 1 : 0u);
      s23 += (wi & 1u ? win[i][1] : 0u) + (wi & 2u ? win[i][1] << 1 : 0u);
    }
    store_blur(y, s01, s23);
  };
  auto push_row = [&](int r, uint32_t v) {
    if (RESIZE && core_lane && r >= seg0 && r < seg1)   // row base uniform, lane offset >= 0
      *reinterpret_cast<uint32_t*>(dev::uniform_ptr(dstf + (int64_t)r * a.dpitch) + (uint32_t)xb) = v;
    // lane neighbours by DPP wave shifts (VALU, no LDS round trip); lane 0 / 63 read 0
    // (bound_ctrl), and those lanes are halo lanes whose blurred output is never stored
    const uint32_t L = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138 /*wave_shr:1*/, 0xF, 0xF, true);
    const uint32_t R = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130 /*wave_shl:1*/, 0xF, 0xF, true);
    const uint32_t sc = __builtin_amdgcn_sad_u8(v, 0u, 0u);
    const uint32_t l2 = (L >> 16) & 0xFF, l3 = L >> 24, c0 = v & 0xFF, c3 = v >> 24;
    const uint32_t r0 = R & 0xFF, r1 = (R >> 8) & 0xFF;
    const uint32_t h0 = sc - c3 + l2 + l3, h1 = sc + l3, h2 = sc + r0, h3 = sc - c0 + r0 + r1;
#pragma unroll
    for (int i = 0; i < 4; i++) { win[i][0] = win[i + 1][0]; win[i][1] = win[i + 1][1]; }
    win[4][0] = h0 | (h1 << 16);
    win[4][1] = h2 | (h3 << 16);
    // blurred row y = r - 2 once rows y-2 .. y+2 are in (all wave-uniform); the last row of
    // the level also closes the two bottom rows
    const int y = r - 2;
    if (y >= seg0 && y < seg1) {
      if (y >= 2 && y <= dh - 3) emit_interior(y);
      else emit_border(y);
    }
    if (r == dh - 1) {
      if (dh - 2 >= seg0 && dh - 2 < seg1 && dh - 2 > y) emit_border(dh - 2);
      if (dh - 1 >= seg0 && dh - 1 < seg1 && dh - 1 > y) emit_border(dh - 1);
    }
  };
  auto pack4 = [&](const int (&h)[4]) {
    return (uint32_t)h[0] | ((uint32_t)h[1] << 8) | ((uint32_t)h[2] << 16) | ((uint32_t)h[3] << 24);
  };

  uint32_t pf[kPF][NDW];
  if (RESIZE) {
    // the segment's row tables (<= 68 rows) live in two VGPRs per lane and are read with
    // v_readlane (wave-uniform row index): no scalar-memory round trip per output row
    const int nrows = r_end - r_begin;
    uint32_t tabA = 0, tabB = 0, betA = 0, betB = 0;
    {
      auto pack_rows = [&](int r) {
        const int lo = min(max(a.yofs[r], 0), sh - 1), hi = min(max(a.yofs[r] + 1, 0), sh - 1);
        return (uint32_t)lo | ((uint32_t)hi << 16);
      };
      auto pack_beta = [&](int r) {
        return (uint32_t)(uint16_t)a.beta[2 * r] | ((uint32_t)(uint16_t)a.beta[2 * r + 1] << 16);
      };
      if (lane < nrows) { tabA = pack_rows(r_begin + lane); betA = pack_beta(r_begin + lane); }
      if (lane + 64 < nrows) { tabB = pack_rows(r_begin + 64 + lane); betB = pack_beta(r_begin + 64 + lane); }
    }
    auto row_tab = [&](int r) -> uint32_t {
      const int i = r - r_begin;
      return i < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)tabA, i)
                    : (uint32_t)__builtin_amdgcn_readlane((int)tabB, i - 64);
    };
    auto row_beta = [&](int r) -> uint32_t {
      const int i = r - r_begin;
      return i < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)betA, i)
                    : (uint32_t)__builtin_amdgcn_readlane((int)betB, i - 64);
    };
    const int sr0 = (int)(row_tab(r_begin) & 0xFFFF), sr1 = (int)(row_tab(r_end - 1) >> 16);
    // wave-uniform: every pixel of the strip (mirrors included) is in the SSE2 range (all
    // strips but the one holding the scalar tail), so the per-pixel select disappears
    const bool wave_sse = __ballot(simd != 15) == 0;
    // Two instances of the row loop, one per vertical form (the wave-uniform choice is made once,
    // so nothing of the scalar form is hoisted into the SSE2 loop).  The horizontal sums s << 4
    // (alphas pre-shifted) and the SSE2 operands (s >> 4) << 8 = (s << 4) & ~0xFF of the two
    // newest source rows ping-pong between register sets A and B by source-row parity (kPF is
    // even), so no per-row copies.
    static_assert(kPF % 2 == 0, "source-row ping-pong needs an even rows-in-flight count");
    auto run = [&](auto sse_tag) {
      constexpr bool SSE = decltype(sse_tag)::value;
      int hA[4] = {0, 0, 0, 0}, hB[4] = {0, 0, 0, 0};
      uint32_t xA[4] = {0, 0, 0, 0}, xB[4] = {0, 0, 0, 0};
      // the scalar-tail form's operands s = h >> 4 (strips holding the tail only), ping-pong too
      uint32_t uA[4] = {0, 0, 0, 0}, uB[4] = {0, 0, 0, 0};
      int r = r_begin;
      uint32_t tr = row_tab(r);
      auto consume = [&](int sr, const uint32_t (&v)[NDW], int (&hc)[4], uint32_t (&xc)[4],
                         uint32_t (&uc)[4], int (&hp)[4], uint32_t (&xp)[4], uint32_t (&up)[4]) {
        stage_and_gather(sr, v, hc);
#pragma unroll
        for (int k = 0; k < 4; k++) xc[k] = (uint32_t)hc[k] & 0x00FFFF00u;   // hc < 2^24
        if (!SSE) {
#pragma unroll
          for (int k = 0; k < 4; k++) uc[k] = (uint32_t)hc[k] >> 4;
        }
        while (r < r_end && (int)(tr >> 16) == sr) {
          const bool same = (int)(tr & 0xFFFF) == sr;
          const uint32_t bb = row_beta(r);
          int o[4];
          // (x0 b0 >> 16) = mulhi_u24(x0 << 8, b0 << 8) (sse_vres8); b in [0, 2048]
          const uint32_t B0 = (bb & 0xFFFFu) << 8, B1 = (bb >> 16) << 8;
          // both taps on this source row (the clamped edge rows, rare): the previous set
          // takes its value (every later output row of this source row is such a row too).
          // The empty asm keeps this a scalar branch: if-converted, the selects would also
          // hide the 24-bit operand range (quarter-rate v_mul_hi_u32)
          if (same) {
            asm volatile("" ::: "memory");
#pragma unroll
            for (int k = 0; k < 4; k++) { xp[k] = xc[k]; up[k] = uc[k]; }
          }
          if (SSE) {
#pragma unroll
            for (int k = 0; k < 4; k++) o[k] = (int)sse_vres8(xp[k], xc[k], B0, B1);
          } else {
            // the strip holding the scalar tail: the SSE2 form as above for pixels below
            // simd_end, FixedPtCast's (s0 b0 + s1 b1 + 2^21) >> 22 on 24-bit multiply-adds for
            // the tail (s <= 522240, b0 + b1 = 2048: no overflow, and the result is <= 255, so
            // vres_fixed's clamp is a no-op), then a per-pixel select (vres, bit for bit)
            const uint32_t b0 = bb & 0xFFFFu, b1 = bb >> 16;
#pragma unroll
            for (int k = 0; k < 4; k++) {
              const uint32_t vs = sse_vres8(xp[k], xc[k], B0, B1);
              const uint32_t vf = (__umul24(up[k], b0) + (__umul24(uc[k], b1) + (1u << 21))) >> 22;
              o[k] = (int)(((simd >> k) & 1) ? vs : vf);
            }
          }
          push_row(r, pack4(o));
          r++;
          if (r < r_end) tr = row_tab(r);
        }
      };
#pragma unroll
      for (int u = 0; u < kPF; u++)
        if (sr0 + u <= sr1) load_row(sr0 + u, pf[u]);
      for (int sr = sr0; sr <= sr1; sr += kPF) {   // kPF source rows in flight
#pragma unroll
        for (int u = 0; u < kPF; u++) {
          if (sr + u <= sr1) {
            if (u & 1) consume(sr + u, pf[u], hB, xB, uB, hA, xA, uA);
            else consume(sr + u, pf[u], hA, xA, uA, hB, xB, uB);
            if (sr + u + kPF <= sr1) load_row(sr + u + kPF, pf[u]);
          }
        }
      }
    };
    if (wave_sse) run(std::true_type{});
    else run(std::false_type{});
  } else {
    auto consume = [&](int r, const uint32_t (&v)[NDW]) {
      int h[4];
      stage_and_gather(r, v, h);
      push_row(r, pack4(h));
    };
#pragma unroll
    for (int u = 0; u < kPF; u++)
      if (r_begin + u < r_end) load_row(r_begin + u, pf[u]);
    for (int r = r_begin; r < r_end; r += kPF) {
#pragma unroll
      for (int u = 0; u < kPF; u++) {
        if (r + u < r_end) {
          consume(r + u, pf[u]);
          if (r + u + kPF < r_end) load_row(r + u + kPF, pf[u]);
        }
      }
    }
  }
}

void launch_pyr_blur(const PyrArgs& a, bool resize, bool wide, hipStream_t st) {
  const unsigned g = xcd_grid(a.nframes, (a.tiles_x * a.tiles_y + 3) / 4);
  if (!resize)
    hipLaunchKernelGGL((k_pyr_rows<false, 1>), dim3(g), dim3(256), 0, st, a);
  else if (!wide)
    hipLaunchKernelGGL((k_pyr_rows<true, 2>), dim3(g), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((k_pyr_rows<true, 3>), dim3(g), dim3(256), 0, st, a);
}

// ---------------------------------------------------------------------------
// mask pyramid: cv::resize(INTER_NEAREST) chain, unpadded levels
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_mask_nearest(const uint8_t* __restrict__ src, int sw,
                                                      int sh, int spitch, uint8_t* __restrict__ dst,
                                                      int dw, int dh, int dpitch, int64_t fstride) {
  const int dx = blockIdx.x * 64 + (threadIdx.x & 63);
  const int dy = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (dx >= dw || dy >= dh) return;
  const double ifx = 1. / ((double)dw / sw), ify = 1. / ((double)dh / sh);
  const int sx = min((int)floor(dx * ifx), sw - 1);
  const int sy = min((int)floor(dy * ify), sh - 1);
  const int64_t f = (int64_t)blockIdx.z * fstride;
  dst[f + (int64_t)dy * dpitch + dx] = src[f + (int64_t)sy * spitch + sx];
}

__global__ void k_copy_bytes(const uint8_t* __restrict__ src, int64_t sstride, int spitch,
                             uint8_t* __restrict__ dst, int64_t dstride, int dpitch, int w, int h) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (x >= w || y >= h) return;
  dst[(int64_t)blockIdx.z * dstride + (int64_t)y * dpitch + x] =
      src[(int64_t)blockIdx.z * sstride + (int64_t)y * spitch + x];
}

// mask pyramids of n masks; level 0 comes from d_masks (n x H x W, pitch W) unless
// d_masks == dst (level 0 already in place at pitch bpitch)
void launch_mask_pyramids(const Plan& pl, const uint8_t* d_masks, int n, uint8_t* dst,
                          hipStream_t st) {
  const LevelPlan& L0 = pl.lv[0];
  dim3 b(256);
  if (d_masks != dst)
    hipLaunchKernelGGL(k_copy_bytes, dim3((L0.w + 63) / 64, (L0.h + 3) / 4, n), b, 0, st, d_masks,
                       (int64_t)L0.w * L0.h, L0.w, dst, pl.mask_frame_bytes, L0.bpitch, L0.w, L0.h);
  for (int l = 1; l < pl.nlevels; l++) {
    const LevelPlan& S = pl.lv[l - 1];
    const LevelPlan& D = pl.lv[l];
    hipLaunchKernelGGL(k_mask_nearest, dim3((D.w + 63) / 64, (D.h + 3) / 4, n), b, 0, st,
                       dst + S.mask_off, S.w, S.h, S.bpitch, dst + D.mask_off, D.w, D.h, D.bpitch,
                       pl.mask_frame_bytes);
  }
}

}  // namespace mcs
