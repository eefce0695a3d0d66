// K1 + K5 fused: one pyramid level = cv::resize(INTER_LINEAR) of level l-1 and
// the 5x5 normalised box blur of level l, computed from one LDS tile.
//
// Reference: ComputePyramid src/mdBRIEFextractorOct.cpp:1158-1201 (resize chain) and the
// in-place boxFilter of operator() :1298-1301.  The reference pads every level by 25 px of
// BORDER_REFLECT_101 (:1185-1197) only so that later stages may read outside it; nothing
// downstream reads outside a level except the blur, which reflects explicitly here.
//
// Tile: 124 x 16 output pixels per 256-thread workgroup; the level-l tile is recomputed
// with a 2-pixel halo (128 x 20) so raw and blurred tiles leave in one pass (stores are
// aligned dwords: levels >= 1 and all blurred levels have a 64-byte-aligned row pitch).
#include "common.hpp"
#include "extractor_kernels.hpp"

namespace mcs {

__device__ __forceinline__ int refl101(int p, int n) {
  p = p < 0 ? -p : p;
  return p >= n ? 2 * n - 2 - p : p;
}

__device__ __forceinline__ int vres(int s0, int s1, int b0, int b1, bool simd) {
  int v;
  if (simd) {  // OpenCV 3.1 SSE2 VResizeLinearVec_32s8u
    const int x0 = max(-32768, min(32767, s0 >> 4));
    const int y0 = max(-32768, min(32767, s1 >> 4));
    int t = ((x0 * b0) >> 16) + ((y0 * b1) >> 16);
    t = max(-32768, min(32767, t));
    t = max(-32768, min(32767, t + 2));
    v = t >> 2;
  } else {
    v = (s0 * b0 + s1 * b1 + (1 << 21)) >> 22;  // FixedPtCast<int,uchar,22>
  }
  return max(0, min(255, v));
}

// (2s + 25) / 50 for 2s + 25 <= 12775 (s = 5x5 sum of u8) by multiply-shift;
// exact: 20972 / 2^20 - 1/50 < 4.6e-7 and 12775 * 4.6e-7 < 1/50 (checked on the host too)
__device__ __forceinline__ uint32_t div50(uint32_t n) { return (n * 20972u) >> 20; }

// Row-streaming pyramid level: one wave owns a strip of `core` (<= 248) output columns and a
// segment of `seg_rows` rows.  Lane L holds 4 consecutive pixels [xs-4+4L, xs+4L); lane 0 and
// the lane after the core are the +-2 px halo of the blur.  Rows are produced top to bottom
// (with a 2-row halo above and below the segment), each row:
//   RESIZE: the source rows it needs (yofs[r], yofs[r]+1) are streamed once per wave with
//           aligned dword loads (one row prefetched ahead), horizontally resized per lane
//           (coefficients in registers) and kept for the next output row;
//   level 0: the input row is streamed the same way;
// then the raw row is written out (RESIZE), horizontal 5-sums go into a per-wave LDS ring of
// 8 rows, and once row r+2 exists the blurred row r is summed vertically and written.
// No workgroup barriers: every wave works alone (wave-local LDS ordering only).
constexpr int kStageDW = 192;    // staged source row (dwords), scale <= 2.2
constexpr int kRowBufDW = 66;    // raw row bytes of px [xs-4, xs+260)
constexpr int kRing = 8;

struct PyrWaveLds {
  uint32_t stage[kStageDW];
  uint32_t row[kRowBufDW];
  uint2 ring[kRing][64];
};

template <bool RESIZE>
__global__ __launch_bounds__(256) void k_pyr_rows(PyrArgs a) {
  __shared__ PyrWaveLds lds_all[4];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  PyrWaveLds& W = lds_all[wv];
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
  uint8_t* const rowb = reinterpret_cast<uint8_t*>(W.row);
  const uint8_t* const stb = reinterpret_cast<const uint8_t*>(W.stage);

  // source columns staged per row: [c_lo, c_hi]
  int c_lo, c_hi;
  int sx[4], sx1[4], a0[4], a1[4];
  bool simd[4];
  if (RESIZE) {
    c_lo = a.xofs[max(xs - 4, 0)];
    c_hi = min(a.xofs[min(xs + core + 3, dw - 1)] + 1, a.sw - 1);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int p = min(max(xb + k, 0), dw - 1);
      sx[k] = a.xofs[p] - c_lo;
      sx1[k] = min(a.xofs[p] + 1, a.sw - 1) - c_lo;
      a0[k] = a.alpha[2 * p];
      a1[k] = a.alpha[2 * p + 1];
      simd[k] = p < a.simd_end;
    }
  } else {
    c_lo = max(xs - 4, 0);
    c_hi = min(xs + core + 3, dw - 1);
  }
  const int nbytes0 = c_hi - c_lo + 1;
  const int sh = RESIZE ? a.sh : dh;

  // ---- streamed source row: aligned dwords covering [c_lo, c_hi] of row sr
  auto row_base = [&](int sr) -> const uint8_t* { return S + (int64_t)sr * a.spitch; };
  auto load_row = [&](int sr, uint32_t (&v)[3]) {
    const uintptr_t st = (uintptr_t)(row_base(sr) + c_lo);
    const uint32_t* ap = reinterpret_cast<const uint32_t*>(st & ~(uintptr_t)3);
    const int ndw = ((int)(st & 3) + nbytes0 + 3) >> 2;
    const bool last = sr == sh - 1;
#pragma unroll
    for (int m = 0; m < 3; m++) {
      const int j = lane + 64 * m;
      v[m] = 0;
      if (j < ndw) {
        const uintptr_t q = (uintptr_t)(ap + j);
        if (!last || q + 4 <= (uintptr_t)(row_base(sr) + (RESIZE ? a.sw : dw))) {
          v[m] = ap[j];
        } else {   // never read past the end of the last row (it may end the buffer)
          const uintptr_t end = (uintptr_t)(row_base(sr) + (RESIZE ? a.sw : dw));
          for (int k = 0; k < 4; k++)
            if (q + k < end) v[m] |= (uint32_t)(*reinterpret_cast<const uint8_t*>(q + k)) << (8 * k);
        }
      }
    }
  };
  auto stage_row = [&](const uint32_t (&v)[3]) {
#pragma unroll
    for (int m = 0; m < 3; m++) {
      const int j = lane + 64 * m;
      if (j < kStageDW) W.stage[j] = v[m];
    }
  };

  // ---- raw row -> store, horizontal 5-sums into the ring, blurred rows out
  int next_emit = seg0;
  uint8_t* const dstf = RESIZE ? a.dst + (int64_t)f * a.dst_fstride : nullptr;
  uint8_t* const blrf = a.blur + (int64_t)f * a.blur_fstride;
  auto push_row = [&](int r, uint32_t v) {
    if (RESIZE && core_lane && r >= seg0 && r < seg1)
      *reinterpret_cast<uint32_t*>(dstf + (int64_t)r * a.dpitch + xb) = v;
    W.row[lane] = v;
    dev::wave_sync();
    // reflect-101 across the level's left / right border (px -1,-2 and dw, dw+1)
    if (lane == 0 && xs == 0) { rowb[3] = rowb[5]; rowb[2] = rowb[6]; }
    if (lane == 1 && xcore1 == dw) {
      const int ib = dw - (xs - 4);
      rowb[ib] = rowb[ib - 2];
      rowb[ib + 1] = rowb[ib - 3];
    }
    dev::wave_sync();
    if (lane >= 1 && lane < kRowBufDW - 1) {
      const uint32_t L = W.row[lane - 1], C = W.row[lane], R = W.row[lane + 1];
      const uint32_t sc = __builtin_amdgcn_sad_u8(C, 0u, 0u);
      const uint32_t l2 = (L >> 16) & 0xFF, l3 = L >> 24, c0 = C & 0xFF, c3 = C >> 24;
      const uint32_t r0 = R & 0xFF, r1 = (R >> 8) & 0xFF;
      const uint32_t h0 = sc - c3 + l2 + l3, h1 = sc + l3, h2 = sc + r0, h3 = sc - c0 + r0 + r1;
      W.ring[r & (kRing - 1)][lane] = make_uint2(h0 | (h1 << 16), h2 | (h3 << 16));
    }
    dev::wave_sync();
    const int upto = (r == dh - 1) ? dh - 1 : r - 2;
    for (; next_emit <= upto && next_emit < seg1; next_emit++) {
      const int y = next_emit;
      uint32_t s01 = 0, s23 = 0;
#pragma unroll
      for (int d = -2; d <= 2; d++) {
        const uint2 h = W.ring[refl101(y + d, dh) & (kRing - 1)][lane];
        s01 += h.x;   // two u16 lanes, no carry (5 * 1275 < 65536)
        s23 += h.y;
      }
      if (core_lane) {
        const uint32_t o = div50(2 * (s01 & 0xFFFF) + 25) | (div50(2 * (s01 >> 16) + 25) << 8) |
                           (div50(2 * (s23 & 0xFFFF) + 25) << 16) | (div50(2 * (s23 >> 16) + 25) << 24);
        *reinterpret_cast<uint32_t*>(blrf + (int64_t)y * a.bpitch + xb) = o;
      }
    }
  };

  if (RESIZE) {
    // source rows feeding output rows [r_begin, r_end)
    auto lo_of = [&](int r) { return min(max(a.yofs[r], 0), sh - 1); };
    auto hi_of = [&](int r) { return min(max(a.yofs[r] + 1, 0), sh - 1); };
    const int sr0 = lo_of(r_begin), sr1 = hi_of(r_end - 1);
    int hprev[4] = {0, 0, 0, 0}, hcur[4] = {0, 0, 0, 0};
    uint32_t pf[3];
    load_row(sr0, pf);
    int r = r_begin;
    for (int sr = sr0; sr <= sr1; sr++) {
      uint32_t cur[3] = {pf[0], pf[1], pf[2]};
      if (sr < sr1) load_row(sr + 1, pf);
      const int shft = (int)(((uintptr_t)(row_base(sr) + c_lo)) & 3);
      stage_row(cur);
      dev::wave_sync();
#pragma unroll
      for (int k = 0; k < 4; k++) {
        hprev[k] = hcur[k];
        hcur[k] = stb[shft + sx[k]] * a0[k] + stb[shft + sx1[k]] * a1[k];
      }
      dev::wave_sync();
      for (; r < r_end && hi_of(r) == sr; r++) {
        const bool same = lo_of(r) == sr;
        const int b0 = a.beta[2 * r], b1 = a.beta[2 * r + 1];
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int s0 = same ? hcur[k] : hprev[k];
          v |= (uint32_t)vres(s0, hcur[k], b0, b1, simd[k]) << (8 * k);
        }
        push_row(r, v);
      }
    }
  } else {
    uint32_t pf[3];
    load_row(r_begin, pf);
    for (int r = r_begin; r < r_end; r++) {
      uint32_t cur[3] = {pf[0], pf[1], pf[2]};
      if (r + 1 < r_end) load_row(r + 1, pf);
      const int shft = (int)(((uintptr_t)(row_base(r) + c_lo)) & 3);
      stage_row(cur);
      dev::wave_sync();
      // lane's 4 px [xb, xb+4) sit at staged byte shft + (xb - c_lo); px outside the level
      // are replaced by the border reflection in push_row
      const int o = shft + (xb - c_lo);
      uint32_t v = 0;
      if (o >= 0 && o + 4 <= 4 * kStageDW) {
        const uint32_t w0 = W.stage[o >> 2], w1 = W.stage[min((o >> 2) + 1, kStageDW - 1)];
        v = __builtin_amdgcn_alignbyte(w1, w0, (uint32_t)(o & 3));
      }
      dev::wave_sync();
      push_row(r, v);
    }
  }
}

void launch_pyr_blur(const PyrArgs& a, bool resize, bool wide, hipStream_t st) {
  (void)wide;
  const unsigned g = xcd_grid(a.nframes, (a.tiles_x * a.tiles_y + 3) / 4);
  if (resize)
    hipLaunchKernelGGL(k_pyr_rows<true>, dim3(g), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(k_pyr_rows<false>, dim3(g), dim3(256), 0, st, a);
}

// ---------------------------------------------------------------------------
// mask pyramid: cv::resize(INTER_NEAREST) chain, unpadded levels
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_mask_nearest(const uint8_t* __restrict__ src, int sw,
                                                      int sh, uint8_t* __restrict__ dst, int dw,
                                                      int dh, int64_t fstride) {
  const int dx = blockIdx.x * 64 + (threadIdx.x & 63);
  const int dy = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (dx >= dw || dy >= dh) return;
  const double ifx = 1. / ((double)dw / sw), ify = 1. / ((double)dh / sh);
  const int sx = min((int)floor(dx * ifx), sw - 1);
  const int sy = min((int)floor(dy * ify), sh - 1);
  const int64_t f = (int64_t)blockIdx.z * fstride;
  dst[f + (int64_t)dy * dw + dx] = src[f + (int64_t)sy * sw + sx];
}

__global__ void k_copy_bytes(const uint8_t* __restrict__ src, int64_t sstride,
                             uint8_t* __restrict__ dst, int64_t dstride, int w, int h) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (x >= w || y >= h) return;
  dst[(int64_t)blockIdx.z * dstride + (int64_t)y * w + x] =
      src[(int64_t)blockIdx.z * sstride + (int64_t)y * w + x];
}

void launch_mask_pyramids(const Plan& pl, const uint8_t* d_masks, int n, uint8_t* dst,
                          hipStream_t st) {
  const LevelPlan& L0 = pl.lv[0];
  dim3 b(256);
  hipLaunchKernelGGL(k_copy_bytes, dim3((L0.w + 63) / 64, (L0.h + 3) / 4, n), b, 0, st, d_masks,
                     (int64_t)L0.w * L0.h, dst, pl.mask_frame_bytes, L0.w, L0.h);
  for (int l = 1; l < pl.nlevels; l++) {
    const LevelPlan& S = pl.lv[l - 1];
    const LevelPlan& D = pl.lv[l];
    hipLaunchKernelGGL(k_mask_nearest, dim3((D.w + 63) / 64, (D.h + 3) / 4, n), b, 0, st,
                       dst + S.mask_off, S.w, S.h, dst + D.mask_off, D.w, D.h,
                       pl.mask_frame_bytes);
  }
}

// any nonzero mask pixel in a cell's detection window?  (runByPixelsMask can only keep
// keypoints on nonzero mask pixels, so a cell without any produces no candidates)
__global__ __launch_bounds__(64) void k_cell_maskflags(const CellDesc* __restrict__ cells,
                                                       int ncells, const uint8_t* __restrict__ mp,
                                                       int64_t mfs, LevelPtrs lp,
                                                       uint8_t* __restrict__ flags) {
  const int c = blockIdx.x, m = blockIdx.y;
  const CellDesc cd = cells[c];
  const int ww = max(0, cd.wx1 - cd.wx0), wh = max(0, cd.wy1 - cd.wy0);
  const uint8_t* mk = mp + (int64_t)m * mfs + lp.mask_off[cd.level];
  const int w = lp.w[cd.level];
  bool any = false;
  for (int i = threadIdx.x; i < ww * wh; i += 64) {
    const int y = i / ww, x = i - y * ww;
    any |= mk[(int64_t)(cd.wy0 + y) * w + cd.wx0 + x] != 0;
  }
  const uint64_t b = __ballot(any);
  if (threadIdx.x == 0) flags[(int64_t)m * ncells + c] = b != 0;
}

void launch_cell_maskflags(const Plan& pl, const CellDesc* d_cells, const uint8_t* mask_pyr,
                           int n_masks, uint8_t* flags, hipStream_t st) {
  LevelPtrs lp;
  for (int l = 0; l < kMaxLevels; l++) {
    const bool v = l < pl.nlevels;
    lp.w[l] = v ? pl.lv[l].w : 0; lp.h[l] = v ? pl.lv[l].h : 0;
    lp.pitch[l] = v ? pl.lv[l].pitch : 0; lp.bpitch[l] = v ? pl.lv[l].bpitch : 0;
    lp.pyr_off[l] = v ? pl.lv[l].pyr_off : 0; lp.img_off[l] = v ? pl.lv[l].img_off : 0;
    lp.mask_off[l] = v ? pl.lv[l].mask_off : 0;
  }
  hipLaunchKernelGGL(k_cell_maskflags, dim3((unsigned)pl.cells.size(), n_masks), dim3(64), 0, st,
                     d_cells, (int)pl.cells.size(), mask_pyr, pl.mask_frame_bytes, lp, flags);
}

}  // namespace mcs
