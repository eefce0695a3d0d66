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

constexpr int kPTW = 124, kPTH = 16, kPH = 2;   // core tile; halo tile = 128 x 20
constexpr int kHH = kPTH + 2 * kPH;              // 20 halo rows = 5 per wave
constexpr int kSrcMaxW = 288, kSrcMaxH = 48;     // source tile bound (scale <= 2.2, host-checked)
constexpr int kLvlW = kPTW + 8;                  // level tile origin at x0-4 (aligned core)

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

// One workgroup = 4 waves; wave w owns halo rows w, w+4, ...; lane owns halo columns
// lane and lane+64 (their resize coefficients stay in registers, row coefficients are
// wave-uniform scalars).
template <bool RESIZE>
__global__ __launch_bounds__(256) void k_pyr_blur(PyrArgs a) {
  __shared__ uint8_t s_src[RESIZE ? kSrcMaxH * kSrcMaxW : 4];
  __shared__ __attribute__((aligned(16))) uint8_t s_lvl[kHH * kLvlW];
  __shared__ uint16_t s_hs[kHH * kPTW];
  int f, item;
  if (!xcd_frame_map(blockIdx.x, a.nframes, a.tiles_x * a.tiles_y, &f, &item)) return;
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int x0 = (item % a.tiles_x) * kPTW, y0 = (item / a.tiles_x) * kPTH;
  const int dw = a.dw, dh = a.dh;
  const int lrow0 = y0 - kPH;  // s_lvl row 0 <-> level row y0-2
  const int lcol0 = x0 - 4;    // s_lvl col 0 <-> level col x0-4
  const uint8_t* S = a.src + (int64_t)f * a.src_fstride;
  const int ry0 = max(0, lrow0), ry1 = min(dh, y0 + kPTH + kPH);
  const int rx0 = max(0, x0 - kPH), rx1 = min(dw, x0 + kPTW + kPH);

  if (RESIZE) {
    const int sh = a.sh, sw = a.sw;
    const int sr0 = min(max(a.yofs[ry0], 0), sh - 1);
    const int sr1 = min(max(a.yofs[ry1 - 1] + 1, 0), sh - 1) + 1;
    const int sc0 = a.xofs[rx0], sc1 = min(a.xofs[rx1 - 1] + 1, sw - 1) + 1;
    for (int r = wv; r < sr1 - sr0; r += 4) {
      const uint8_t* srow = S + (int64_t)(sr0 + r) * a.spitch + sc0;
      for (int c = lane; c < sc1 - sc0; c += 64) s_src[r * kSrcMaxW + c] = srow[c];
    }
    // per-lane column coefficients for halo columns lane, lane + 64
    int sx[2], sx1[2], a0[2], a1[2];
    bool simd[2], cval[2];
#pragma unroll
    for (int m = 0; m < 2; m++) {
      const int c = x0 - kPH + lane + 64 * m;
      cval[m] = c >= rx0 && c < rx1;
      const int cc = cval[m] ? c : rx0;
      sx[m] = a.xofs[cc] - sc0;
      sx1[m] = min(a.xofs[cc] + 1, sw - 1) - sc0;
      a0[m] = a.alpha[2 * cc];
      a1[m] = a.alpha[2 * cc + 1];
      simd[m] = cc < a.simd_end;
    }
    __syncthreads();
    for (int r = ry0 + wv; r < ry1; r += 4) {
      const int sy = a.yofs[r];
      const int b0 = a.beta[2 * r], b1 = a.beta[2 * r + 1];
      const uint8_t* r0 = s_src + (min(max(sy, 0), sh - 1) - sr0) * kSrcMaxW;
      const uint8_t* r1 = s_src + (min(max(sy + 1, 0), sh - 1) - sr0) * kSrcMaxW;
      uint8_t* out = s_lvl + (r - lrow0) * kLvlW + (x0 - kPH - lcol0);
#pragma unroll
      for (int m = 0; m < 2; m++) {
        if (!cval[m]) continue;
        const int s0 = r0[sx[m]] * a0[m] + r0[sx1[m]] * a1[m];
        const int s1 = r1[sx[m]] * a0[m] + r1[sx1[m]] * a1[m];
        out[lane + 64 * m] = (uint8_t)vres(s0, s1, b0, b1, simd[m]);
      }
    }
  } else {
    for (int r = ry0 + wv; r < ry1; r += 4) {
      const uint8_t* srow = S + (int64_t)r * a.spitch;
      uint8_t* out = s_lvl + (r - lrow0) * kLvlW;
#pragma unroll
      for (int m = 0; m < 2; m++) {
        const int c = x0 - kPH + lane + 64 * m;
        if (c >= rx0 && c < rx1) out[c - lcol0] = srow[c];
      }
    }
  }
  __syncthreads();
  // raw level-l core tile -> HBM (aligned dwords: 31 per row, 16 rows)
  if (RESIZE) {
    for (int i = tid; i < kPTH * (kPTW / 4); i += 256) {
      const int ty = i / (kPTW / 4), tx = (i % (kPTW / 4)) * 4;
      const int y = y0 + ty;
      if (y < dh && x0 + tx < dw) {
        const uint32_t v = *reinterpret_cast<const uint32_t*>(&s_lvl[(ty + kPH) * kLvlW + 4 + tx]);
        *reinterpret_cast<uint32_t*>(a.dst + (int64_t)f * a.dst_fstride + (int64_t)y * a.dpitch + x0 + tx) = v;
      }
    }
  }
  // horizontal 5-sums (reflect-101 only at the level border), core columns
  for (int r = ry0 + wv; r < ry1; r += 4) {
    const uint8_t* row = s_lvl + (r - lrow0) * kLvlW;
#pragma unroll
    for (int m = 0; m < 2; m++) {
      const int cl = lane + 64 * m;
      if (cl >= kPTW) continue;
      const int c = x0 + cl;
      int s = 0;
      if (c < dw) {
        if (c >= 2 && c < dw - 2) {
          const uint8_t* q = row + (c - lcol0);
          s = q[-2] + q[-1] + q[0] + q[1] + q[2];
        } else {
#pragma unroll
          for (int d = -2; d <= 2; d++) s += row[refl101(c + d, dw) - lcol0];
        }
      }
      s_hs[(r - lrow0) * kPTW + cl] = (uint16_t)s;
    }
  }
  __syncthreads();
  for (int i = tid; i < kPTH * (kPTW / 4); i += 256) {
    const int ty = i / (kPTW / 4), tx = (i % (kPTW / 4)) * 4;
    const int y = y0 + ty;
    if (y < dh && x0 + tx < dw) {
      int rr[5];
#pragma unroll
      for (int d = -2; d <= 2; d++) rr[d + 2] = (refl101(y + d, dh) - lrow0) * kPTW;
      uint32_t packed = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int s = s_hs[rr[0] + tx + k] + s_hs[rr[1] + tx + k] + s_hs[rr[2] + tx + k] +
                      s_hs[rr[3] + tx + k] + s_hs[rr[4] + tx + k];
        packed |= (uint32_t)((2 * s + 25) / 50) << (8 * k);
      }
      *reinterpret_cast<uint32_t*>(a.blur + (int64_t)f * a.blur_fstride + (int64_t)y * a.bpitch + x0 + tx) = packed;
    }
  }
}

void launch_pyr_blur(const PyrArgs& a, bool resize, hipStream_t st) {
  const unsigned g = xcd_grid(a.nframes, a.tiles_x * a.tiles_y);
  if (resize)
    hipLaunchKernelGGL(k_pyr_blur<true>, dim3(g), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(k_pyr_blur<false>, dim3(g), dim3(256), 0, st, a);
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
