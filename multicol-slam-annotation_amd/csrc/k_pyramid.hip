// K1 + K5 fused: one pyramid level = cv::resize(INTER_LINEAR) of level l-1 and
// the 5x5 normalised box blur of level l, computed from one LDS tile.
//
// Reference: ComputePyramid src/mdBRIEFextractorOct.cpp:1158-1201 (resize chain) and the
// in-place boxFilter of operator() :1298-1301.  The reference pads every level by 25 px of
// BORDER_REFLECT_101 (:1185-1197) only so that later stages may read outside it; nothing
// downstream reads outside a level except the blur, which reflects explicitly here.
//
// Tile: 64 x 16 output pixels per 256-thread workgroup; the level-l tile is recomputed with
// a 2-pixel halo so raw and blurred tiles leave in one pass (stores are aligned dwords:
// levels >= 1 and all blurred levels have a 64-byte-aligned row pitch).
#include "common.hpp"
#include "extractor_kernels.hpp"

namespace mcs {

constexpr int kPTW = 64, kPTH = 16, kPH = 2;
constexpr int kSrcMaxW = 160, kSrcMaxH = 48;   // host-checked bounds of the source tile
constexpr int kLvlW = kPTW + 8;                 // level tile origin at x0-4 (aligned core)
constexpr int kLvlH = kPTH + 2 * kPH;

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

template <bool RESIZE>
__global__ __launch_bounds__(256) void k_pyr_blur(PyrArgs a) {
  __shared__ uint8_t s_src[RESIZE ? kSrcMaxH * kSrcMaxW : 4];
  __shared__ __attribute__((aligned(16))) uint8_t s_lvl[kLvlH * kLvlW];
  __shared__ uint16_t s_hs[kLvlH * kPTW];
  int f, item;
  if (!xcd_frame_map(blockIdx.x, a.nframes, a.tiles_x * a.tiles_y, &f, &item)) return;
  const int tid = threadIdx.x;
  const int x0 = (item % a.tiles_x) * kPTW, y0 = (item / a.tiles_x) * kPTH;
  const int dw = a.dw, dh = a.dh;
  const int ry0 = max(0, y0 - kPH), ry1 = min(dh, y0 + kPTH + kPH);
  const int rx0 = max(0, x0 - kPH), rx1 = min(dw, x0 + kPTW + kPH);
  const int hr = ry1 - ry0, hc = rx1 - rx0;
  const int lrow0 = y0 - kPH;  // s_lvl row 0 <-> level row y0-2
  const int lcol0 = x0 - 4;    // s_lvl col 0 <-> level col x0-4
  const uint8_t* S = a.src + (int64_t)f * a.src_fstride;

  if (RESIZE) {
    const int sh = a.sh, sw = a.sw;
    auto clipr = [sh](int y) { return y < 0 ? 0 : (y < sh ? y : sh - 1); };
    const int sr0 = clipr(a.yofs[ry0]), sr1 = clipr(a.yofs[ry1 - 1] + 1) + 1;
    const int sc0 = a.xofs[rx0], sc1 = min(a.xofs[rx1 - 1] + 1, sw - 1) + 1;
    const int srows = sr1 - sr0, scols = sc1 - sc0;
    for (int i = tid; i < srows * scols; i += 256) {
      const int r = i / scols, c = i - r * scols;
      s_src[r * kSrcMaxW + c] = S[(int64_t)(sr0 + r) * a.spitch + sc0 + c];
    }
    __syncthreads();
    for (int i = tid; i < hr * hc; i += 256) {
      const int r = ry0 + i / hc, c = rx0 + i % hc;
      const int sx = a.xofs[c] - sc0;
      const int sx1 = min(a.xofs[c] + 1, sw - 1) - sc0;
      const int a0 = a.alpha[2 * c], a1 = a.alpha[2 * c + 1];
      const int sy = a.yofs[r];
      const uint8_t* r0 = s_src + (clipr(sy) - sr0) * kSrcMaxW;
      const uint8_t* r1 = s_src + (clipr(sy + 1) - sr0) * kSrcMaxW;
      const int s0 = r0[sx] * a0 + r0[sx1] * a1;
      const int s1 = r1[sx] * a0 + r1[sx1] * a1;
      s_lvl[(r - lrow0) * kLvlW + (c - lcol0)] =
          (uint8_t)vres(s0, s1, a.beta[2 * r], a.beta[2 * r + 1], c < a.simd_end);
    }
  } else {
    for (int i = tid; i < hr * hc; i += 256) {
      const int r = ry0 + i / hc, c = rx0 + i % hc;
      s_lvl[(r - lrow0) * kLvlW + (c - lcol0)] = S[(int64_t)r * a.spitch + c];
    }
  }
  __syncthreads();
  // raw level-l core tile -> HBM (aligned dwords)
  const int ty = tid >> 4, tx = (tid & 15) * 4;
  const int y = y0 + ty;
  if (RESIZE && y < dh && x0 + tx < dw) {
    const uint32_t v = *reinterpret_cast<const uint32_t*>(&s_lvl[(ty + kPH) * kLvlW + 4 + tx]);
    *reinterpret_cast<uint32_t*>(a.dst + (int64_t)f * a.dst_fstride + (int64_t)y * a.dpitch + x0 + tx) = v;
  }
  // horizontal 5-sums for the halo rows, core columns (reflect-101 at the level border)
  for (int i = tid; i < hr * kPTW; i += 256) {
    const int r = i / kPTW, c = x0 + (i % kPTW);
    int s = 0;
    if (c < dw) {
      const uint8_t* row = s_lvl + (ry0 + r - lrow0) * kLvlW;
#pragma unroll
      for (int d = -2; d <= 2; d++) s += row[refl101(c + d, dw) - lcol0];
    }
    s_hs[(ry0 + r - lrow0) * kPTW + (c - x0)] = (uint16_t)s;
  }
  __syncthreads();
  if (y < dh && x0 + tx < dw) {
    uint32_t packed = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      int s = 0;
#pragma unroll
      for (int d = -2; d <= 2; d++) s += s_hs[(refl101(y + d, dh) - lrow0) * kPTW + tx + k];
      packed |= (uint32_t)((2 * s + 25) / 50) << (8 * k);
    }
    *reinterpret_cast<uint32_t*>(a.blur + (int64_t)f * a.blur_fstride + (int64_t)y * a.bpitch + x0 + tx) = packed;
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
