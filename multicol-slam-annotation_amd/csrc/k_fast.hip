// K2: FAST-9/16 + per-cell 3x3 non-max suppression + runByPixelsMask, one wave per FAST
// cell, four cells per 256-thread workgroup, all cells of a frame on one XCD.
//
// Reference: ComputeKeyPointsOctTree src/mdBRIEFextractorOct.cpp:874-949, which runs
// FastFeatureDetector(th, nonmax, TYPE_9_16)::detect on every 30 px cell ROI; the OpenCV
// semantics (FAST_t<16>, cornerScore<16>, NMS before the mask) are pinned in SURVEY A.4.
//
// Per cell the wave runs three phases over its LDS tile (window + 3 px halo):
//   A  compass pre-test on every window pixel: a 9-long arc of the 16-circle always holds
//      two ADJACENT compass points (0/4/8/12), so a pixel can only be a corner if such a pair
//      is all-darker or all-brighter.  Survivors are compacted in raster order.
//   B  exact test + score for the survivors only, branch-free: with d_k = v - p_k,
//      dark arc  = max_k min(d_k..d_k+8),  bright arc = -min_k max(d_k..d_k+8)
//      (v_min3/v_max3 doubling); corner <=> either > t; score = max(t, dark, bright) - 1,
//      which is exactly cornerScore<16>'s a0/b0 recursion.
//   C  NMS (strict > against the 8 neighbours inside the same window, others count 0) and
//      the mask test for the corners of the previous chunk, compacted in raster order.
#include "common.hpp"
#include "extractor_kernels.hpp"

namespace mcs {

constexpr int kChunk = 256;

// Per-wave LDS carve-up, sized on the host from the largest FAST window of the plan (about
// 31 x 31 px for 30 px cells) so a workgroup needs ~16 KB instead of a 64 px worst case:
//   tile  [th_max][tp]      window + 3 px halo (+3 bytes alignment slack per row)
//   smap  [ww*wh]           score + 1 for corners, 0 otherwise (window raster)
//   surv  u16[kChunk]       compass-test survivors of the current chunk (y<<8 | x)
//   corner u16[2][kChunk]   corners of the current / previous chunk
__device__ __forceinline__ int min3i(int a, int b, int c) { return min(min(a, b), c); }
__device__ __forceinline__ int max3i(int a, int b, int c) { return max(max(a, b), c); }

__global__ __launch_bounds__(256) void k_fast_cells(FastArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_dyn[];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int kFTP = a.tile_pitch;
  uint8_t* const tile = lds_dyn + wv * a.wave_lds;
  uint8_t* const smap = tile + a.smap_off;
  uint16_t* const surv = reinterpret_cast<uint16_t*>(tile + a.surv_off);
  uint16_t* const corner_base = surv + kChunk;
  int f, item;
  const int cells_per_block_row = (a.ncells + 3) / 4;
  if (!xcd_frame_map(blockIdx.x, a.nframes, cells_per_block_row, &f, &item)) return;
  const int ci = item * 4 + wv;
  if (ci >= a.ncells) return;
  const CellDesc c = a.cells[ci];
  const int l = c.level;
  int32_t* cnt_out = a.cell_counts + (int64_t)f * a.ncells + ci;
  const uint8_t* mask = nullptr;
  if (a.mask_pyr) {
    const int mi = a.mask_index ? a.mask_index[f] : 0;
    if (a.cell_flags && a.cell_flags[(int64_t)mi * a.ncells + ci] == 0) {
      if (lane == 0) *cnt_out = 0;
      return;
    }
    mask = a.mask_pyr + (int64_t)mi * a.mask_fstride + a.lp.mask_off[l];
  }
  const int pitch = a.lp.pitch[l], mw = a.lp.w[l];
  const uint8_t* img = (l == 0) ? a.img0 + (int64_t)f * a.img0_fstride
                                : a.pyr + (int64_t)f * a.pyr_fstride + a.lp.pyr_off[l];
  const int ww = max(0, c.wx1 - c.wx0), wh = max(0, c.wy1 - c.wy0);
  const int npx = ww * wh;
  const int th = wh + 6, nd = (ww + 6 + 3) >> 2;
  // ---- stage tile (window + 3px halo) with aligned dword loads + alignbyte;
  // row = i / nd by a multiply-high with the cell's magic (exact for i < 2^16)
  {
    const uint32_t magic = 0xFFFFFFFFu / (uint32_t)nd + 1u;
    const uint8_t* gbase = img + (int64_t)(c.wy0 - 3) * pitch + (c.wx0 - 3);
    for (int i = lane; i < th * nd; i += 64) {
      const int r = (int)__umulhi((uint32_t)i, magic), j = i - r * nd;
      const uint8_t* gp = gbase + (int64_t)r * pitch + 4 * j;
      const uint32_t* ap = dev::align_down4(gp);
      const uint32_t d0 = ap[0], d1 = ap[1];
      *reinterpret_cast<uint32_t*>(&tile[r * kFTP + 4 * j]) =
          __builtin_amdgcn_alignbyte(d1, d0, (uint32_t)((uintptr_t)gp & 3));
    }
  }
  for (int i = lane; i < (npx + 3) / 4; i += 64) reinterpret_cast<uint32_t*>(smap)[i] = 0u;
  dev::wave_sync();

  const int t = a.threshold;
  uint32_t* out = a.slots + (int64_t)f * a.slots_fstride + c.slot_off;
  int count = 0;
  int ncorner_prev = 0;
  int prev_buf = 0;
  const int nchunks = (npx + kChunk - 1) / kChunk;

  auto nms_emit = [&](int buf, int nc) {
    for (int j0 = 0; j0 < nc; j0 += 64) {
      const int j = j0 + lane;
      bool keep = false;
      int x = 0, y = 0, s = 0;
      if (j < nc) {
        const int pk = corner_base[buf * kChunk + j];
        y = pk >> 8; x = pk & 0xFF;
        s = smap[y * ww + x] - 1;
        keep = true;
#pragma unroll
        for (int dy = -1; dy <= 1; dy++)
#pragma unroll
          for (int dx = -1; dx <= 1; dx++) {
            if (dx == 0 && dy == 0) continue;
            const int xx = x + dx, yy = y + dy;
            int ns = 0;
            if (xx >= 0 && xx < ww && yy >= 0 && yy < wh) {
              const int e = smap[yy * ww + xx];
              ns = e ? e - 1 : 0;
            }
            keep = keep && (s > ns);
          }
        if (keep && mask) keep = mask[(int64_t)(c.wy0 + y) * mw + (c.wx0 + x)] != 0;
      }
      const uint64_t b = __ballot(keep);
      if (keep) {
        const int pos = count + __popcll(b & dev::lanemask_lt());
        out[pos] = (uint32_t)(c.wx0 + x - kMinBorder) | ((uint32_t)(c.wy0 + y - kMinBorder) << 12) |
                   ((uint32_t)s << 24);
      }
      count += __popcll(b);
    }
  };

  // raster position of this lane's pixel, advanced by 64 pixels per step without divisions
  int py = lane / max(ww, 1), px = lane - py * max(ww, 1);
  const int sdy = 64 / max(ww, 1), sdx = 64 - sdy * max(ww, 1);
  for (int ch = 0; ch < nchunks; ch++) {
    const int base = ch * kChunk;
    // ---- A: compass pre-test, ordered compaction of survivors
    int ns = 0;
#pragma unroll
    for (int k = 0; k < kChunk / 64; k++) {
      const int i = base + 64 * k + lane;
      const int y = py, x = px;
      px += sdx; py += sdy;
      if (px >= ww) { px -= ww; py++; }
      bool pass = false;
      if (i < npx) {
        const uint8_t* p = &tile[(y + 3) * kFTP + x + 3];
        const int v = p[0];
        const int q0 = p[3 * kFTP], q4 = p[3], q8 = p[-3 * kFTP], q12 = p[-3];
        const int lo = v - t, hi = v + t;
        const bool d0 = q0 < lo, d4 = q4 < lo, d8 = q8 < lo, d12 = q12 < lo;
        const bool b0 = q0 > hi, b4 = q4 > hi, b8 = q8 > hi, b12 = q12 > hi;
        pass = (d0 && d4) || (d4 && d8) || (d8 && d12) || (d12 && d0) ||
               (b0 && b4) || (b4 && b8) || (b8 && b12) || (b12 && b0);
      }
      const uint64_t bal = __ballot(pass);
      if (pass) surv[ns + __popcll(bal & dev::lanemask_lt())] = (uint16_t)((y << 8) | x);
      ns += __popcll(bal);
    }
    dev::wave_sync();
    // ---- B: exact FAST test + score for survivors; corners kept in raster order
    const int cur_buf = ch & 1;
    int ncorner = 0;
    for (int j0 = 0; j0 < ns; j0 += 64) {
      const int j = j0 + lane;
      bool corner = false;
      int idx = 0;
      if (j < ns) {
        idx = surv[j];
        const int y = idx >> 8, x = idx & 0xFF;
        const uint8_t* p = &tile[(y + 3) * kFTP + x + 3];
        const int v = p[0];
        int d[16];
        // circle (dx,dy): (0,3),(1,3),(2,2),(3,1),(3,0),(3,-1),(2,-2),(1,-3),(0,-3),(-1,-3),
        //                 (-2,-2),(-3,-1),(-3,0),(-3,1),(-2,2),(-1,3)
        d[0] = v - p[3 * kFTP];      d[1] = v - p[3 * kFTP + 1];  d[2] = v - p[2 * kFTP + 2];
        d[3] = v - p[kFTP + 3];      d[4] = v - p[3];             d[5] = v - p[-kFTP + 3];
        d[6] = v - p[-2 * kFTP + 2]; d[7] = v - p[-3 * kFTP + 1]; d[8] = v - p[-3 * kFTP];
        d[9] = v - p[-3 * kFTP - 1]; d[10] = v - p[-2 * kFTP - 2]; d[11] = v - p[-kFTP - 3];
        d[12] = v - p[-3];           d[13] = v - p[kFTP - 3];     d[14] = v - p[2 * kFTP - 2];
        d[15] = v - p[3 * kFTP - 1];
        int m3[16], M3[16];
#pragma unroll
        for (int k = 0; k < 16; k++) {
          m3[k] = min3i(d[k], d[(k + 1) & 15], d[(k + 2) & 15]);
          M3[k] = max3i(d[k], d[(k + 1) & 15], d[(k + 2) & 15]);
        }
        int dark = -1000, brightmin = 1000;
#pragma unroll
        for (int k = 0; k < 16; k++) {
          dark = max(dark, min3i(m3[k], m3[(k + 3) & 15], m3[(k + 6) & 15]));
          brightmin = min(brightmin, max3i(M3[k], M3[(k + 3) & 15], M3[(k + 6) & 15]));
        }
        const int bright = -brightmin;
        corner = dark > t || bright > t;
        if (corner) {
          const int score = max(max(t, dark), bright) - 1;
          smap[y * ww + x] = (uint8_t)(score + 1);
        }
      }
      const uint64_t bal = __ballot(corner);
      if (corner) corner_base[cur_buf * kChunk + ncorner + __popcll(bal & dev::lanemask_lt())] = (uint16_t)idx;
      ncorner += __popcll(bal);
    }
    dev::wave_sync();
    // ---- C: NMS + mask for the previous chunk (its neighbour rows are now scored)
    if (ch > 0) nms_emit(prev_buf, ncorner_prev);
    dev::wave_sync();
    prev_buf = cur_buf;
    ncorner_prev = ncorner;
  }
  if (nchunks > 0) nms_emit(prev_buf, ncorner_prev);
  if (lane == 0) *cnt_out = count;
}

void launch_fast_cells(const FastArgs& a, hipStream_t st) {
  const unsigned g = xcd_grid(a.nframes, (a.ncells + 3) / 4);
  hipLaunchKernelGGL(k_fast_cells, dim3(g), dim3(256), (size_t)4 * a.wave_lds, st, a);
}

}  // namespace mcs
