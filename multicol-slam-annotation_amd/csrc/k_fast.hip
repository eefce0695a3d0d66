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
//      is all-darker or all-brighter.  Each lane tests a quad of 4 horizontally adjacent
//      pixels with dword LDS reads and packed u16 min/max/saturating-subtract on the even and
//      odd bytes (v_perm split); survivors are compacted in raster order.
//   B  exact test + score for the survivors only, branch-free: with d_k = v - p_k,
//      dark arc  = max_k min(d_k..d_k+8),  bright arc = -min_k max(d_k..d_k+8)
//      (v_min3/v_max3 doubling); corner <=> either > t; score = max(t, dark, bright) - 1,
//      which is exactly cornerScore<16>'s a0/b0 recursion.
//   C  NMS (strict > against the 8 neighbours inside the same window, others count 0) and
//      the mask test for the corners of the previous chunk, compacted in raster order.
#include "common.hpp"
#include "extractor_kernels.hpp"

namespace mcs {

// Per-wave LDS carve-up, sized on the host from the largest FAST window of the plan (about
// 31 x 31 px for 30 px cells) so a workgroup needs ~16 KB instead of a 64 px worst case:
//   tile  [th_max][tp]      window + 3 px halo (+3 bytes alignment slack per row)
//   smap  [(ww+2)*(wh+2)]   score + 1 for corners, 0 otherwise (window raster + zero ring)
//   surv  u16[ww*wh]        compass-test survivors (y<<8 | x), then the corners in place
typedef unsigned short us2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ us2 as_us2(uint32_t w) { return __builtin_bit_cast(us2, w); }
__device__ __forceinline__ uint32_t as_u32(us2 v) { return __builtin_bit_cast(uint32_t, v); }
// even / odd bytes of a dword as two u16 lanes
__device__ __forceinline__ us2 even_b(uint32_t w) { return as_us2(__builtin_amdgcn_perm(0u, w, 0x0c020c00u)); }
__device__ __forceinline__ us2 odd_b(uint32_t w) { return as_us2(__builtin_amdgcn_perm(0u, w, 0x0c030c01u)); }
// compass pre-test for two pixels: nonzero u16 lane <=> some adjacent compass pair (a,b),
// (b,c), (c,d), (d,a) is all-darker (max < v - t, v - t saturated at 0: nothing is darker
// than a negative bound) or all-brighter (min > v + t)
__device__ __forceinline__ uint32_t compass2(us2 v, us2 a, us2 b, us2 c, us2 d, us2 t2) {
  const us2 lo = __builtin_elementwise_sub_sat(v, t2), hi = v + t2;
  const us2 md = __builtin_elementwise_min(
      __builtin_elementwise_min(__builtin_elementwise_max(a, b), __builtin_elementwise_max(b, c)),
      __builtin_elementwise_min(__builtin_elementwise_max(c, d), __builtin_elementwise_max(d, a)));
  const us2 mb = __builtin_elementwise_max(
      __builtin_elementwise_max(__builtin_elementwise_min(a, b), __builtin_elementwise_min(b, c)),
      __builtin_elementwise_max(__builtin_elementwise_min(c, d), __builtin_elementwise_min(d, a)));
  return as_u32(__builtin_elementwise_sub_sat(lo, md)) | as_u32(__builtin_elementwise_sub_sat(mb, hi));
}

__device__ __forceinline__ int min3i(int a, int b, int c) { return min(min(a, b), c); }
__device__ __forceinline__ int max3i(int a, int b, int c) { return max(max(a, b), c); }

__global__ __launch_bounds__(256) void k_fast_cells(FastArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_dyn[];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int kFTP = a.tile_pitch;
  uint8_t* const tile = lds_dyn + wv * a.wave_lds;
  uint8_t* const smap = tile + a.smap_off;
  uint16_t* const surv = reinterpret_cast<uint16_t*>(tile + a.surv_off);
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
  const int pitch = a.lp.pitch[l], mw = a.lp.bpitch[l];   // mask pyramid pitch = bpitch
  const uint8_t* img = (l == 0) ? a.img0 + (int64_t)f * a.img0_fstride
                                : a.pyr + (int64_t)f * a.pyr_fstride + a.lp.pyr_off[l];
  const int ww = max(0, c.wx1 - c.wx0), wh = max(0, c.wy1 - c.wy0);
  // tile column c = window column c - 4 (so a quad's centre dword is aligned); a row holds
  // the quads' reads up to window column 4*nq + 3 + 4
  const int nq = (ww + 3) >> 2;
  const int th = wh + 6, nd = nq + 2;
  // ---- stage tile (window + 3px halo) with aligned dword loads + alignbyte;
  // row = i / nd by a multiply-high with the cell's magic (exact for i < 2^16)
  {
    const uint32_t magic = 0xFFFFFFFFu / (uint32_t)nd + 1u;
    const uint8_t* gbase = img + (int64_t)(c.wy0 - 3) * pitch + (c.wx0 - 4);
    for (int i = lane; i < th * nd; i += 64) {
      const int r = (int)__umulhi((uint32_t)i, magic), j = i - r * nd;
      const uint8_t* gp = gbase + (int64_t)r * pitch + 4 * j;
      const uint32_t* ap = dev::align_down4(gp);
      const uint32_t d0 = ap[0], d1 = ap[1];
      *reinterpret_cast<uint32_t*>(&tile[r * kFTP + 4 * j]) =
          __builtin_amdgcn_alignbyte(d1, d0, (uint32_t)((uintptr_t)gp & 3));
    }
  }
  for (int i = lane; i < ((ww + 2) * (wh + 2) + 3) / 4; i += 64) reinterpret_cast<uint32_t*>(smap)[i] = 0u;
  dev::wave_sync();

  const int t = a.threshold;
  uint32_t* out = a.slots + (int64_t)f * a.slots_fstride + c.slot_off;
  const int sp = ww + 2;   // smap pitch: one zero ring around the window (NMS needs no bounds)

  // ---- A: compass pre-test of every quad; survivors appended in raster order
  // quad raster position of this lane, advanced by 64 quads per step without divisions
  const int nq1 = max(nq, 1);
  int qy = lane / nq1, qx = lane - qy * nq1;
  const int qdy = 64 / nq1, qdx = 64 - qdy * nq1;
  const uint32_t tt = (uint32_t)t;
  const us2 t2 = as_us2(tt | (tt << 16));
  const int nsteps = (nq * wh + 63) / 64;
  int ns = 0;
  for (int st = 0; st < nsteps; st++) {
    const int y = qy, x = 4 * qx;
    qx += qdx; qy += qdy;
    if (qx >= nq1) { qx -= nq1; qy++; }
    uint32_t pe = 0, po = 0;
    if (y < wh) {
      const uint8_t* p = &tile[(y + 3) * kFTP + x];
      const uint32_t c0 = *reinterpret_cast<const uint32_t*>(p);
      const uint32_t c1 = *reinterpret_cast<const uint32_t*>(p + 4);
      const uint32_t c2 = *reinterpret_cast<const uint32_t*>(p + 8);
      const uint32_t up = *reinterpret_cast<const uint32_t*>(p - 3 * kFTP + 4);   // q8
      const uint32_t dn = *reinterpret_cast<const uint32_t*>(p + 3 * kFTP + 4);   // q0
      const uint32_t rt = __builtin_amdgcn_alignbyte(c2, c1, 3u);                 // q4: x+3..x+6
      const uint32_t lf = __builtin_amdgcn_alignbyte(c1, c0, 1u);                 // q12: x-3..x
      pe = compass2(even_b(c1), even_b(dn), even_b(rt), even_b(up), even_b(lf), t2);
      po = compass2(odd_b(c1), odd_b(dn), odd_b(rt), odd_b(up), odd_b(lf), t2);
    }
    // pixel k of the quad: 0 = pe.lo, 1 = po.lo, 2 = pe.hi, 3 = po.hi (pixels past the row
    // end belong to no window and are dropped)
    const bool s0 = (pe & 0xFFFFu) != 0;
    const bool s1 = (po & 0xFFFFu) != 0 && x + 1 < ww;
    const bool s2 = (pe >> 16) != 0 && x + 2 < ww;
    const bool s3 = (po >> 16) != 0 && x + 3 < ww;
    const uint64_t lt = dev::lanemask_lt();
    const uint64_t b0 = __ballot(s0), b1 = __ballot(s1), b2 = __ballot(s2), b3 = __ballot(s3);
    int pos = ns + __popcll(b0 & lt) + __popcll(b1 & lt) + __popcll(b2 & lt) + __popcll(b3 & lt);
    const int idx = (y << 8) | x;
    if (s0) surv[pos] = (uint16_t)idx;
    pos += s0;
    if (s1) surv[pos] = (uint16_t)(idx + 1);
    pos += s1;
    if (s2) surv[pos] = (uint16_t)(idx + 2);
    pos += s2;
    if (s3) surv[pos] = (uint16_t)(idx + 3);
    ns += __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
  }
  dev::wave_sync();

  // ---- B: exact FAST test + score for the survivors in full 64-lane batches; corners are
  // compacted in place (write index <= read index, reads of a batch precede its writes), so
  // the list stays in raster order
  int ncorner = 0;
  for (int j0 = 0; j0 < ns; j0 += 64) {
    const int j = j0 + lane;
    bool corner = false;
    int idx = 0;
    if (j < ns) {
      idx = surv[j];
      const int y = idx >> 8, x = idx & 0xFF;
      const uint8_t* p = &tile[(y + 3) * kFTP + x + 4];
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
        smap[(y + 1) * sp + x + 1] = (uint8_t)(score + 1);
      }
    }
    const uint64_t bal = __ballot(corner);
    if (corner) surv[ncorner + __popcll(bal & dev::lanemask_lt())] = (uint16_t)idx;
    ncorner += __popcll(bal);
  }
  dev::wave_sync();

  // ---- C: 3x3 NMS on the finished score map (neighbours outside the window count 0: the
  // zero ring) + runByPixelsMask, emitted in raster order
  int count = 0;
  for (int j0 = 0; j0 < ncorner; j0 += 64) {
    const int j = j0 + lane;
    bool keep = false;
    int x = 0, y = 0, s = 0;
    if (j < ncorner) {
      const int pk = surv[j];
      y = pk >> 8; x = pk & 0xFF;
      const uint8_t* m = &smap[(y + 1) * sp + x + 1];
      const int e = m[0];
      s = e - 1;
      // s > max(e_k - 1, 0)  <=>  e > e_k  and  s > 0
      const int mx = max(max(max(m[-sp - 1], m[-sp]), max(m[-sp + 1], m[-1])),
                         max(max(m[1], m[sp - 1]), max(m[sp], m[sp + 1])));
      keep = s > 0 && e > mx;
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
  if (lane == 0) *cnt_out = count;
}

void launch_fast_cells(const FastArgs& a, hipStream_t st) {
  const unsigned g = xcd_grid(a.nframes, (a.ncells + 3) / 4);
  hipLaunchKernelGGL(k_fast_cells, dim3(g), dim3(256), (size_t)4 * a.wave_lds, st, a);
}

}  // namespace mcs
