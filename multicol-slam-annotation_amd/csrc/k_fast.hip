// K2: FAST-9/16 + per-cell 3x3 non-max suppression + runByPixelsMask.  One wave walks a run of
// kCellsPerWave consecutive cells of one frame (four waves per 256-thread workgroup, all of
// a frame's waves on one XCD) and software-pipelines them: while it scores cell k from its
// LDS tile, the tile and mask bitmap of cell k+1 are already in flight into registers.
//
// Reference: ComputeKeyPointsOctTree src/mdBRIEFextractorOct.cpp:874-949, which runs
// FastFeatureDetector(th, nonmax, TYPE_9_16)::detect on every 30 px cell ROI; the OpenCV
// semantics (FAST_t<16>, cornerScore<16>, NMS before the mask) are pinned in SURVEY A.4.
//
// Per cell the wave runs three phases over its LDS tile (window + 3 px halo):
//   A  compass pre-test on every window pixel, 4 pixels per lane: a 9-long arc of the
//      16-circle always holds two ADJACENT compass points (0/4/8/12), so a corner needs
//      (D0|D8)&(D4|D12) or (B0|B8)&(B4|B12) (D = darker than v-t, B = brighter than v+t).
//      The compares are byte-wise: v_lerp_u8(v, ~p, r) = floor((v - p + 255 + r) / 2) per
//      byte is >= K exactly when v - p > t (K = (t + 256 + r) / 2, r = t & 1), and a second
//      lerp against ~(K-1) moves (>= K) into the byte's top bit.  Survivors are compacted in
//      raster order.
//   B  exact test + score for the survivors only, branch-free: with d_k = v - p_k,
//      dark arc  = max_k min(d_k..d_k+8),  bright arc = -min_k max(d_k..d_k+8)
//      (v_min3/v_max3 doubling); corner <=> either > t; score = max(t, dark, bright) - 1,
//      which is exactly cornerScore<16>'s a0/b0 recursion.
//   C  NMS (strict > against the 8 neighbours inside the same window, others count 0) and
//      the mask bit of the pixel (from the cell's prefetched bitmap), compacted in raster
//      order.
#include "common.hpp"
#include "extractor_kernels.hpp"

namespace mcs {

#ifndef MCS_FAST_CPW
#define MCS_FAST_CPW 8
#endif
constexpr int kCellsPerWave = MCS_FAST_CPW;

__device__ __forceinline__ int min3i(int a, int b, int c) { return min(min(a, b), c); }
__device__ __forceinline__ int max3i(int a, int b, int c) { return max(max(a, b), c); }

// Per-wave LDS carve-up, sized on the host from the largest FAST window of the plan (about
// 31 x 31 px for 30 px cells):
//   tile  [th_max][tp]      window + 3 px halo (+3 bytes alignment slack per row)
//   smap  [(ww+2)*(wh+2)]   score + 1 for corners, 0 otherwise (window raster + zero ring)
//   surv  u16[ww*wh]        compass-test survivors (y<<8 | x), then the corners in place
// NT = tile dwords prefetched per lane (>= ceil(tile_dwords / 64)).
#ifndef MCS_FAST_OCC
#define MCS_FAST_OCC 1
#endif
template <int NT>
__global__ __launch_bounds__(256, MCS_FAST_OCC) void k_fast_cells(FastArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_dyn[];
  // the wave index as a scalar: the cell run, its descriptors and every per-cell quantity
  // are wave-uniform (SGPRs and scalar branches)
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int kFTP = a.tile_pitch;
  uint8_t* const tile = lds_dyn + wv * a.wave_lds;
  uint8_t* const smap = tile + a.smap_off;
  uint16_t* const surv = reinterpret_cast<uint16_t*>(tile + a.surv_off);
  int f, item;
  const int runs = (a.ncells + kCellsPerWave - 1) / kCellsPerWave;
  if (!xcd_frame_map(blockIdx.x, a.nframes, (runs + 3) / 4, &f, &item)) return;
  const int run = item * 4 + wv;
  if (run >= runs) return;
  const int c_begin = run * kCellsPerWave, c_end = min(a.ncells, c_begin + kCellsPerWave);
  int32_t* const cnt_out = a.cell_counts + (int64_t)f * a.ncells;
  uint32_t* const outf = a.slots + (int64_t)f * a.slots_fstride;
  const uint64_t* const mbits =
      a.mask_bits ? a.mask_bits + (int64_t)(a.mask_index ? a.mask_index[f] : 0) * a.ncells * kMaskBitRows
                  : nullptr;
  const int t = a.threshold;

  // ---- prefetch of one cell: tile dwords (two aligned loads per 4 tile bytes, merged with
  // alignbyte when written to LDS) and this lane's row of the window's mask bitmap
  uint32_t p0[NT], p1[NT];
  uint32_t mlo = 0xFFFFFFFFu, mhi = 0xFFFFFFFFu;
  auto geom = [&](const CellDesc& c, int& ww, int& wh, int& nd, const uint8_t*& gbase) {
    ww = max(0, c.wx1 - c.wx0); wh = max(0, c.wy1 - c.wy0);
    nd = ((ww + 3) >> 2) + 2;
    const int l = c.level;
    const uint8_t* img = (l == 0) ? a.img0 + (int64_t)f * a.img0_fstride
                                  : a.pyr + (int64_t)f * a.pyr_fstride + a.lp.pyr_off[l];
    gbase = img + (int64_t)(c.wy0 - 3) * a.lp.pitch[l] + (c.wx0 - 4);
  };
  auto prefetch = [&](int ci) {
    const CellDesc c = a.cells[ci];
    int ww, wh, nd;
    const uint8_t* gbase;
    geom(c, ww, wh, nd, gbase);
    const int n = (wh + 6) * nd, pitch = a.lp.pitch[c.level];
    // row = i / nd by a multiply-high with the cell's magic (exact for i < 2^16)
    const uint32_t magic = 0xFFFFFFFFu / (uint32_t)nd + 1u;
#pragma unroll
    for (int k = 0; k < NT; k++) {
      const int i = min(lane + 64 * k, n - 1);
      const int r = (int)__umulhi((uint32_t)i, magic), j = i - r * nd;
      const uint32_t* ap = dev::align_down4(gbase + (int64_t)r * pitch + 4 * j);
      p0[k] = ap[0];
      p1[k] = ap[1];
    }
    if (mbits) {
      const uint32_t* mb = reinterpret_cast<const uint32_t*>(mbits + (int64_t)ci * kMaskBitRows + lane);
      mlo = mb[0];
      mhi = mb[1];
    }
  };

  prefetch(c_begin);
  for (int ci = c_begin; ci < c_end; ci++) {
    const CellDesc c = a.cells[ci];
    int ww, wh, nd;
    const uint8_t* gbase;
    geom(c, ww, wh, nd, gbase);
    const int pitch = a.lp.pitch[c.level];
    const int th = wh + 6;
    // ---- this cell's prefetched tile -> LDS, zero the score map
    dev::wave_sync();
    {
      const int n = th * nd;
      const uint32_t magic = 0xFFFFFFFFu / (uint32_t)nd + 1u;
#pragma unroll
      for (int k = 0; k < NT; k++) {
        const int i = lane + 64 * k;
        if (i < n) {
          const int r = (int)__umulhi((uint32_t)i, magic), j = i - r * nd;
          const uint32_t sh = (uint32_t)((uintptr_t)(gbase + (int64_t)r * pitch + 4 * j) & 3);
          *reinterpret_cast<uint32_t*>(&tile[r * kFTP + 4 * j]) = __builtin_amdgcn_alignbyte(p1[k], p0[k], sh);
        }
      }
    }
    for (int i = lane; i < ((ww + 2) * (wh + 2) + 3) / 4; i += 64) reinterpret_cast<uint32_t*>(smap)[i] = 0u;
    const uint32_t clo = mlo, chi = mhi;
    const bool any_mask = !mbits || __ballot((lane < wh) && ((clo | chi) != 0)) != 0;
    if (ci + 1 < c_end) prefetch(ci + 1);    // in flight while this cell is scored
    if (!any_mask) {   // no usable mask pixel in the window: runByPixelsMask drops everything
      if (lane == 0) cnt_out[ci] = 0;
      continue;
    }
    dev::wave_sync();

    uint32_t* out = outf + c.slot_off;
    const int sp = ww + 2;   // smap pitch: one zero ring around the window (NMS needs no bounds)

    // ---- A: compass pre-test of every quad; survivors appended in raster order
    const int nq = (ww + 3) >> 2;
    const int nq1 = max(nq, 1);
    int qy = lane / nq1, qx = lane - qy * nq1;
    const int qdy = 64 / nq1, qdx = 64 - qdy * nq1;
    const int nsteps = (nq * wh + 63) / 64;
    int ns = 0;
    for (int st = 0; st < nsteps; st++) {
      const int y = qy, x = 4 * qx;
      qx += qdx; qy += qdy;
      if (qx >= nq1) { qx -= nq1; qy++; }
      uint32_t s = 0;
      if (y < wh) {
        const uint8_t* p = &tile[(y + 3) * kFTP + x];
        const uint32_t c0 = *reinterpret_cast<const uint32_t*>(p);
        const uint32_t c1 = *reinterpret_cast<const uint32_t*>(p + 4);
        const uint32_t c2 = *reinterpret_cast<const uint32_t*>(p + 8);
        const uint32_t up = *reinterpret_cast<const uint32_t*>(p - 3 * kFTP + 4);   // q8
        const uint32_t dn = *reinterpret_cast<const uint32_t*>(p + 3 * kFTP + 4);   // q0
        const uint32_t rt = __builtin_amdgcn_alignbyte(c2, c1, 3u);                 // q4: x+3..x+6
        const uint32_t lf = __builtin_amdgcn_alignbyte(c1, c0, 1u);                 // q12: x-3..x
        const uint32_t nv = ~c1;
        auto dk = [&](uint32_t q) {
          return __builtin_amdgcn_lerp(__builtin_amdgcn_lerp(c1, ~q, a.rbits), a.kk, 0u);
        };
        auto bk = [&](uint32_t q) {
          return __builtin_amdgcn_lerp(__builtin_amdgcn_lerp(q, nv, a.rbits), a.kk, 0u);
        };
        s = ((dk(dn) | dk(up)) & (dk(rt) | dk(lf))) | ((bk(dn) | bk(up)) & (bk(rt) | bk(lf)));
      }
      // pixel k of the quad = byte k (pixels past the row end belong to no window)
      const bool s0 = (s & 0x80u) != 0;
      const bool s1 = (s & 0x8000u) != 0 && x + 1 < ww;
      const bool s2 = (s & 0x800000u) != 0 && x + 2 < ww;
      const bool s3 = (s & 0x80000000u) != 0 && x + 3 < ww;
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
        if (corner) smap[(y + 1) * sp + x + 1] = (uint8_t)max(max(t, dark), bright);  // score + 1
      }
      const uint64_t bal = __ballot(corner);
      if (corner) surv[ncorner + __popcll(bal & dev::lanemask_lt())] = (uint16_t)idx;
      ncorner += __popcll(bal);
    }
    dev::wave_sync();

    // ---- C: 3x3 NMS on the finished score map (neighbours outside the window count 0: the
    // zero ring) + runByPixelsMask (window row y's bitmap lives in lane y), raster order
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
      }
      if (mbits) {
        const uint32_t rlo = (uint32_t)__shfl((int)clo, y, 64), rhi = (uint32_t)__shfl((int)chi, y, 64);
        keep = keep && (((x < 32 ? rlo >> x : rhi >> (x - 32)) & 1u) != 0);
      }
      const uint64_t b = __ballot(keep);
      if (keep) {
        const int pos = count + __popcll(b & dev::lanemask_lt());
        out[pos] = (uint32_t)(c.wx0 + x - kMinBorder) | ((uint32_t)(c.wy0 + y - kMinBorder) << 12) |
                   ((uint32_t)s << 24);
      }
      count += __popcll(b);
    }
    if (lane == 0) cnt_out[ci] = count;
  }
}

void launch_fast_cells(const FastArgs& a_in, hipStream_t st) {
  FastArgs a = a_in;
  // byte-wise FAST compare constants (file header); t = 255 admits no corner: K = 256, which
  // no byte reaches, is kk = 0 (the second lerp then never sets a top bit)
  const int t = a.threshold;
  const uint32_t r = (uint32_t)(t & 1), K = (uint32_t)(t + 256 + (int)r) / 2;
  a.rbits = r * 0x01010101u;
  a.kk = (K <= 255 ? (~(K - 1) & 0xFFu) : 0u) * 0x01010101u;
  const int runs = (a.ncells + kCellsPerWave - 1) / kCellsPerWave;
  const unsigned g = xcd_grid(a.nframes, (runs + 3) / 4);
  const size_t lds = (size_t)4 * a.wave_lds;
  if (a.tile_dwords <= 8 * 64)
    hipLaunchKernelGGL(k_fast_cells<8>, dim3(g), dim3(256), lds, st, a);
  else
    hipLaunchKernelGGL(k_fast_cells<20>, dim3(g), dim3(256), lds, st, a);
}

}  // namespace mcs
