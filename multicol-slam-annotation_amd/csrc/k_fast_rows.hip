// K2, row-streaming form: FAST-9/16 + cell-local 3x3 non-max suppression + runByPixelsMask
// over a run of consecutive cells of one cell row (FastUnit), one wave per run.
//
// Reference: ComputeKeyPointsOctTree src/mdBRIEFextractorOct.cpp:874-949, which runs
// FastFeatureDetector(th, nonmax, TYPE_9_16)::detect on every 30 px cell ROI (OpenCV semantics
// of FAST_t<16>, cornerScore<16> and NMS-before-mask pinned in SURVEY A.4).
//
// Why one pass over the run gives the per-cell results: the corner test and cornerScore of a
// pixel read only its 16-circle, never the ROI, and with the one threshold t a corner's score
// max(t, dark, bright) - 1 is max(dark, bright) - 1.  The ROI decides only which neighbours
// take part in the NMS: those inside the same cell's detection window (rows outside it and
// columns across a cell border count as non-corners).  So every pixel is tested once, and
// only the NMS looks at cell borders.
//
// The run is streamed in bands of kBand detection rows:
//   load  the band's new raw rows (one dword per lane, issued one band ahead) enter a
//         register window (rows y0-3 .. y0+kBand+2), and all kBand + 6 rows of that window are
//         written to a linear LDS band window (256 B per row): a survivor's 7 x 7 neighbourhood
//         is then one base address + immediate offsets
//   A     compass pre-test per quad from the register window, 4 pixels per lane, survivors
//         -> list in raster order
//   B     exact test + score of the survivors in full 64-lane batches from the band window:
//         score + 1 into a linear score window (rows y0-2 .. y0+kBand; the two rows above the
//         band are carried over from the previous band), corners compacted in place (raster
//         order)
//   C     NMS of every corner whose lower neighbour row is scored (the band's last row waits
//         for the next band), the mask bit, and the append to the cell's slot list: raster
//         order within a cell, the order OpenCV's FAST emits them in.
#include "common.hpp"
#include "extractor_kernels.hpp"

namespace mcs {

namespace {
#ifndef MCS_FAST_BAND
#define MCS_FAST_BAND 5
#endif
constexpr int kBand = MCS_FAST_BAND;   // detection rows per band (3..8; 5 measured fastest)
static_assert(kBand >= 3 && kBand <= 8, "band height");
// score rows alive at once: the NMS of a band reads rows y0 - 2 .. y1 and the band zeroes
// y0 .. y0 + kBand, so the score window holds rows y0 - 2 .. y0 + kBand
constexpr int kScoreRows = kBand + 3;
// LDS: the four waves' raw band windows (kBand + 6 rows of 256 B), then their score windows,
// then their lists (carried corners, then the band's survivors, compacted in place into its
// corners)
constexpr int kRingBytes = (kBand + 6) * 256, kScoreBytes = kScoreRows * 256;
// a run's detection span is <= 246 px (kFastUnitSpan - 6): <= 246 carried corners + 246 kBand
// survivors
constexpr int kListCap = 248 + kBand * 248;
constexpr int kScoreBase = 4 * kRingBytes, kListBase = kScoreBase + 4 * kScoreBytes;
constexpr int kLdsBytes = kListBase + 4 * 2 * (kListCap + 2);   // + a dummy slot per list

typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
// packed f16 min3 / max3 (v_pk_minimum3_f16 / v_pk_maximum3_f16 on gfx950); all operands are
// integers in [-255, 255] here, exact in f16
__device__ __forceinline__ h2 hmin3(h2 a, h2 b, h2 c) {
  return __builtin_elementwise_minimum(__builtin_elementwise_minimum(a, b), c);
}
__device__ __forceinline__ h2 hmax3(h2 a, h2 b, h2 c) {
  return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}

__device__ __forceinline__ int fr_max3(int a, int b, int c) { return max(max(a, b), c); }

// FAST TYPE_7_12 / TYPE_5_8 of one pixel (OpenCV FAST_t<12> / <8> + cornerScore; restated in
// oracle/extractor_oracle.cpp fast_small): the circle from the ring (pixel e = y << 8 | x),
// the quick test on the SAME pixel pairs as for 16 with wrapped offsets (pixel[k] =
// pixel[k mod P]), a (K+1)-arc with K = P / 2 on the side(s) the quick test left, and
// score + 1 = max(t, best dark arc minimum, best bright arc minimum).  Returns score + 1, or 0.
template <int P>
__device__ __forceinline__ int fast_small(const uint8_t* lds, uint32_t ring_base, int e, int t) {
  // ring_base: LDS byte of pixel (y, x) = ring_base + e (e = y << 8 | x) in the band window
  constexpr int K = P / 2;
  // (dx, dy) of OpenCV's offsets12 / offsets8
  constexpr int c12[12][2] = {{0, 2}, {1, 2}, {2, 1}, {2, 0}, {2, -1}, {1, -2},
                              {0, -2}, {-1, -2}, {-2, -1}, {-2, 0}, {-2, 1}, {-1, 2}};
  constexpr int c8[8][2] = {{0, 1}, {1, 1}, {1, 0}, {1, -1}, {0, -1}, {-1, -1}, {-1, 0}, {-1, 1}};
  auto at = [&](int dx, int dy) -> int {
    return lds[ring_base + (uint32_t)(e + dy * 256 + dx)];
  };
  const int v = at(0, 0);
  int d[P];
#pragma unroll
  for (int k = 0; k < P; k++) d[k] = v - (P == 12 ? at(c12[k][0], c12[k][1]) : at(c8[k % 8][0], c8[k % 8][1]));
  // tab bits: 1 = darker than v - t (d > t), 2 = brighter than v + t (d < -t)
  auto tb = [&](int k) -> int { const int q = d[k % P]; return (q > t ? 1 : 0) | (q < -t ? 2 : 0); };
  const int qd = (tb(0) | tb(8)) & (tb(2) | tb(10)) & (tb(4) | tb(12)) & (tb(6) | tb(14)) &
                 (tb(1) | tb(9)) & (tb(3) | tb(11)) & (tb(5) | tb(13)) & (tb(7) | tb(15));
  int dark = -256, bright = -256;
#pragma unroll
  for (int k = 0; k < P; k++) {
    int mn = d[k], mxv = d[k];
#pragma unroll
    for (int j = 1; j <= K; j++) { mn = min(mn, d[(k + j) % P]); mxv = max(mxv, d[(k + j) % P]); }
    dark = max(dark, mn);
    bright = max(bright, -mxv);
  }
  const bool corner = ((qd & 1) && dark > t) || ((qd & 2) && bright > t);
  return corner ? max(max(t, dark), bright) : 0;
}
}  // namespace

// Tuning probe (tools/gpu/fast_probe.py, variant builds with -DMCS_FAST_PROBE only): shader
// cycles per phase summed over all waves: [0] band loads + ring writes, [1] compass + list,
// [2] exact test + score, [3] NMS + mask + append, [4] whole wave, [5] bands, [6] skipped
// (fully masked) bands, [7] setup before the first band.
#ifdef MCS_FAST_PROBE
__device__ unsigned long long g_fast_probe[8];
#define FP_T(v) const long long v = __builtin_amdgcn_s_memtime()
#define FP_ADD(k, v) (acc_[k] += (unsigned long long)(v))
#else
#define FP_T(v) do { } while (0)
#define FP_ADD(k, v) do { } while (0)
#endif

template <int PAT>
__global__ __launch_bounds__(256) void k_fast_rows(FastRowArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t ring_base = (uint32_t)wv * kRingBytes;
  const uint32_t sc_base = kScoreBase + (uint32_t)wv * kScoreBytes;
  uint32_t* const ring32 = reinterpret_cast<uint32_t*>(lds + ring_base);
  uint8_t* const sc8 = lds + sc_base;
  uint16_t* const list = reinterpret_cast<uint16_t*>(lds + kListBase + wv * 2 * (kListCap + 2));
  // band-relative LDS bases, set per band: pixel e = (y << 8 | x) of the band is raw byte
  // raw_rel + e and score byte sc_rel + e
  uint32_t raw_rel = 0, sc_rel = 0;
  auto sc_at = [&](int e, int dy, int dx) -> uint8_t& {
    return lds[sc_rel + (uint32_t)(e + dy * 256 + dx)];
  };
  int f, item;
  if (!xcd_frame_map(blockIdx.x, a.nframes, (a.nunits + 3) / 4, &f, &item)) return;
  const int ui = item * 4 + wv;
  if (ui >= a.nunits) return;
  // the octree (next launch) adds the frame's keypoint count into frame_count[f]: unit 0 zeroes
  // it on its way out instead of a memset launch between the two.  Only on the way out: a store
  // before the kernel's uniform loads would make them vector loads (the compiler may no longer
  // prove them unclobbered), which cost 0.1 ms per step
  auto zero_count = [&] { if (ui == 0 && lane == 0) a.frame_count[f] = 0; };
  const int mi = a.mask_index ? min(max(a.mask_index[f], 0), a.nmasks - 1) : 0;
  const FastUnit u = a.units[(int64_t)mi * a.unit_mstride + ui];
#ifdef MCS_FAST_PROBE
  unsigned long long acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const long long t_begin_ = __builtin_amdgcn_s_memtime();
#endif
  const int level = u.level, nc = u.ncells, wh = u.wy1 - u.wy0;
  int32_t* const cnt_out = a.cell_counts + (int64_t)f * a.ncells + u.cell0;
  if (wh <= 0) {
    if (lane < nc) cnt_out[lane] = 0;
    zero_count();
    return;
  }
  // mask rows of the run (the level of the frame's mask pyramid, pitch bpitch: aligned dwords)
  const uint8_t* const mrow0 =
      a.mask_pyr ? a.mask_pyr + (int64_t)mi * a.mask_fstride +
                       a.lp.mask_off[level] + (int64_t)(u.wy0 - 3) * a.lp.bpitch[level] + u.xa
                 : nullptr;
  const int mpitch = a.lp.bpitch[level];
  const int t = a.threshold;
  const int xa = u.xa, wc = u.wcell, span = u.ux1 - u.ux0;
  const uint32_t magic = 65536u / (uint32_t)wc + 1u;   // cx / wc for cx < 256, wc <= 64
  const int pitch = a.lp.pitch[level];
  const uint8_t* const img = (level == 0) ? a.img0 + (int64_t)f * a.img0_fstride
                                          : a.pyr + (int64_t)f * a.pyr_fstride + a.lp.pyr_off[level];
  const uint8_t* const row0 = img + (int64_t)(u.wy0 - 3) * pitch + xa;
  // raw rows y_rel in [0, wh + 6); detection rows [3, wh + 3)

  // top bit of byte k: pixel xa + 4 lane + k is a detection pixel of the run
  uint32_t detm = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int x = xa + 4 * lane + k;
    detm |= (x >= u.ux0 && x < u.ux1) ? (0x80u << (8 * k)) : 0u;
  }
  const int slot_off = lane < nc ? a.cells[u.cell0 + lane].slot_off : 0;   // lane k: cell k
  uint32_t* const outf = a.slots + (int64_t)f * a.slots_fstride;
  int cnt = 0;                                                            // lane k: cell k

  // raw row r (y_rel) of the run: one aligned dword per lane, the row's byte offset undone by
  // alignbyte with the next lane's dword (lane 63 is never consumed)
  // No clamping: the last prefetch reaches at most 3 rows past the run's raw rows (row
  // wy1 + 5 <= h - 20 of the level) and mask row wy0 - 1 >= 0, all inside the level.
  auto load_row = [&](int r) -> uint32_t {
    return dev::align_down4(row0 + r * pitch)[lane];
  };
  auto fix_row = [&](int r, uint32_t own) -> uint32_t {
    const uint32_t sh = (uint32_t)((uintptr_t)(row0 + r * pitch) & 3);
    const uint32_t nxt = (uint32_t)__builtin_amdgcn_mov_dpp((int)own, 0x130 /*wave_shl:1*/, 0xF, 0xF, true);
    return __builtin_amdgcn_alignbyte(nxt, own, sh);
  };
  // mask bytes of raw row r (all 0xFF without a mask)
  auto load_mrow = [&](int r) -> uint32_t {
    if (!mrow0) return 0xFFFFFFFFu;
    return reinterpret_cast<const uint32_t*>(mrow0 + r * mpitch)[lane];
  };

  // the score window starts zeroed: rows outside the detection window read as non-corners
#pragma unroll
  for (int i = 0; i < kScoreRows; i++) *reinterpret_cast<uint32_t*>(sc8 + 256 * i + 4 * lane) = 0u;
  // register window: rows y0 - 3 .. y0 + 2 of the current band (the compass reads registers;
  // the exact test reads the ring)
  uint32_t w[6];
#pragma unroll
  for (int i = 0; i < 6; i++) w[i] = load_row(i);
  uint32_t pf[kBand];
#pragma unroll
  for (int i = 0; i < kBand; i++) pf[i] = load_row(6 + i);
  // mask rows y0 - 1 .. y0 + kBand of the current band (m) and the next band's new ones (mpf)
  uint32_t m[kBand + 2], mpf[kBand];
#pragma unroll
  for (int i = 0; i < kBand + 2; i++) m[i] = load_mrow(2 + i);
#pragma unroll
  for (int i = 0; i < kBand; i++) mpf[i] = load_mrow(kBand + 4 + i);
#pragma unroll
  for (int i = 0; i < 6; i++) w[i] = fix_row(i, w[i]);

  const int nbands = (wh + kBand - 1) / kBand;
  int ncarry = 0;   // corners of the previous band's last row, at the front of the list
#ifdef MCS_FAST_PROBE
  FP_ADD(7, __builtin_amdgcn_s_memtime() - t_begin_);
#endif
  for (int b = 0; b < nbands; b++) {
    FP_T(t0_);
    const int y0 = 3 + b * kBand, y1 = min(y0 + kBand, 3 + wh);
    // rows y0 + 3 .. y0 + kBand + 2 arrive; the next band's rows go in flight
    uint32_t rows[6 + kBand];
#pragma unroll
    for (int i = 0; i < 6; i++) rows[i] = w[i];
#pragma unroll
    for (int i = 0; i < kBand; i++) rows[6 + i] = fix_row(y0 + 3 + i, pf[i]);
    if (b > 0) {   // mask rows y0 - 1 .. y0 + kBand
#pragma unroll
      for (int i = 0; i < 2; i++) m[i] = m[kBand + i];
#pragma unroll
      for (int i = 0; i < kBand; i++) m[2 + i] = mpf[i];
    }
    if (b + 1 < nbands) {
#pragma unroll
      for (int i = 0; i < kBand; i++) pf[i] = load_row(y0 + kBand + 3 + i);
#pragma unroll
      for (int i = 0; i < kBand; i++) mpf[i] = load_mrow(y0 + kBand + 1 + i);
    }
#pragma unroll
    for (int i = 0; i < 6; i++) w[i] = rows[kBand + i];
    // the band window: raw rows y0 - 3 .. y0 + kBand + 2 at window rows 0 .. kBand + 5 (the
    // previous band's reads of the window are all done: in-order LDS within the wave)
#pragma unroll
    for (int i = 0; i < kBand + 6; i++) ring32[(i << 6) + lane] = rows[i];
    raw_rel = ring_base - (uint32_t)((y0 - 3) << 8);
    // score window rows y0 - 2 .. y0 + kBand: the previous band's rows y0 - 2, y0 - 1 (its
    // window rows kBand, kBand + 1) move to rows 0, 1; this band's rows and the row below them
    // are zeroed (on the last band that row lies below the detection window and must read 0)
    if (b > 0) {
      const uint32_t c0 = *reinterpret_cast<const uint32_t*>(sc8 + 256 * kBand + 4 * lane);
      const uint32_t c1 = *reinterpret_cast<const uint32_t*>(sc8 + 256 * (kBand + 1) + 4 * lane);
      dev::wave_sync();
      *reinterpret_cast<uint32_t*>(sc8 + 4 * lane) = c0;
      *reinterpret_cast<uint32_t*>(sc8 + 256 + 4 * lane) = c1;
#pragma unroll
      for (int i = 2; i < kScoreRows; i++) *reinterpret_cast<uint32_t*>(sc8 + 256 * i + 4 * lane) = 0u;
    }
    sc_rel = sc_base - (uint32_t)((y0 - 2) << 8);

    // A band whose mask rows y0 - 1 .. y0 + kBand are all zero emits nothing, and nothing it
    // scores is read by an NMS that can emit (the neighbour bands' corners on rows y0 - 1 and
    // y1 are masked out too): skip it, dropping the carried corners.
    {
      uint32_t any = 0;
#pragma unroll
      for (int i = 0; i < kBand + 2; i++) any |= m[i];
      if (__ballot(any != 0) == 0) {
        ncarry = 0;
#ifdef MCS_FAST_PROBE
        FP_ADD(6, __builtin_amdgcn_s_memtime() - t0_);
#endif
        continue;
      }
    }

    FP_T(t1_);
    FP_ADD(0, t1_ - t0_);
    FP_ADD(5, 1);
    // ---- A: compass pre-test from the register window, 4 pixels per lane: a 9-long arc of the
    // 16-circle always holds two ADJACENT compass points (0/4/8/12), so a corner needs
    // (D0|D8)&(D4|D12) or (B0|B8)&(B4|B12) (D = darker than v-t, B = brighter than v+t), tested
    // byte-wise with v_lerp_u8 (launch_fast_rows); survivors
    // appended after the carried corners in raster order
    int ns = 0;
    const uint64_t lt = dev::lanemask_lt();
    uint32_t sv[kBand];
#pragma unroll
    for (int i = 0; i < kBand; i++) {
      const int y = y0 + i;
      const uint32_t c1 = rows[i + 3], up = rows[i] /* q8 */, dn = rows[i + 6] /* q0 */;
      const uint32_t L = (uint32_t)__builtin_amdgcn_mov_dpp((int)c1, 0x138 /*wave_shr:1*/, 0xF, 0xF, true);
      const uint32_t R = (uint32_t)__builtin_amdgcn_mov_dpp((int)c1, 0x130 /*wave_shl:1*/, 0xF, 0xF, true);
      const uint32_t rt = __builtin_amdgcn_alignbyte(R, c1, 3u);   // q4: x+3..x+6
      const uint32_t lf = __builtin_amdgcn_alignbyte(c1, L, 1u);   // q12: x-3..x
      const uint32_t nv = ~c1;
      auto dk = [&](uint32_t q) { return __builtin_amdgcn_lerp(__builtin_amdgcn_lerp(c1, ~q, a.rbits), a.kk, 0u); };
      auto bk = [&](uint32_t q) { return __builtin_amdgcn_lerp(__builtin_amdgcn_lerp(q, nv, a.rbits), a.kk, 0u); };
      // 12 / 8 point circles: no pre-test, every detection pixel goes to the exact test
      sv[i] = (y >= y1) ? 0u
              : PAT != 16 ? detm
                          : ((((dk(dn) | dk(up)) & (dk(rt) | dk(lf))) |
                              ((bk(dn) | bk(up)) & (bk(rt) | bk(lf)))) & detm);
    }
    // compaction: the lane's exclusive prefix of its survivor counts (0..4 per row) by DPP
    // scans, three rows per scan in 10-bit fields (a row's wave total is <= 62 x 4 = 248, so
    // no field carries into the next; one scan per row measured 0.652 against 0.638 ms per
    // step); the four entries per row are written unconditionally, those of non-survivors to a
    // dummy slot
    constexpr int kNP = (kBand + 2) / 3;
    uint32_t pc[kNP], px[kNP], ptot[kNP];
#pragma unroll
    for (int q = 0; q < kNP; q++) pc[q] = 0u;
#pragma unroll
    for (int i = 0; i < kBand; i++) pc[i / 3] |= (uint32_t)__builtin_popcount(sv[i]) << (10 * (i % 3));
#pragma unroll
    for (int q = 0; q < kNP; q++) {
      const uint32_t inc = (uint32_t)dev::wave_incl_scan((int)pc[q]);
      px[q] = inc - pc[q];                               // exclusive, field by field (no borrows)
      ptot[q] = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    }
#pragma unroll
    for (int i = 0; i < kBand; i++) {
      const int y = y0 + i;
      const uint32_t s = sv[i];
      const int pos0 = ncarry + ns + (int)((px[i / 3] >> (10 * (i % 3))) & 0x3FFu);
      ns += (int)((ptot[i / 3] >> (10 * (i % 3))) & 0x3FFu);
      const int k0 = (s >> 7) & 1, k1 = (s >> 15) & 1, k2 = (s >> 23) & 1, k3 = s >> 31;
      const int pos1 = pos0 + k0, pos2 = pos1 + k1, pos3 = pos2 + k2;
      const int idx = (y << 8) | (4 * lane);
      list[k0 ? pos0 : kListCap] = (uint16_t)idx;
      list[k1 ? pos1 : kListCap] = (uint16_t)(idx + 1);
      list[k2 ? pos2 : kListCap] = (uint16_t)(idx + 2);
      list[k3 ? pos3 : kListCap] = (uint16_t)(idx + 3);
    }
    dev::wave_sync();
    FP_T(t2_);
    FP_ADD(1, t2_ - t1_);

    // ---- B: exact FAST test + score of the survivors, two per lane (batch j0: survivors
    // j0 + lane and j0 + 64 + lane in the low / high halves).  With d_k = v - p_k, cornerScore's
    // darkest 9-arc max_k min(d_k..d_k+8) is v - min_k max(p_k..p_k+8) and the brightest
    // max_k min(p_k..p_k+8) - v; both extrema run on the raw pixel pairs as f16 bit patterns
    // (0..255 are f16 denormals, ordered like the integers; the kernel keeps f16 denormals) by
    // packed min3/max3 doubling.  corner <=> dark > t or bright > t, score + 1 =
    // max(t, dark, bright).  Corners are compacted in place behind the carried ones (write
    // index <= read index, all reads of a batch precede its writes): raster order is kept.
    int ncorn = ncarry, nlast = 0;   // nlast: corners on the band's last row
    if (PAT != 16) {
      for (int j0 = 0; j0 < ns; j0 += 64) {
        const int ja = j0 + lane;
        const int ea = list[ncarry + min(ja, ns - 1)];
        const int s1 = fast_small<PAT == 16 ? 12 : PAT>(lds, raw_rel, ea, t);
        const bool ca = ja < ns && s1 > 0;
        if (ca) sc_at(ea, 0, 0) = (uint8_t)s1;
        const uint64_t bal_a = __ballot(ca);
        // every read of this batch precedes its writes (ja >= write index)
        if (ca) list[ncorn + __popcll(bal_a & lt)] = (uint16_t)ea;
        ncorn += __popcll(bal_a);
        nlast += __popcll(__ballot(ca && (ea >> 8) == y1 - 1));
      }
    }
    for (int j0 = 0; PAT == 16 && j0 < ns; j0 += 128) {
      const int ja = j0 + lane, jb = j0 + 64 + lane;
      const int ea = list[ncarry + min(ja, ns - 1)], eb = list[ncarry + min(jb, ns - 1)];
      // band-window bytes of both survivors' (y - 3, x - 3): the 7 x 7 neighbourhood is at
      // immediate offsets from them
      const uint8_t* const pa0 = lds + (raw_rel + (uint32_t)ea - 3u * 256u - 3u);
      const uint8_t* const pb0 = lds + (raw_rel + (uint32_t)eb - 3u * 256u - 3u);
      auto pix = [&](int dy, int dx) -> h2 {
        const uint32_t pa = pa0[(dy + 3) * 256 + dx + 3], pb = pb0[(dy + 3) * 256 + dx + 3];
        return __builtin_bit_cast(h2, pa | (pb << 16));
      };
      h2 p[16];
      // circle (dx,dy): (0,3),(1,3),(2,2),(3,1),(3,0),(3,-1),(2,-2),(1,-3),(0,-3),(-1,-3),
      //                 (-2,-2),(-3,-1),(-3,0),(-3,1),(-2,2),(-1,3)
      p[0] = pix(3, 0);   p[1] = pix(3, 1);   p[2] = pix(2, 2);   p[3] = pix(1, 3);
      p[4] = pix(0, 3);   p[5] = pix(-1, 3);  p[6] = pix(-2, 2);  p[7] = pix(-3, 1);
      p[8] = pix(-3, 0);  p[9] = pix(-3, -1); p[10] = pix(-2, -2); p[11] = pix(-1, -3);
      p[12] = pix(0, -3); p[13] = pix(1, -3); p[14] = pix(2, -2); p[15] = pix(3, -1);
      const int va = pa0[3 * 256 + 3], vb = pb0[3 * 256 + 3];
      h2 mx[16], mn[16];
#pragma unroll
      for (int k = 0; k < 16; k++) {
        mx[k] = hmax3(p[k], p[(k + 1) & 15], p[(k + 2) & 15]);
        mn[k] = hmin3(p[k], p[(k + 1) & 15], p[(k + 2) & 15]);
      }
      h2 amx[16], amn[16];   // max / min over the 9-arc starting at k
#pragma unroll
      for (int k = 0; k < 16; k++) {
        amx[k] = hmax3(mx[k], mx[(k + 3) & 15], mx[(k + 6) & 15]);
        amn[k] = hmin3(mn[k], mn[(k + 3) & 15], mn[(k + 6) & 15]);
      }
#pragma unroll
      for (int n = 16; n > 1; n = (n + 2) / 3) {   // 16 -> 6 -> 2 -> 1: min_k amx, max_k amn
#pragma unroll
        for (int k = 0; k < (n + 2) / 3; k++) {
          const h2 x1 = amx[3 * k], y1v = amn[3 * k];
          const h2 x2 = 3 * k + 1 < n ? amx[3 * k + 1] : x1, y2 = 3 * k + 1 < n ? amn[3 * k + 1] : y1v;
          const h2 x3 = 3 * k + 2 < n ? amx[3 * k + 2] : x1, y3 = 3 * k + 2 < n ? amn[3 * k + 2] : y1v;
          amx[k] = hmin3(x1, x2, x3);
          amn[k] = hmax3(y1v, y2, y3);
        }
      }
      const uint32_t bmx = __builtin_bit_cast(uint32_t, amx[0]), bmn = __builtin_bit_cast(uint32_t, amn[0]);
      const int dark_a = va - (int)(bmx & 0xFFFFu), dark_b = vb - (int)(bmx >> 16);
      const int bright_a = (int)(bmn & 0xFFFFu) - va, bright_b = (int)(bmn >> 16) - vb;
      const bool ca = ja < ns && (dark_a > t || bright_a > t);
      const bool cb = jb < ns && (dark_b > t || bright_b > t);
      if (ca) sc_at(ea, 0, 0) = (uint8_t)max(max(t, dark_a), bright_a);   // score + 1
      if (cb) sc_at(eb, 0, 0) = (uint8_t)max(max(t, dark_b), bright_b);
      const uint64_t bal_a = __ballot(ca);
      if (ca) list[ncorn + __popcll(bal_a & lt)] = (uint16_t)ea;
      ncorn += __popcll(bal_a);
      const uint64_t bal_b = __ballot(cb);
      if (cb) list[ncorn + __popcll(bal_b & lt)] = (uint16_t)eb;
      ncorn += __popcll(bal_b);
      nlast += __popcll(__ballot(ca && (ea >> 8) == y1 - 1)) + __popcll(__ballot(cb && (eb >> 8) == y1 - 1));
    }
    dev::wave_sync();
    FP_T(t3_);
    FP_ADD(2, t3_ - t2_);

    // ---- C: NMS (3x3 within the cell) + runByPixelsMask + append to the cell's slots
    const bool last_band = b + 1 == nbands;
    const int nproc = last_band ? ncorn : ncorn - nlast;
    for (int j0 = 0; j0 < nproc; j0 += 64) {
      const int j = j0 + lane;
      bool keep = false;
      int k = 0;
      uint32_t rec = 0;
      if (j < nproc) {
        const int e = list[j], y = e >> 8, x = e & 0xFF;
        const int cx = xa + x - u.ux0;
        k = (int)(((uint32_t)cx * magic) >> 16);
        const int cs = k * wc, ce = min(cs + wc, span);
        auto sv = [&](int dy, int dx) -> int { return sc_at(e, dy, dx); };
        const int e0 = sv(0, 0);
        int mx = max(sv(-1, 0), sv(1, 0));
        if (cx > cs) mx = max(mx, fr_max3(sv(-1, -1), sv(0, -1), sv(1, -1)));
        if (cx + 1 < ce) mx = max(mx, fr_max3(sv(-1, 1), sv(0, 1), sv(1, 1)));
        keep = e0 >= 2 && e0 > mx;   // score > 0 and > every in-cell neighbour's score
        rec = (uint32_t)(xa + x - kMinBorder) | ((uint32_t)(u.wy0 + y - 3 - kMinBorder) << 12) |
              ((uint32_t)(e0 - 1) << 24);
      }
      // runByPixelsMask: the mask byte of (y, x) from the lane holding column x of mask row y
      // (row y - (y0 - 1) of the register window m)
      {
        const int e = list[min(j, nproc - 1)];
        const int ri = ((e >> 8) & 0x7F) - (y0 - 1), x = e & 0xFF;
        uint32_t mw = 0;
#pragma unroll
        for (int i = 0; i <= kBand; i++) {
          const uint32_t mi = (uint32_t)__builtin_amdgcn_ds_bpermute((x >> 2) << 2, (int)m[i]);
          mw = ri == i ? mi : mw;
        }
        keep = keep && ((mw >> (8 * (x & 3))) & 0xFFu) != 0;
      }
      uint64_t bk = __ballot(keep);
      while (bk) {   // one pass per distinct cell among the batch's keypoints
        const int kc = __builtin_amdgcn_readlane(k, (int)__builtin_ctzll(bk));
        const bool mine = keep && k == kc;
        const uint64_t bm = __ballot(mine);
        const int base = __builtin_amdgcn_readlane(cnt, kc) + __builtin_amdgcn_readlane(slot_off, kc);
        if (mine) outf[base + __popcll(bm & lt)] = rec;
        if (lane == kc) cnt += __popcll(bm);
        bk &= ~bm;
      }
    }
    ncarry = 0;
    if (!last_band && nlast > 0) {   // the band's last-row corners move to the front
      uint32_t v[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int jj = lane + 64 * i;
        v[i] = jj < nlast ? list[nproc + jj] : 0u;
      }
      dev::wave_sync();
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int jj = lane + 64 * i;
        if (jj < nlast) list[jj] = (uint16_t)v[i];
      }
      ncarry = nlast;
    }
    dev::wave_sync();
    FP_T(t4_);
    FP_ADD(3, t4_ - t3_);
  }
  if (lane < nc) cnt_out[lane] = cnt;
  zero_count();
#ifdef MCS_FAST_PROBE
  acc_[4] += (unsigned long long)(__builtin_amdgcn_s_memtime() - t_begin_);
  if (lane == 0)
    for (int k = 0; k < 8; k++) atomicAdd(&g_fast_probe[k], acc_[k]);
#endif
}

#ifdef MCS_FAST_PROBE
extern "C" int mcs_debug_fast_probe(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fast_probe), sizeof(g_fast_probe)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_fast_probe), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

void launch_fast_rows(const FastRowArgs& a_in, hipStream_t st) {
  // (pattern 12 / 8: the compare constants are unused)
  FastRowArgs a = a_in;
  // byte-wise compare constants of the compass pre-test: v_lerp_u8(v, ~p, r) =
  // floor((v - p + 255 + r) / 2) per byte is >= K exactly when v - p > t (K = (t + 256 + r) / 2,
  // r = t & 1), and a second lerp against ~(K-1) moves (>= K) into the byte's top bit; t = 255
  // admits no corner: K = 256, which no byte reaches, is kk = 0
  const int t = a.threshold;
  const uint32_t r = (uint32_t)(t & 1), K = (uint32_t)(t + 256 + (int)r) / 2;
  a.rbits = r * 0x01010101u;
  a.kk = (K <= 255 ? (~(K - 1) & 0xFFu) : 0u) * 0x01010101u;
  const unsigned g = xcd_grid(a.nframes, (a.nunits + 3) / 4);
  if (a.pattern == 12) hipLaunchKernelGGL(k_fast_rows<12>, dim3(g), dim3(256), 0, st, a);
  else if (a.pattern == 8) hipLaunchKernelGGL(k_fast_rows<8>, dim3(g), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(k_fast_rows<16>, dim3(g), dim3(256), 0, st, a);
}

}  // namespace mcs
