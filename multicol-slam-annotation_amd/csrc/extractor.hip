// MI355X (gfx950) feature extractor: pyramid -> blur -> FAST cells -> octree ->
// orientation + rotated BRIEF, batched over many camera-frames resident in HBM.
//
// Reference path (billamiable/MultiCol-SLAM-Annotation):
//   mdBRIEFextractorOct::operator()        src/mdBRIEFextractorOct.cpp:1244-1337
//   ComputePyramid                         :1158-1201   -> k_resize_linear, k_mask_nearest
//   ComputeKeyPointsOctTree (FAST part)    :863-949     -> k_fast_cells
//   DistributeOctTree / DivideNode         :569-861     -> k_octree
//   computeOrientation / IC_Angle          :221-248     -> k_orient_desc (part 1)
//   boxFilter 5x5                          :1301        -> k_blur5
//   compute_ORB / rotatePattern            :285-354     -> k_orient_desc (part 2)
// OpenCV semantics the reference delegates to are pinned in SURVEY.md Appendix A; the
// CPU restatement in oracle/ follows the same pins.  Compiled with -ffp-contract=off:
// fastAtan2 and the pattern rotation must not fuse multiply-adds.
#include "common.hpp"
#include "extractor_plan.hpp"
#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

namespace mcs {

__constant__ int c_pattern[2048] = {
#include "pattern_orb64.inc"
};
__constant__ int c_umax[kHalfPatch + 1];

// ===========================================================================
// K1: cv::resize INTER_LINEAR 8U, level l-1 -> level l
// One thread per output pixel; 64x4 threads per block; blockIdx.z = frame.
// ===========================================================================
__global__ __launch_bounds__(256) void k_resize_linear(
    const uint8_t* __restrict__ src, int64_t src_fstride, int sw, int sh,
    uint8_t* __restrict__ dst, int64_t dst_fstride, int dw, int dh,
    const int32_t* __restrict__ xofs, const int16_t* __restrict__ alpha,
    const int32_t* __restrict__ yofs, const int16_t* __restrict__ beta, int simd_end) {
  const int dx = blockIdx.x * 64 + (threadIdx.x & 63);
  const int dy = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (dx >= dw || dy >= dh) return;
  const uint8_t* S = src + (int64_t)blockIdx.z * src_fstride;
  const int sx = xofs[dx];
  const int sx1 = min(sx + 1, sw - 1);
  const int a0 = alpha[2 * dx], a1 = alpha[2 * dx + 1];
  const int sy = yofs[dy];
  const int r0 = sy < 0 ? 0 : (sy < sh ? sy : sh - 1);
  const int r1 = sy + 1 < 0 ? 0 : (sy + 1 < sh ? sy + 1 : sh - 1);
  const int s0 = S[(int64_t)r0 * sw + sx] * a0 + S[(int64_t)r0 * sw + sx1] * a1;
  const int s1 = S[(int64_t)r1 * sw + sx] * a0 + S[(int64_t)r1 * sw + sx1] * a1;
  const int b0 = beta[2 * dy], b1 = beta[2 * dy + 1];
  int v;
  if (dx < simd_end) {
    // OpenCV 3.1 SSE2 VResizeLinearVec_32s8u: packs(S>>4), mulhi by beta, adds, +2, >>2
    const int x0 = max(-32768, min(32767, s0 >> 4));
    const int y0 = max(-32768, min(32767, s1 >> 4));
    int t = ((x0 * b0) >> 16) + ((y0 * b1) >> 16);
    t = max(-32768, min(32767, t));
    t = max(-32768, min(32767, t + 2));
    v = t >> 2;
  } else {
    v = (s0 * b0 + s1 * b1 + (1 << 21)) >> 22;  // FixedPtCast<int,uchar,22>
  }
  dst[(int64_t)blockIdx.z * dst_fstride + (int64_t)dy * dw + dx] = (uint8_t)max(0, min(255, v));
}

// cv::resize INTER_NEAREST for the mask pyramid
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

// ===========================================================================
// K5: boxFilter 5x5 normalized, BORDER_REFLECT_101: round(sum/25)
// ===========================================================================
__device__ __forceinline__ int reflect101(int p, int n) {
  p = p < 0 ? -p : p;
  return p >= n ? 2 * n - 2 - p : p;
}

__global__ __launch_bounds__(256) void k_blur5(const uint8_t* __restrict__ src, int64_t sfs,
                                               uint8_t* __restrict__ dst, int64_t dfs, int w,
                                               int h) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (x >= w || y >= h) return;
  const uint8_t* S = src + (int64_t)blockIdx.z * sfs;
  int s = 0;
  if (x >= 2 && x < w - 2 && y >= 2 && y < h - 2) {
#pragma unroll
    for (int dy = -2; dy <= 2; dy++) {
      const uint8_t* r = S + (int64_t)(y + dy) * w + x;
      s += r[-2] + r[-1] + r[0] + r[1] + r[2];
    }
  } else {
    for (int dy = -2; dy <= 2; dy++)
      for (int dx = -2; dx <= 2; dx++)
        s += S[(int64_t)reflect101(y + dy, h) * w + reflect101(x + dx, w)];
  }
  dst[(int64_t)blockIdx.z * dfs + (int64_t)y * w + x] = (uint8_t)((2 * s + 25) / 50);
}

// ===========================================================================
// K2: FAST-9/16 + cell-local 3x3 NMS + runByPixelsMask, one wave per FAST cell
// (ComputeKeyPointsOctTree :892-948 with OpenCV FAST_t<16> semantics).
// Survivors are written in reference order (row-major inside the cell) as packed
// (x_rel | y_rel << 12 | score << 24), x_rel/y_rel relative to minBorder = 22.
// ===========================================================================
struct FastArgs {
  const uint8_t* img0;  int64_t img0_fstride;   // level 0 frames
  const uint8_t* pyr;   int64_t pyr_fstride;    // levels >= 1
  const uint8_t* mask_pyr; int64_t mask_fstride; // registered mask pyramids (nullable)
  const int32_t* mask_index;                    // per-frame mask id (nullable -> 0)
  const CellDesc* cells; int ncells;
  uint32_t* slots; int64_t slots_fstride;
  int32_t* cell_counts;
  int threshold;
  int32_t lw[kMaxLevels], lh[kMaxLevels];
  int64_t lpyr_off[kMaxLevels], limg_off[kMaxLevels];
};

__device__ __forceinline__ bool has_run9(uint32_t m) {
  m |= m << 16;
  uint32_t a = m & (m >> 1);
  a &= a >> 2;
  a &= a >> 4;
  a &= m >> 8;
  return (a & 0xFFFFu) != 0;
}

constexpr int kTile = kMaxCellDim + 6;

__global__ __launch_bounds__(64) void k_fast_cells(FastArgs a) {
  __shared__ uint8_t tile[kTile * kTile];
  __shared__ uint16_t sc[kMaxCellDim * kMaxCellDim];  // bit 8: corner, low 8 bits: score
  const int ci = blockIdx.x, f = blockIdx.y, lane = threadIdx.x;
  const CellDesc c = a.cells[ci];
  const int l = c.level, w = a.lw[l];
  const uint8_t* img = (l == 0) ? a.img0 + (int64_t)f * a.img0_fstride
                                : a.pyr + (int64_t)f * a.pyr_fstride + a.lpyr_off[l];
  const int ww = max(0, c.wx1 - c.wx0), wh = max(0, c.wy1 - c.wy0);
  const int tw = ww + 6, th = wh + 6;
  // stage the cell ROI (+3 halo) in LDS
  for (int i = lane; i < tw * th; i += 64) {
    const int ty = i / tw, tx = i - ty * tw;
    tile[ty * tw + tx] = img[(int64_t)(c.wy0 - 3 + ty) * w + (c.wx0 - 3 + tx)];
  }
  __syncthreads();
  const int t = a.threshold;
  // circle offsets (x, y) of FAST_t<16> makeOffsets
  const int ox[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
  const int oy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
  for (int i = lane; i < ww * wh; i += 64) {
    const int y = i / ww, x = i - y * ww;
    const uint8_t* p = tile + (y + 3) * tw + (x + 3);
    const int v = p[0];
    int cir[16];
#pragma unroll
    for (int k = 0; k < 16; k++) cir[k] = p[oy[k] * tw + ox[k]];
    uint32_t dark = 0, bright = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      dark |= (uint32_t)(cir[k] < v - t) << k;
      bright |= (uint32_t)(cir[k] > v + t) << k;
    }
    uint16_t out = 0;
    if (has_run9(dark) || has_run9(bright)) {
      // cornerScore<16>
      int d[25];
#pragma unroll
      for (int k = 0; k < 25; k++) d[k] = v - cir[k & 15];
      int a0 = t;
#pragma unroll
      for (int k = 0; k < 16; k += 2) {
        int m = min(d[k + 1], d[k + 2]);
        m = min(m, d[k + 3]); m = min(m, d[k + 4]); m = min(m, d[k + 5]);
        m = min(m, d[k + 6]); m = min(m, d[k + 7]); m = min(m, d[k + 8]);
        a0 = max(a0, min(m, d[k]));
        a0 = max(a0, min(m, d[k + 9]));
      }
      int b0 = -a0;
#pragma unroll
      for (int k = 0; k < 16; k += 2) {
        int m = max(d[k + 1], d[k + 2]);
        m = max(m, d[k + 3]); m = max(m, d[k + 4]); m = max(m, d[k + 5]);
        m = max(m, d[k + 6]); m = max(m, d[k + 7]); m = max(m, d[k + 8]);
        b0 = min(b0, max(m, d[k]));
        b0 = min(b0, max(m, d[k + 9]));
      }
      out = (uint16_t)(0x100 | ((-b0 - 1) & 0xFF));
    }
    sc[y * ww + x] = out;
  }
  __syncthreads();
  // NMS inside the window + mask + ordered compaction
  const uint8_t* mask = nullptr;
  if (a.mask_pyr) {
    const int mi = a.mask_index ? a.mask_index[f] : 0;
    mask = a.mask_pyr + (int64_t)mi * a.mask_fstride + a.limg_off[l];
  }
  uint32_t* out = a.slots + (int64_t)f * a.slots_fstride + c.slot_off;
  int count = 0;
  for (int base = 0; base < ww * wh; base += 64) {
    const int i = base + lane;
    bool keep = false;
    int s = 0, x = 0, y = 0;
    if (i < ww * wh) {
      y = i / ww; x = i - y * ww;
      const uint16_t v = sc[i];
      if (v & 0x100) {
        s = v & 0xFF;
        keep = true;
#pragma unroll
        for (int dy = -1; dy <= 1; dy++)
#pragma unroll
          for (int dx = -1; dx <= 1; dx++) {
            if (dx == 0 && dy == 0) continue;
            const int xx = x + dx, yy = y + dy;
            const int ns = (xx >= 0 && xx < ww && yy >= 0 && yy < wh) ? (sc[yy * ww + xx] & 0xFF) : 0;
            keep = keep && (s > ns);
          }
        if (keep && mask) keep = mask[(int64_t)(c.wy0 + y) * w + (c.wx0 + x)] != 0;
      }
    }
    const uint64_t b = __ballot(keep);
    if (keep) {
      const int pos = count + __popcll(b & dev::lanemask_lt());
      const uint32_t xr = (uint32_t)(c.wx0 + x - kMinBorder), yr = (uint32_t)(c.wy0 + y - kMinBorder);
      out[pos] = xr | (yr << 12) | ((uint32_t)s << 24);
    }
    count += __popcll(b);
  }
  if (lane == 0) a.cell_counts[(int64_t)f * a.ncells + ci] = count;
}

// ===========================================================================
// K3: DistributeOctTree as a data-parallel, order-exact emulation, one workgroup per
// (frame, level).  See DESIGN.md "octree".  The std::list order of the reference is
// reproduced exactly: children are pushed to the front in (node order, n1..n4) order,
// untouched nodes keep their relative order; final-phase node choice follows
// sort(size, pointer) with pointer order pinned to creation order.
// ===========================================================================
struct OctArgs {
  LevelPlan lv[kMaxLevels];
  const CellDesc* cells;
  const int32_t* cell_counts; int ncells;
  const uint32_t* slots; int64_t slots_fstride;
  uint32_t* cand; int32_t* cnode; int64_t cand_fstride;
  uint32_t* sel; int64_t sel_fstride;
  int32_t* sel_count; int nlevels;
  int32_t* frame_count;
};

constexpr int kOctThreads = 256;
constexpr int kOctPer = kOctMaxL / kOctThreads;  // nodes per thread in node scans

__device__ __forceinline__ int oct_quad(uint32_t pk, int midx, int midy) {
  const int x = pk & 0xFFF, y = (pk >> 12) & 0xFFF;
  return (x >= midx ? 1 : 0) + (y >= midy ? 2 : 0);
}

__global__ __launch_bounds__(kOctThreads) void k_octree(OctArgs a) {
  const int l = blockIdx.x, f = blockIdx.y, tid = threadIdx.x;
  const LevelPlan& L = a.lv[l];
  __shared__ int s_pref[kMaxCellsPerLevel];  // cell prefix; reused as sort keys
  __shared__ int s_scan[kOctThreads / 64 + 1];
  __shared__ int16_t nx0[2][kOctMaxL], ny0[2][kOctMaxL], nx1[2][kOctMaxL], ny1[2][kOctMaxL];
  __shared__ int ncnt[2][kOctMaxL], nseq[2][kOctMaxL];
  __shared__ int ccnt[kOctMaxL * 4];  // child counts; reused for best keys
  __shared__ int npos[kOctMaxL * 4];  // new position per (node, child); kept uses slot 0
  __shared__ int nflag[kOctMaxL];     // expanding / in-E / processed flags
  __shared__ int s_var[8];

  uint32_t* cand = a.cand + (int64_t)f * a.cand_fstride + L.cand_off;
  int32_t* cnode = a.cnode + (int64_t)f * a.cand_fstride + L.cand_off;
  const uint32_t* slots = a.slots + (int64_t)f * a.slots_fstride;
  const int32_t* counts = a.cell_counts + (int64_t)f * a.ncells + L.cell_begin;
  const int nc = L.cell_end - L.cell_begin;
  const int N = L.nfeat;

  // ---- 1. gather candidates of this level in reference (cell, row, col) order
  int n = 0;
  for (int base = 0; base < nc; base += kOctThreads) {
    const int i = base + tid;
    const int v = i < nc ? counts[i] : 0;
    int tot;
    const int ex = dev::block_excl_scan<kOctThreads>(v, s_scan, &tot);
    if (i < nc) s_pref[i] = n + ex;
    n += tot;
  }
  __syncthreads();
  {
    const int wv = tid >> 6, lane = tid & 63;
    for (int c = wv; c < nc; c += kOctThreads / 64) {
      const int cnt = counts[c];
      const uint32_t* src = slots + a.cells[L.cell_begin + c].slot_off;
      const int dst = s_pref[c];
      for (int k = lane; k < cnt; k += 64) cand[dst + k] = src[k];
    }
  }
  __syncthreads();

  // ---- 2. initial nodes (:650-683)
  const int nIni = L.nini;
  int cur = 0;
  if (tid < nIni) {
    nx0[0][tid] = (int16_t)(int)(L.hx * (double)tid);
    nx1[0][tid] = (int16_t)(int)(L.hx * (double)(tid + 1));
    ny0[0][tid] = 0;
    ny1[0][tid] = (int16_t)L.height_rel;
    ncnt[0][tid] = 0;
    nseq[0][tid] = tid;
  }
  __syncthreads();
  for (int k = tid; k < n; k += kOctThreads) {
    const int x = cand[k] & 0xFFF;
    const int node = (int)((double)(float)x / L.hx);
    cnode[k] = node;
    atomicAdd(&ncnt[0][node], 1);
  }
  __syncthreads();
  if (tid == 0) {  // erase empty initial nodes, keep order
    int m = 0;
    for (int i = 0; i < nIni; i++) {
      if (ncnt[0][i] > 0) {
        nx0[1][m] = nx0[0][i]; ny0[1][m] = ny0[0][i]; nx1[1][m] = nx1[0][i]; ny1[1][m] = ny1[0][i];
        ncnt[1][m] = ncnt[0][i]; nseq[1][m] = nseq[0][i];
        npos[i] = m++;
      }
    }
    s_var[0] = m;
  }
  __syncthreads();
  for (int k = tid; k < n; k += kOctThreads) cnode[k] = npos[cnode[k]];
  cur = 1;
  int Lsz = s_var[0];
  int seqc = nIni;
  __syncthreads();

  // ---- 3. main subdivision loop (:692-837)
  bool finished = false;
  int lastPushBase = 0;
  while (true) {
    const int prevSize = Lsz;
    const int nxt = cur ^ 1;
    for (int i = tid; i < Lsz; i += kOctThreads) {
      nflag[i] = ncnt[cur][i] > 1;
      ccnt[4 * i] = ccnt[4 * i + 1] = ccnt[4 * i + 2] = ccnt[4 * i + 3] = 0;
    }
    __syncthreads();
    for (int k = tid; k < n; k += kOctThreads) {
      const int nd = cnode[k];
      if (nflag[nd]) {
        const int midx = nx0[cur][nd] + ((nx1[cur][nd] - nx0[cur][nd] + 1) >> 1);
        const int midy = ny0[cur][nd] + ((ny1[cur][nd] - ny0[cur][nd] + 1) >> 1);
        atomicAdd(&ccnt[4 * nd + oct_quad(cand[k], midx, midy)], 1);
      }
    }
    __syncthreads();
    // per thread: kOctPer consecutive nodes -> pushes (expanding) / kept
    int pushes = 0, kept = 0, expandKids = 0;
    const int i0 = tid * kOctPer;
    for (int j = 0; j < kOctPer; j++) {
      const int i = i0 + j;
      if (i >= Lsz) break;
      if (nflag[i]) {
        for (int q = 0; q < 4; q++) {
          const int cq = ccnt[4 * i + q];
          pushes += cq > 0;
          expandKids += cq > 1;
        }
      } else {
        kept++;
      }
    }
    int P, K, E2;
    const int pushBase = dev::block_excl_scan<kOctThreads>(pushes, s_scan, &P);
    const int keptBase = dev::block_excl_scan<kOctThreads>(kept, s_scan, &K);
    dev::block_excl_scan<kOctThreads>(expandKids, s_scan, &E2);
    {
      int s = pushBase, kp = keptBase;
      for (int j = 0; j < kOctPer; j++) {
        const int i = i0 + j;
        if (i >= Lsz) break;
        if (nflag[i]) {
          const int x0 = nx0[cur][i], y0 = ny0[cur][i], x1 = nx1[cur][i], y1 = ny1[cur][i];
          const int mx = x0 + ((x1 - x0 + 1) >> 1), my = y0 + ((y1 - y0 + 1) >> 1);
          for (int q = 0; q < 4; q++) {
            const int cq = ccnt[4 * i + q];
            if (cq == 0) continue;
            const int pos = P - 1 - s;
            npos[4 * i + q] = pos;
            nx0[nxt][pos] = (int16_t)((q & 1) ? mx : x0);
            nx1[nxt][pos] = (int16_t)((q & 1) ? x1 : mx);
            ny0[nxt][pos] = (int16_t)((q & 2) ? my : y0);
            ny1[nxt][pos] = (int16_t)((q & 2) ? y1 : my);
            ncnt[nxt][pos] = cq;
            nseq[nxt][pos] = seqc + s;
            s++;
          }
        } else {
          const int pos = P + kp;
          npos[4 * i] = pos;
          nx0[nxt][pos] = nx0[cur][i]; nx1[nxt][pos] = nx1[cur][i];
          ny0[nxt][pos] = ny0[cur][i]; ny1[nxt][pos] = ny1[cur][i];
          ncnt[nxt][pos] = ncnt[cur][i];
          nseq[nxt][pos] = nseq[cur][i];
          kp++;
        }
      }
    }
    __syncthreads();
    for (int k = tid; k < n; k += kOctThreads) {
      const int nd = cnode[k];
      if (nflag[nd]) {
        const int midx = nx0[cur][nd] + ((nx1[cur][nd] - nx0[cur][nd] + 1) >> 1);
        const int midy = ny0[cur][nd] + ((ny1[cur][nd] - ny0[cur][nd] + 1) >> 1);
        cnode[k] = npos[4 * nd + oct_quad(cand[k], midx, midy)];
      } else {
        cnode[k] = npos[4 * nd];
      }
    }
    lastPushBase = seqc;
    seqc += P;
    Lsz = P + K;
    cur = nxt;
    __syncthreads();
    if (Lsz >= N || Lsz == prevSize) { finished = true; break; }
    if (Lsz + 3 * E2 > N) break;  // -> final phase
  }

  // ---- 4. final phase (:771-836): divide largest nodes first until >= N
  if (!finished) {
    int roundBase = lastPushBase;
    while (true) {
      const int prevSize = Lsz;
      const int nxt = cur ^ 1;
      unsigned long long* keys = reinterpret_cast<unsigned long long*>(s_pref);  // 2048 x u64
      // E = nodes created in the previous round with > 1 key
      int inE = 0;
      const int i0 = tid * kOctPer;
      for (int j = 0; j < kOctPer; j++) {
        const int i = i0 + j;
        if (i < Lsz) inE += (nseq[cur][i] >= roundBase && ncnt[cur][i] > 1);
      }
      int M;
      int eb = dev::block_excl_scan<kOctThreads>(inE, s_scan, &M);
      int M2 = 1;
      while (M2 < M) M2 <<= 1;
      for (int j = 0; j < kOctPer; j++) {
        const int i = i0 + j;
        if (i < Lsz) {
          const bool e = nseq[cur][i] >= roundBase && ncnt[cur][i] > 1;
          nflag[i] = 0;
          ccnt[4 * i] = ccnt[4 * i + 1] = ccnt[4 * i + 2] = ccnt[4 * i + 3] = 0;
          if (e) {
            keys[eb++] = ((unsigned long long)ncnt[cur][i] << 40) |
                         ((unsigned long long)nseq[cur][i] << 12) | (unsigned long long)i;
            nflag[i] = 1;
          }
        }
      }
      for (int i = M + tid; i < M2; i += kOctThreads) keys[i] = 0ull;
      __syncthreads();
      // bitonic sort, descending
      for (int k = 2; k <= M2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
          for (int i = tid; i < M2; i += kOctThreads) {
            const int ixj = i ^ j;
            if (ixj > i) {
              const unsigned long long ki = keys[i], kj = keys[ixj];
              const bool desc = (i & k) == 0;
              if (desc ? (ki < kj) : (ki > kj)) { keys[i] = kj; keys[ixj] = ki; }
            }
          }
          __syncthreads();
        }
      }
      // child counts of E nodes
      for (int k = tid; k < n; k += kOctThreads) {
        const int nd = cnode[k];
        if (nflag[nd]) {
          const int midx = nx0[cur][nd] + ((nx1[cur][nd] - nx0[cur][nd] + 1) >> 1);
          const int midy = ny0[cur][nd] + ((ny1[cur][nd] - ny0[cur][nd] + 1) >> 1);
          atomicAdd(&ccnt[4 * nd + oct_quad(cand[k], midx, midy)], 1);
        }
      }
      __syncthreads();
      // sorted position j -> delta (nonempty children - 1); processed prefix
      int dsum = 0;
      const int j0 = tid * kOctPer;  // M <= kOctMaxL
      int dl[kOctPer], kl[kOctPer];
      for (int jj = 0; jj < kOctPer; jj++) {
        const int j = j0 + jj;
        dl[jj] = 0; kl[jj] = 0;
        if (j < M) {
          const int nd = (int)(keys[j] & 0xFFF);
          int kids = 0;
          for (int q = 0; q < 4; q++) kids += ccnt[4 * nd + q] > 0;
          kl[jj] = kids;
          dl[jj] = kids - 1;
        }
        dsum += dl[jj];
      }
      int Dtot;
      int dpre = dev::block_excl_scan<kOctThreads>(dsum, s_scan, &Dtot);
      // first j with Lsz + inclusive(delta) >= N -> processed = j+1
      if (tid == 0) s_var[1] = M;
      __syncthreads();
      {
        int run = dpre;
        for (int jj = 0; jj < kOctPer; jj++) {
          const int j = j0 + jj;
          if (j >= M) break;
          run += dl[jj];
          if (Lsz + run >= N) { atomicMin(&s_var[1], j + 1); break; }
        }
      }
      __syncthreads();
      const int Mp = s_var[1];
      // pushes of processed sorted nodes (in sorted order, children n1..n4)
      int mykids = 0;
      for (int jj = 0; jj < kOctPer; jj++)
        if (j0 + jj < Mp) mykids += kl[jj];
      int Pn;
      int kbase = dev::block_excl_scan<kOctThreads>(mykids, s_scan, &Pn);
      // mark processed (nflag = 2) and place children
      {
        int s = kbase;
        for (int jj = 0; jj < kOctPer; jj++) {
          const int j = j0 + jj;
          if (j >= Mp) break;
          const int nd = (int)(keys[j] & 0xFFF);
          nflag[nd] = 2;
          const int x0 = nx0[cur][nd], y0 = ny0[cur][nd], x1 = nx1[cur][nd], y1 = ny1[cur][nd];
          const int mx = x0 + ((x1 - x0 + 1) >> 1), my = y0 + ((y1 - y0 + 1) >> 1);
          for (int q = 0; q < 4; q++) {
            const int cq = ccnt[4 * nd + q];
            if (cq == 0) continue;
            const int pos = Pn - 1 - s;
            npos[4 * nd + q] = pos;
            nx0[nxt][pos] = (int16_t)((q & 1) ? mx : x0);
            nx1[nxt][pos] = (int16_t)((q & 1) ? x1 : mx);
            ny0[nxt][pos] = (int16_t)((q & 2) ? my : y0);
            ny1[nxt][pos] = (int16_t)((q & 2) ? y1 : my);
            ncnt[nxt][pos] = cq;
            nseq[nxt][pos] = seqc + s;
            s++;
          }
        }
      }
      __syncthreads();
      // remaining (unprocessed) list nodes keep their order after the pushes
      int kept = 0;
      for (int j = 0; j < kOctPer; j++) {
        const int i = i0 + j;
        if (i < Lsz && nflag[i] != 2) kept++;
      }
      int Kn;
      int kb = dev::block_excl_scan<kOctThreads>(kept, s_scan, &Kn);
      for (int j = 0; j < kOctPer; j++) {
        const int i = i0 + j;
        if (i < Lsz && nflag[i] != 2) {
          const int pos = Pn + kb++;
          npos[4 * i] = pos;
          nx0[nxt][pos] = nx0[cur][i]; nx1[nxt][pos] = nx1[cur][i];
          ny0[nxt][pos] = ny0[cur][i]; ny1[nxt][pos] = ny1[cur][i];
          ncnt[nxt][pos] = ncnt[cur][i];
          nseq[nxt][pos] = nseq[cur][i];
        }
      }
      __syncthreads();
      for (int k = tid; k < n; k += kOctThreads) {
        const int nd = cnode[k];
        if (nflag[nd] == 2) {
          const int midx = nx0[cur][nd] + ((nx1[cur][nd] - nx0[cur][nd] + 1) >> 1);
          const int midy = ny0[cur][nd] + ((ny1[cur][nd] - ny0[cur][nd] + 1) >> 1);
          cnode[k] = npos[4 * nd + oct_quad(cand[k], midx, midy)];
        } else {
          cnode[k] = npos[4 * nd];
        }
      }
      roundBase = seqc;
      seqc += Pn;
      Lsz = Pn + Kn;
      cur = nxt;
      __syncthreads();
      if (Lsz >= N || Lsz == prevSize) break;
    }
  }

  // ---- 5. retain the best (first max) key per node, in list order (:839-858)
  unsigned int* best = reinterpret_cast<unsigned int*>(ccnt);
  for (int i = tid; i < Lsz; i += kOctThreads) best[i] = 0u;
  __syncthreads();
  for (int k = tid; k < n; k += kOctThreads) {
    const uint32_t pk = cand[k];
    atomicMax(&best[cnode[k]], ((pk >> 24) << 24) | (0xFFFFFFu - (unsigned)k));
  }
  __syncthreads();
  uint32_t* sel = a.sel + (int64_t)f * a.sel_fstride + L.sel_off;
  for (int i = tid; i < Lsz; i += kOctThreads) sel[i] = cand[0xFFFFFFu - (best[i] & 0xFFFFFFu)];
  if (tid == 0) {
    a.sel_count[(int64_t)f * a.nlevels + l] = Lsz;
    atomicAdd(&a.frame_count[f], Lsz);
  }
}

// ===========================================================================
// K4+K6: IC_Angle (unblurred level) + rotated BRIEF (blurred level), one wave per
// keypoint; output keypoints/descriptors in the reference's level-concatenated order.
// ===========================================================================
struct DescArgs {
  LevelPlan lv[kMaxLevels];
  int nlevels;
  const uint8_t* img0; int64_t img0_fstride;
  const uint8_t* pyr; int64_t pyr_fstride;
  const uint8_t* blur; int64_t blur_fstride;
  const uint32_t* sel; int64_t sel_fstride; int sel_per_frame;
  const int32_t* sel_count;
  mcs_keypoint* kps; uint8_t* desc; int cap; int desc_size;
};

__device__ __forceinline__ float fast_atan2_dev(float y, float x) {
  // OpenCV fastAtan2: float ops, no contraction (explicit _rn intrinsics)
  const float k = (float)(180 / 3.14159265358979323846);
  const float p1 = __fmul_rn(0.9997878412794807f, k), p3 = __fmul_rn(-0.3258083974640975f, k);
  const float p5 = __fmul_rn(0.1555786518463281f, k), p7 = __fmul_rn(-0.04432655554792128f, k);
  const float ax = fabsf(x), ay = fabsf(y);
  float a, c, c2;
  const float eps = (float)2.220446049250313080847e-16;
  if (ax >= ay) {
    c = __fdiv_rn(ay, __fadd_rn(ax, eps));
    c2 = __fmul_rn(c, c);
    a = __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1), c);
  } else {
    c = __fdiv_rn(ax, __fadd_rn(ay, eps));
    c2 = __fmul_rn(c, c);
    a = __fsub_rn(90.f, __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1), c));
  }
  if (x < 0) a = __fsub_rn(180.f, a);
  if (y < 0) a = __fsub_rn(360.f, a);
  return a;
}

__global__ __launch_bounds__(256) void k_orient_desc(DescArgs a) {
  const int f = blockIdx.y, lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
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
  const int w = L.w;
  const uint8_t* img = (l == 0) ? a.img0 + (int64_t)f * a.img0_fstride
                                : a.pyr + (int64_t)f * a.pyr_fstride + L.pyr_off;
  // IC_Angle: integer moments over the r=16 circular patch
  int m10 = 0, m01 = 0;
  for (int idx = lane; idx < 33 * 33; idx += 64) {
    const int v = idx / 33 - kHalfPatch, u = idx % 33 - kHalfPatch;
    const int av = v < 0 ? -v : v;
    const int au = u < 0 ? -u : u;
    if (au <= c_umax[av]) {
      const int I = img[(int64_t)(cy + v) * w + (cx + u)];
      m10 += u * I;
      m01 += v * I;
    }
  }
  m10 = dev::wave_sum(m10);
  m01 = dev::wave_sum(m01);
  const float angle = fast_atan2_dev((float)m01, (float)m10);
  // rotated BRIEF on the blurred level (compute_ORB :303-354)
  const float DEG2RADf = (float)3.14159265358979323846 / 180.f;
  const double theta = (double)__fmul_rn(angle, DEG2RADf);
  const double ca = cos(theta), sa = sin(theta);
  const uint8_t* bl = a.blur + (int64_t)f * a.blur_fstride + L.img_off;
  const int nwords = a.desc_size / 8;
  uint8_t* dptr = a.desc + ((int64_t)f * a.cap + outIdx) * a.desc_size;
  for (int r = 0; r < nwords; r++) {
    const int t = r * 64 + lane;  // test index: byte t/8, bit t%8
    const int px0 = c_pattern[4 * t], py0 = c_pattern[4 * t + 1];
    const int px1 = c_pattern[4 * t + 2], py1 = c_pattern[4 * t + 3];
    const int rx0 = (int)rint(__dsub_rn(__dmul_rn((double)px0, ca), __dmul_rn((double)py0, sa)));
    const int ry0 = (int)rint(__dadd_rn(__dmul_rn((double)px0, sa), __dmul_rn((double)py0, ca)));
    const int rx1 = (int)rint(__dsub_rn(__dmul_rn((double)px1, ca), __dmul_rn((double)py1, sa)));
    const int ry1 = (int)rint(__dadd_rn(__dmul_rn((double)px1, sa), __dmul_rn((double)py1, ca)));
    const int t0 = bl[(int64_t)(cy + ry0) * w + (cx + rx0)];
    const int t1 = bl[(int64_t)(cy + ry1) * w + (cx + rx1)];
    const uint64_t bits = __ballot(t0 < t1);
    if (lane == 0) reinterpret_cast<uint64_t*>(dptr)[r] = bits;
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

// ===========================================================================
// host side
// ===========================================================================
template <typename T>
static int dalloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  MCS_HIP_CHECK(hipMalloc((void**)p, count * sizeof(T)));
  return MCS_OK;
}

}  // namespace mcs

struct mcs_extractor {
  mcs::Plan plan;
  int device = 0;
  int max_frames = 0;
  // device tables
  int32_t* d_xofs = nullptr; int16_t* d_alpha = nullptr;
  int32_t* d_yofs = nullptr; int16_t* d_beta = nullptr;
  mcs::CellDesc* d_cells = nullptr;
  // workspace
  uint8_t* d_pyr = nullptr;      // [F][pyr_frame_bytes]
  uint8_t* d_blur = nullptr;     // [F][img_frame_bytes]
  uint32_t* d_slots = nullptr;   // [F][slots_per_frame]
  int32_t* d_cell_counts = nullptr;  // [F][ncells]
  uint32_t* d_cand = nullptr;    // [F][cand_per_frame]
  int32_t* d_cnode = nullptr;    // [F][cand_per_frame]
  uint32_t* d_sel = nullptr;     // [F][sel_per_frame]
  int32_t* d_sel_count = nullptr;  // [F][nlevels]
  // masks
  uint8_t* d_mask_pyr = nullptr; int n_masks = 0;     // registered
  uint8_t* d_mask_single = nullptr;                   // single-frame call mask pyramid
  // single-frame staging
  uint8_t* d_in = nullptr;
  mcs_keypoint* d_kps = nullptr; uint8_t* d_desc = nullptr; int32_t* d_count = nullptr;
  // last call (for read_stage)
  const uint8_t* last_img0 = nullptr;
  int last_frames = 0;
  // live stage timing: ring of event sets (MCS_EXTRACTOR_NSTAGES + 1 events per call)
  static constexpr int kRing = 256;
  bool timing = false;
  hipEvent_t* ev = nullptr;   // [kRing][NSTAGES+1]
  int ev_count = 0;           // calls recorded since last reset (<= kRing)
};

namespace mcs {

static void fill_fast_level_tables(const Plan& pl, FastArgs& fa) {
  for (int l = 0; l < kMaxLevels; l++) {
    fa.lw[l] = l < pl.nlevels ? pl.lv[l].w : 0;
    fa.lh[l] = l < pl.nlevels ? pl.lv[l].h : 0;
    fa.lpyr_off[l] = l < pl.nlevels ? pl.lv[l].pyr_off : 0;
    fa.limg_off[l] = l < pl.nlevels ? pl.lv[l].img_off : 0;
  }
}

static int build_mask_pyramids(mcs_extractor* h, const uint8_t* d_masks, int n, uint8_t* dst,
                               hipStream_t st) {
  const Plan& pl = h->plan;
  const LevelPlan& L0 = pl.lv[0];
  dim3 b(256);
  dim3 g0((L0.w + 63) / 64, (L0.h + 3) / 4, n);
  hipLaunchKernelGGL(k_copy_bytes, g0, b, 0, st, d_masks, (int64_t)L0.w * L0.h, dst,
                     pl.img_frame_bytes, L0.w, L0.h);
  for (int l = 1; l < pl.nlevels; l++) {
    const LevelPlan& S = pl.lv[l - 1];
    const LevelPlan& D = pl.lv[l];
    dim3 g((D.w + 63) / 64, (D.h + 3) / 4, n);
    // per-frame stride identical for src/dst (both inside the same mask pyramid slot)
    hipLaunchKernelGGL(k_mask_nearest, g, b, 0, st, dst + S.img_off, S.w, S.h, dst + D.img_off,
                       D.w, D.h, pl.img_frame_bytes);
  }
  MCS_HIP_CHECK(hipGetLastError());
  return MCS_OK;
}

static inline void stage_mark(mcs_extractor* h, int stage, hipStream_t st) {
  if (!h->timing || h->ev_count >= mcs_extractor::kRing) return;
  (void)hipEventRecord(h->ev[h->ev_count * (MCS_EXTRACTOR_NSTAGES + 1) + stage], st);
}

// Core batched pipeline on device buffers.
static int run_batch(mcs_extractor* h, const uint8_t* d_images, int F, const uint8_t* mask_pyr,
                     const int32_t* d_mask_index, mcs_keypoint* d_kps, int32_t* d_counts,
                     uint8_t* d_desc, hipStream_t st) {
  const Plan& pl = h->plan;
  const int nl = pl.nlevels;
  const int64_t img0_fs = (int64_t)pl.W * pl.H;
  dim3 b256(256);
  stage_mark(h, 0, st);
  // K1: pyramid chain
  for (int l = 1; l < nl; l++) {
    const LevelPlan& S = pl.lv[l - 1];
    const LevelPlan& D = pl.lv[l];
    const uint8_t* src = (l == 1) ? d_images : h->d_pyr + S.pyr_off;
    const int64_t sfs = (l == 1) ? img0_fs : pl.pyr_frame_bytes;
    dim3 g((D.w + 63) / 64, (D.h + 3) / 4, F);
    hipLaunchKernelGGL(k_resize_linear, g, b256, 0, st, src, sfs, S.w, S.h, h->d_pyr + D.pyr_off,
                       pl.pyr_frame_bytes, D.w, D.h, h->d_xofs + pl.xtab_off[l],
                       h->d_alpha + 2 * pl.xtab_off[l], h->d_yofs + pl.ytab_off[l],
                       h->d_beta + 2 * pl.ytab_off[l], D.simd_end);
  }
  stage_mark(h, 1, st);
  // K5: blur every level (only levels with keypoints are read)
  for (int l = 0; l < nl; l++) {
    const LevelPlan& L = pl.lv[l];
    const uint8_t* src = (l == 0) ? d_images : h->d_pyr + L.pyr_off;
    const int64_t sfs = (l == 0) ? img0_fs : pl.pyr_frame_bytes;
    dim3 g((L.w + 63) / 64, (L.h + 3) / 4, F);
    hipLaunchKernelGGL(k_blur5, g, b256, 0, st, src, sfs, h->d_blur + L.img_off,
                       pl.img_frame_bytes, L.w, L.h);
  }
  stage_mark(h, 2, st);
  // K2: FAST cells
  {
    FastArgs fa;
    fa.img0 = d_images; fa.img0_fstride = img0_fs;
    fa.pyr = h->d_pyr; fa.pyr_fstride = pl.pyr_frame_bytes;
    fa.mask_pyr = mask_pyr; fa.mask_fstride = pl.img_frame_bytes;
    fa.mask_index = d_mask_index;
    fa.cells = h->d_cells; fa.ncells = (int)pl.cells.size();
    fa.slots = h->d_slots; fa.slots_fstride = pl.slots_per_frame;
    fa.cell_counts = h->d_cell_counts;
    fa.threshold = std::min(std::max(pl.p.fast_threshold, 0), 255);
    fill_fast_level_tables(pl, fa);
    dim3 g((unsigned)pl.cells.size(), F);
    hipLaunchKernelGGL(k_fast_cells, g, dim3(64), 0, st, fa);
  }
  MCS_HIP_CHECK(hipMemsetAsync(d_counts, 0, sizeof(int32_t) * F, st));
  stage_mark(h, 3, st);
  // K3: octree
  {
    OctArgs oa;
    std::memcpy(oa.lv, pl.lv, sizeof(oa.lv));
    oa.cells = h->d_cells;
    oa.cell_counts = h->d_cell_counts; oa.ncells = (int)pl.cells.size();
    oa.slots = h->d_slots; oa.slots_fstride = pl.slots_per_frame;
    oa.cand = h->d_cand; oa.cnode = h->d_cnode; oa.cand_fstride = pl.cand_per_frame;
    oa.sel = h->d_sel; oa.sel_fstride = pl.sel_per_frame;
    oa.sel_count = h->d_sel_count; oa.nlevels = nl;
    oa.frame_count = d_counts;
    dim3 g(nl, F);
    hipLaunchKernelGGL(k_octree, g, dim3(kOctThreads), 0, st, oa);
  }
  stage_mark(h, 4, st);
  // K4+K6: orientation + descriptor
  {
    DescArgs da;
    std::memcpy(da.lv, pl.lv, sizeof(da.lv));
    da.nlevels = nl;
    da.img0 = d_images; da.img0_fstride = img0_fs;
    da.pyr = h->d_pyr; da.pyr_fstride = pl.pyr_frame_bytes;
    da.blur = h->d_blur; da.blur_fstride = pl.img_frame_bytes;
    da.sel = h->d_sel; da.sel_fstride = pl.sel_per_frame; da.sel_per_frame = pl.sel_per_frame;
    da.sel_count = h->d_sel_count;
    da.kps = d_kps; da.desc = d_desc; da.cap = pl.sel_per_frame; da.desc_size = pl.p.desc_size;
    dim3 g((pl.sel_per_frame + 3) / 4, F);
    hipLaunchKernelGGL(k_orient_desc, g, b256, 0, st, da);
  }
  stage_mark(h, 5, st);
  if (h->timing && h->ev_count < mcs_extractor::kRing) h->ev_count++;
  MCS_HIP_CHECK(hipGetLastError());
  h->last_img0 = d_images;
  h->last_frames = F;
  return MCS_OK;
}

}  // namespace mcs

using namespace mcs;

extern "C" {

void mcs_extractor_default_params(mcs_extractor_params* p) {
  if (!p) return;
  p->nfeatures = 1000; p->scale_factor = 1.2f; p->nlevels = 8; p->edge_threshold = 25;
  p->first_level = 0; p->score_type = 0; p->patch_size = 32; p->fast_threshold = 20;
  p->use_agast = 0; p->fast_agast_type = 2; p->do_dbrief = 0; p->learn_masks = 0;
  p->desc_size = 32;
}

int mcs_extractor_create(const mcs_extractor_params* p, int32_t width, int32_t height,
                         int32_t max_frames, int32_t device, mcs_extractor** out) {
  if (!p || !out || max_frames < 1) { set_error("null argument"); return MCS_ERR_ARG; }
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    set_error("no HIP device visible (libmcs_amd has no CPU fallback)");
    return MCS_ERR_NO_DEVICE;
  }
  if (device < 0 || device >= ndev) { set_error("bad device ordinal"); return MCS_ERR_ARG; }
  MCS_HIP_CHECK(hipSetDevice(device));
  mcs_extractor* h = new (std::nothrow) mcs_extractor();
  if (!h) return MCS_ERR_ARG;
  int rc = build_plan(*p, width, height, h->plan);
  if (rc != MCS_OK) { delete h; return rc; }
  h->device = device;
  h->max_frames = max_frames;
  const Plan& pl = h->plan;
  const size_t F = (size_t)max_frames;
  static bool consts_done[64] = {false};
  if (device < 64 && !consts_done[device]) {
    int umax[kHalfPatch + 1];
    {  // ctor :187-202
      int v, v0, vmax = (int)std::floor(kHalfPatch * std::sqrt(2.f) / 2 + 1);
      int vmin = (int)std::ceil(kHalfPatch * std::sqrt(2.f) / 2);
      const double hp2 = kHalfPatch * kHalfPatch;
      for (v = 0; v <= vmax; ++v) umax[v] = cv_round(std::sqrt(hp2 - v * v));
      for (v = kHalfPatch, v0 = 0; v >= vmin; --v) {
        while (umax[v0] == umax[v0 + 1]) ++v0;
        umax[v] = v0;
        ++v0;
      }
    }
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_umax), umax, sizeof(umax)) != hipSuccess) {
      delete h; set_error("hipMemcpyToSymbol(c_umax) failed"); return MCS_ERR_HIP;
    }
    consts_done[device] = true;
  }
#define ALLOC(ptr, n)                                  \
  do {                                                 \
    if ((rc = dalloc(&(ptr), (n))) != MCS_OK) {        \
      mcs_extractor_destroy(h);                        \
      return rc;                                       \
    }                                                  \
  } while (0)
  ALLOC(h->d_xofs, pl.xofs.size());
  ALLOC(h->d_alpha, pl.alpha.size());
  ALLOC(h->d_yofs, pl.yofs.size());
  ALLOC(h->d_beta, pl.beta.size());
  ALLOC(h->d_cells, pl.cells.size());
  ALLOC(h->d_pyr, F * pl.pyr_frame_bytes);
  ALLOC(h->d_blur, F * pl.img_frame_bytes);
  ALLOC(h->d_slots, F * pl.slots_per_frame);
  ALLOC(h->d_cell_counts, F * pl.cells.size());
  ALLOC(h->d_cand, F * pl.cand_per_frame);
  ALLOC(h->d_cnode, F * pl.cand_per_frame);
  ALLOC(h->d_sel, F * pl.sel_per_frame);
  ALLOC(h->d_sel_count, F * pl.nlevels);
  ALLOC(h->d_mask_single, pl.img_frame_bytes);
  ALLOC(h->d_in, (size_t)width * height);
  ALLOC(h->d_kps, pl.sel_per_frame);
  ALLOC(h->d_desc, (size_t)pl.sel_per_frame * pl.p.desc_size);
  ALLOC(h->d_count, 1);
#undef ALLOC
  hipError_t e = hipSuccess;
  if (e == hipSuccess) e = hipMemcpy(h->d_xofs, pl.xofs.data(), pl.xofs.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(h->d_alpha, pl.alpha.data(), pl.alpha.size() * 2, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(h->d_yofs, pl.yofs.data(), pl.yofs.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(h->d_beta, pl.beta.data(), pl.beta.size() * 2, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(h->d_cells, pl.cells.data(), pl.cells.size() * sizeof(CellDesc), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    set_hip_error(e, "upload plan tables", __FILE__, __LINE__);
    mcs_extractor_destroy(h);
    return MCS_ERR_HIP;
  }
  *out = h;
  return MCS_OK;
}

void mcs_extractor_destroy(mcs_extractor* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  void* ptrs[] = {h->d_xofs, h->d_alpha, h->d_yofs, h->d_beta, h->d_cells, h->d_pyr, h->d_blur,
                  h->d_slots, h->d_cell_counts, h->d_cand, h->d_cnode, h->d_sel, h->d_sel_count,
                  h->d_mask_pyr, h->d_mask_single, h->d_in, h->d_kps, h->d_desc, h->d_count};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (h->ev) {
    for (int i = 0; i < mcs_extractor::kRing * (MCS_EXTRACTOR_NSTAGES + 1); i++)
      (void)hipEventDestroy(h->ev[i]);
    delete[] h->ev;
  }
  delete h;
}

int mcs_extractor_enable_timing(mcs_extractor* h, int32_t enable) {
  if (!h) return MCS_ERR_ARG;
  MCS_HIP_CHECK(hipSetDevice(h->device));
  if (enable && !h->ev) {
    const int n = mcs_extractor::kRing * (MCS_EXTRACTOR_NSTAGES + 1);
    h->ev = new hipEvent_t[n];
    for (int i = 0; i < n; i++) MCS_HIP_CHECK(hipEventCreate(&h->ev[i]));
  }
  h->timing = enable != 0;
  h->ev_count = 0;
  return MCS_OK;
}

int mcs_extractor_read_timing(mcs_extractor* h, float* ms_per_stage, int32_t* ncalls,
                              int32_t reset) {
  if (!h || !ms_per_stage) return MCS_ERR_ARG;
  MCS_HIP_CHECK(hipSetDevice(h->device));
  for (int s = 0; s < MCS_EXTRACTOR_NSTAGES; s++) ms_per_stage[s] = 0.f;
  const int K = MCS_EXTRACTOR_NSTAGES + 1;
  for (int c = 0; c < h->ev_count; c++) {
    MCS_HIP_CHECK(hipEventSynchronize(h->ev[c * K + K - 1]));
    for (int s = 0; s < MCS_EXTRACTOR_NSTAGES; s++) {
      float ms = 0.f;
      MCS_HIP_CHECK(hipEventElapsedTime(&ms, h->ev[c * K + s], h->ev[c * K + s + 1]));
      ms_per_stage[s] += ms;
    }
  }
  if (ncalls) *ncalls = h->ev_count;
  if (reset) h->ev_count = 0;
  return MCS_OK;
}

int32_t mcs_extractor_capacity(const mcs_extractor* h) { return h ? h->plan.sel_per_frame : 0; }

int mcs_extractor_levels(const mcs_extractor* h, int32_t* nlevels, int32_t* wh, int32_t* nfeat) {
  if (!h) return MCS_ERR_ARG;
  if (nlevels) *nlevels = h->plan.nlevels;
  for (int l = 0; l < h->plan.nlevels; l++) {
    if (wh) { wh[2 * l] = h->plan.lv[l].w; wh[2 * l + 1] = h->plan.lv[l].h; }
    if (nfeat) nfeat[l] = h->plan.lv[l].nfeat;
  }
  return MCS_OK;
}

int mcs_extractor_set_masks_device(mcs_extractor* h, const uint8_t* d_masks, int32_t n_masks,
                                   void* stream) {
  if (!h || n_masks < 0 || (n_masks > 0 && !d_masks)) return MCS_ERR_ARG;
  MCS_HIP_CHECK(hipSetDevice(h->device));
  if (h->d_mask_pyr) { MCS_HIP_CHECK(hipFree(h->d_mask_pyr)); h->d_mask_pyr = nullptr; }
  h->n_masks = 0;
  if (n_masks == 0) return MCS_OK;
  int rc = dalloc(&h->d_mask_pyr, (size_t)n_masks * h->plan.img_frame_bytes);
  if (rc) return rc;
  rc = build_mask_pyramids(h, d_masks, n_masks, h->d_mask_pyr, (hipStream_t)stream);
  if (rc) return rc;
  h->n_masks = n_masks;
  return MCS_OK;
}

int mcs_extract_batch_device(mcs_extractor* h, const uint8_t* d_images, int32_t n_frames,
                             const int32_t* d_mask_index, mcs_keypoint* d_kps,
                             int32_t* d_counts, uint8_t* d_desc, void* stream) {
  if (!h || !d_images || !d_kps || !d_counts || !d_desc || n_frames < 1) {
    set_error("null argument"); return MCS_ERR_ARG;
  }
  if (n_frames > h->max_frames) { set_error("n_frames > max_frames"); return MCS_ERR_CAPACITY; }
  MCS_HIP_CHECK(hipSetDevice(h->device));
  const uint8_t* mp = h->n_masks > 0 ? h->d_mask_pyr : nullptr;
  return run_batch(h, d_images, n_frames, mp, mp ? d_mask_index : nullptr, d_kps, d_counts,
                   d_desc, (hipStream_t)stream);
}

int mcs_extract(mcs_extractor* h, const uint8_t* image, int32_t stride, const uint8_t* mask,
                int32_t mask_stride, mcs_keypoint* kps, int32_t kps_cap, int32_t* n_out,
                uint8_t* desc, uint8_t* desc_masks) {
  if (!h || !n_out) return MCS_ERR_ARG;
  *n_out = 0;
  if (!image) return MCS_OK;  // empty image: silent return (:1252-1253)
  const Plan& pl = h->plan;
  if (stride < pl.W || (mask && mask_stride < pl.W)) return MCS_ERR_ARG;
  MCS_HIP_CHECK(hipSetDevice(h->device));
  hipStream_t st = nullptr;
  MCS_HIP_CHECK(hipMemcpy2D(h->d_in, pl.W, image, stride, pl.W, pl.H, hipMemcpyHostToDevice));
  const uint8_t* mp = nullptr;
  if (mask) {
    // stage the mask through d_desc-sized scratch: reuse d_mask_single level-0 slot
    MCS_HIP_CHECK(hipMemcpy2D(h->d_mask_single, pl.W, mask, mask_stride, pl.W, pl.H,
                              hipMemcpyHostToDevice));
    int rc = build_mask_pyramids(h, h->d_mask_single, 1, h->d_mask_single, st);
    if (rc) return rc;
    mp = h->d_mask_single;
  }
  int rc = run_batch(h, h->d_in, 1, mp, nullptr, h->d_kps, h->d_count, h->d_desc, st);
  if (rc) return rc;
  int32_t n = 0;
  MCS_HIP_CHECK(hipMemcpy(&n, h->d_count, sizeof(n), hipMemcpyDeviceToHost));
  *n_out = n;
  if (n > kps_cap) { set_error("kps_cap too small"); return MCS_ERR_CAPACITY; }
  if (n > 0) {
    if (kps) MCS_HIP_CHECK(hipMemcpy(kps, h->d_kps, sizeof(mcs_keypoint) * n, hipMemcpyDeviceToHost));
    if (desc) MCS_HIP_CHECK(hipMemcpy(desc, h->d_desc, (size_t)n * pl.p.desc_size, hipMemcpyDeviceToHost));
    if (desc_masks) std::memset(desc_masks, 0, (size_t)n * pl.p.desc_size);
  }
  return MCS_OK;
}

int mcs_extractor_read_stage(mcs_extractor* h, int32_t stage, int32_t frame, int32_t level,
                             void* dst, int64_t cap, int64_t* n_out) {
  if (!h || !n_out || level < 0 || level >= h->plan.nlevels || frame < 0 ||
      frame >= h->last_frames)
    return MCS_ERR_ARG;
  MCS_HIP_CHECK(hipSetDevice(h->device));
  MCS_HIP_CHECK(hipDeviceSynchronize());
  const Plan& pl = h->plan;
  const LevelPlan& L = pl.lv[level];
  *n_out = 0;
  if (stage == 0 || stage == 1) {
    const int64_t nb = (int64_t)L.w * L.h;
    *n_out = nb;
    if (cap < nb) return MCS_ERR_CAPACITY;
    const uint8_t* src;
    if (stage == 0)
      src = level == 0 ? h->last_img0 + (int64_t)frame * pl.W * pl.H
                       : h->d_pyr + (int64_t)frame * pl.pyr_frame_bytes + L.pyr_off;
    else
      src = h->d_blur + (int64_t)frame * pl.img_frame_bytes + L.img_off;
    MCS_HIP_CHECK(hipMemcpy(dst, src, nb, hipMemcpyDeviceToHost));
    return MCS_OK;
  }
  if (stage == 2 || stage == 3) {
    int64_t n = 0;
    const uint32_t* src;
    if (stage == 2) {
      std::vector<int32_t> cc(L.cell_end - L.cell_begin);
      MCS_HIP_CHECK(hipMemcpy(cc.data(), h->d_cell_counts + (int64_t)frame * pl.cells.size() + L.cell_begin,
                              cc.size() * 4, hipMemcpyDeviceToHost));
      for (int v : cc) n += v;
      src = h->d_cand + (int64_t)frame * pl.cand_per_frame + L.cand_off;
    } else {
      int32_t c = 0;
      MCS_HIP_CHECK(hipMemcpy(&c, h->d_sel_count + (int64_t)frame * pl.nlevels + level, 4,
                              hipMemcpyDeviceToHost));
      n = c;
      src = h->d_sel + (int64_t)frame * pl.sel_per_frame + L.sel_off;
    }
    *n_out = n;
    if (cap < 3 * n) return MCS_ERR_CAPACITY;
    std::vector<uint32_t> tmp(n);
    if (n) MCS_HIP_CHECK(hipMemcpy(tmp.data(), src, n * 4, hipMemcpyDeviceToHost));
    int32_t* o = (int32_t*)dst;
    for (int64_t i = 0; i < n; i++) {
      o[3 * i] = tmp[i] & 0xFFF;
      o[3 * i + 1] = (tmp[i] >> 12) & 0xFFF;
      o[3 * i + 2] = tmp[i] >> 24;
    }
    return MCS_OK;
  }
  return MCS_ERR_ARG;
}

}  // extern "C"
