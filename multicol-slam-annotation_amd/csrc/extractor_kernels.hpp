// Kernel argument blocks and launch wrappers of the extractor pipeline (one .hip file per
// stage; the host orchestration lives in extractor.hip).
#pragma once
#include <algorithm>
#include <hip/hip_runtime.h>
#include <cstdint>
#include "extractor_plan.hpp"

namespace mcs {

// Workgroup -> (frame, item) mapping that keeps all workgroups of one frame on one XCD
// (dispatch deals workgroups round-robin over the 8 XCDs; speed only, never correctness).
// Grid = 8 * ceil(F/8) * items_per_frame workgroups; returns false for padding groups.
__device__ __forceinline__ bool xcd_frame_map(int b, int F, int items, int* frame, int* item) {
  const int x = b & 7, k = b >> 3;
  const int f = x + 8 * (k / items);
  *item = k % items;
  *frame = f;
  return f < F;
}
inline unsigned xcd_grid(int F, int items) { return (unsigned)(8 * ((F + 7) / 8) * items); }

struct LevelPtrs {
  int32_t w[kMaxLevels], h[kMaxLevels], pitch[kMaxLevels], bpitch[kMaxLevels];
  int64_t pyr_off[kMaxLevels], img_off[kMaxLevels], mask_off[kMaxLevels];
};

// ---- K1+K5 fused: resize level l-1 -> l (or take level 0) + 5x5 blur of the level
struct PyrArgs {
  const uint8_t* src; int64_t src_fstride; int sw, sh, spitch;  // level l-1 (or level 0)
  uint8_t* dst; int64_t dst_fstride; int dpitch;                // level l raw (RESIZE only)
  uint8_t* blur; int64_t blur_fstride; int bpitch;              // level l blurred
  int dw, dh;
  const int32_t* xofs; const int16_t* alpha; const int32_t* yofs; const int16_t* beta;
  int simd_end;
  int tiles_x, tiles_y, nframes;   // tiles_x = column strips, tiles_y = row segments
  int core, seg_rows;              // strip width (px, multiple of 4, <= 244), segment height
};
// strips of <= 244 columns (61 lanes x 4 px, so a level-0 strip + halo is <= 64 dwords);
// segment height chosen for ~32 waves per frame, at least 8k waves per launch (latency hiding
// for small batches), between 8 and 64 rows.  Per frame that is a fixed geometry, so the
// production step's two halves on two streams (bench.py --split 2: two launches of ~256 frames
// side by side) cut their segments as tall as one launch of the whole batch; a fixed 16k-wave
// target had halved the segments of a half (more halo rows per output row).  Round 6:
// 399 -> 410 M keypoints/s.
inline void pyr_strips(int dw, int dh, int F, PyrArgs& a) {
  const int n = (dw + 243) / 244;
  a.core = ((dw + n - 1) / n + 3) & ~3;
  a.tiles_x = (dw + a.core - 1) / a.core;
#ifndef MCS_PYR_TARGET
#define MCS_PYR_TARGET 8192
#endif
#ifndef MCS_PYR_WAVES_PER_FRAME
#define MCS_PYR_WAVES_PER_FRAME 32
#endif
  // (more waves per frame for the levels under 200 rows only, 48 or 64 with segments down to
  // 6 / 4 rows, and segments down to 4 rows alone measured flat or slower at the end of round 6)
  const long target = std::max<long>(MCS_PYR_TARGET, (long)MCS_PYR_WAVES_PER_FRAME * (F > 0 ? F : 1));
  const long per_seg = (long)a.tiles_x * (F > 0 ? F : 1);
  const int segs = (int)std::max<long>(1, (target + per_seg - 1) / per_seg);
  int rows = (dh + segs - 1) / segs;
#ifndef MCS_PYR_MAXROWS
#define MCS_PYR_MAXROWS 64
#endif
#ifndef MCS_PYR_MINROWS
#define MCS_PYR_MINROWS 8
#endif
  rows = std::min(MCS_PYR_MAXROWS, std::max(MCS_PYR_MINROWS, rows));
  a.seg_rows = rows;
  a.tiles_y = (dh + rows - 1) / rows;
}
// wide: source tiles for scale factors in (1.5, 2.2] (larger LDS footprint)
void launch_pyr_blur(const PyrArgs& a, bool resize, bool wide, hipStream_t st);

void launch_mask_pyramids(const Plan& pl, const uint8_t* d_masks, int n, uint8_t* dst,
                          hipStream_t st);
// ---- K2: FAST over runs of cells (row-streaming), one wave per FastUnit
struct FastRowArgs {
  const uint8_t* img0; int64_t img0_fstride;
  const uint8_t* pyr; int64_t pyr_fstride;
  const uint8_t* mask_pyr; int64_t mask_fstride;  // mask pyramids (nullable = no mask)
  const int32_t* mask_index; int nmasks;           // index clamped to [0, nmasks)
  const FastUnit* units; int nunits;
  int64_t unit_mstride;   // per-mask unit lists (build_masked_units): units of mask m at
                          // units + m * unit_mstride; 0 = one list for every frame
  const CellDesc* cells; int ncells;
  uint32_t* slots; int64_t slots_fstride;
  int32_t* cell_counts;
  int threshold;
  uint32_t kk, rbits;     // byte-wise compare constants (v_lerp_u8), see launch_fast_rows
  int pattern;            // FAST circle: 16 (TYPE_9_16), 12 (TYPE_7_12) or 8 (TYPE_5_8)
  int32_t* frame_count;   // per-frame keypoint counts the octree adds into: zeroed here (unit 0)
  int nframes;
  LevelPtrs lp;
};
void launch_fast_rows(const FastRowArgs& a, hipStream_t st);

// ---- K3: octree
struct OctArgs {
  LevelPlan lv[kMaxLevels];
  const CellDesc* cells;
  const int32_t* cell_counts; int ncells;
  const uint32_t* slots; int64_t slots_fstride;
  uint32_t* cand; int32_t* cnode; int64_t cand_fstride;
  uint32_t* sel; int64_t sel_fstride;
  int32_t* sel_count; int nlevels;
  int32_t* frame_count;
  int nframes;
};
void launch_octree(const OctArgs& a, int max_list, hipStream_t st);

// ---- K4+K6: orientation + descriptors
struct DescArgs {
  LevelPlan lv[kMaxLevels];
  int nlevels;
  const uint8_t* img0; int64_t img0_fstride;
  const uint8_t* pyr; int64_t pyr_fstride;
  const uint8_t* blur; int64_t blur_fstride;
  const uint32_t* sel; int64_t sel_fstride; int sel_per_frame;
  const int32_t* sel_count;
  mcs_keypoint* kps; uint8_t* desc; int cap; int desc_size;
  int nframes;
  // dBRIEF / mdBRIEF (mode 1 / 2; mode 0 = ORB)
  int mode, do_dbrief;
  const mcs_cam_model* cams; const int32_t* cam_index;
  uint8_t* desc_masks;
};
void launch_orient_desc(const DescArgs& a, hipStream_t st);
int upload_desc_constants();

}  // namespace mcs
