// Extractor plan: all per-configuration geometry computed once on the host at
// mcs_extractor_create() (the reference recomputes it every call inside
// ComputePyramid / ComputeKeyPointsOctTree, src/mdBRIEFextractorOct.cpp:1158-1201,
// 863-971).  Plain structs so they can be passed to kernels by value.
#pragma once
#include <cstdint>
#include <vector>
#include "../../include/mcs_extractor.h"

namespace mcs {

constexpr int kMaxLevels = 12;
constexpr int kEdgeThreshold = 25;             // src/mdBRIEFextractorOct.cpp:86
constexpr int kMinBorder = kEdgeThreshold - 3; // :876
constexpr int kPatchSize = 32;                 // :84
constexpr int kHalfPatch = 16;                 // :85
constexpr int kMaxCellDim = 64;                // window bound per FAST cell (host-checked)
constexpr int kMaxCellsPerLevel = 2048;        // LDS prefix table in the octree kernel
constexpr int kOctMaxL = 1024;                 // octree node-list bound (host-checked)
constexpr double kMaxScaleFactor = 2.2;        // pyramid source-tile bound (k_pyramid.hip)

// One FAST cell of ComputeKeyPointsOctTree (:892-948): the detection window is the
// cell ROI shrunk by 3 px (FAST_t rows/cols [3, n-3)), absolute level coordinates.
struct CellDesc {
  int32_t level;
  int16_t wx0, wy0, wx1, wy1;  // window [wx0,wx1) x [wy0,wy1)
  int32_t slot_off;            // first candidate slot of this cell within a frame
  int32_t slot_cap;            // ceil(ww/2)*ceil(wh/2): max survivors of strict 8-NMS
};

// One work unit of the row-streaming FAST kernel (k_fast_rows): a run of consecutive cells of
// one cell row of one level.  Lane L of the wave holds columns [xa + 4L, xa + 4L + 4); the run
// is sized so that every detection pixel's 7x7 neighbourhood lies in lanes 0..62
// (ux0 - 3 >= xa, ux1 + 3 <= xa + 252).  Cell k of the run starts at ux0 + k * wcell (every
// cell of a level is wcell wide except a clamped last one, which ends at ux1).
struct FastUnit {
  int16_t level, ncells;
  int16_t wy0, wy1;    // detection rows of the cell row
  int16_t ux0, ux1;    // detection columns [first cell wx0, last cell wx1)
  int16_t xa, wcell;
  int32_t cell0;       // global index of the run's first cell
};
constexpr int kFastUnitSpan = 252;   // lanes 0..62 x 4 px

struct LevelPlan {
  int32_t w, h;               // level size (cvRound(W / 1.2^l))
  int32_t pitch;              // row pitch of raw level l (level 0: the input width) and of
                              // the blurred level (all levels: align64(w))
  int32_t bpitch;
  int64_t pyr_off;            // offset of the level inside a frame's pyramid workspace (l >= 1)
  int64_t img_off;            // offset inside a frame's blurred-level workspace (pitch bpitch)
  int64_t mask_off;           // offset inside a mask pyramid (pitch bpitch: aligned dword loads)
  int32_t cell_begin, cell_end;
  int32_t cand_off, cand_cap; // candidate gather area within a frame (sum of cell caps)
  int32_t sel_off, sel_cap;   // octree output area within a frame
  int32_t nfeat;              // mnFeaturesPerLevel[l] (:167-179)
  int32_t nini;               // cvRound((maxX-minX)/(maxY-minY)) (:641)
  double hx;                  // (maxX-minX)/nIni (:643)
  int32_t width_rel, height_rel;  // maxX-minX, maxY-minY of the octree domain
  int32_t simd_end;           // first dx computed by the scalar vertical resize form
  int32_t wcell;              // FAST cell width (every cell but a clamped last one)
  int32_t patch_size_scaled;  // (int)(PATCH_SIZE * scaleFactor^l)  (:959)
  float scale;                // (float)mvScaleFactor[l]  (:1305)
};

struct Plan {
  mcs_extractor_params p;
  int32_t W = 0, H = 0, nlevels = 0;
  double scale_factor = 1.2;  // double((float)p.scale_factor)  (:147)
  LevelPlan lv[kMaxLevels];
  std::vector<CellDesc> cells;
  std::vector<FastUnit> fast_units;       // sorted by level
  int32_t unit_begin[kMaxLevels + 1] = {};  // first unit of each level
  int64_t pyr_frame_bytes = 0;   // levels 1..L-1
  int64_t img_frame_bytes = 0;   // levels 0..L-1 (blurred levels, padded pitch)
  int64_t mask_frame_bytes = 0;  // levels 0..L-1 (mask pyramid, pitch bpitch)
  int32_t slots_per_frame = 0;   // sum of cell caps
  int32_t cand_per_frame = 0;    // == slots_per_frame
  int32_t sel_per_frame = 0;     // sum of level sel caps == mcs_extractor_capacity
  int32_t max_cells_level = 0;
  int32_t max_win_w = 0, max_win_h = 0;  // largest FAST window (LDS sizing)
  // resize tables (concatenated over levels 1..L-1)
  std::vector<int32_t> xofs, yofs;
  std::vector<int16_t> alpha, beta;
  std::vector<int64_t> xtab_off, ytab_off;  // per level offsets into the tables
};

// Returns MCS_OK or an error (unsupported geometry / parameters).
int build_plan(const mcs_extractor_params& p, int W, int H, Plan& plan);

// k_fast_rows units for frames of one registered mask (its host copy of the mask pyramid,
// plan layout).  A cell whose detection window holds no mask pixel emits nothing (runByPixels-
// Mask drops every keypoint; NMS never looks across a cell): such cells become `dead` units
// that only zero the cell's count, and each cell row's live range is re-split into the fewest
// runs (`live`), so a wave covers live cells only.
void build_masked_units(const Plan& pl, const uint8_t* mask_pyr, std::vector<FastUnit>& live,
                        std::vector<FastUnit>& dead);

}  // namespace mcs
