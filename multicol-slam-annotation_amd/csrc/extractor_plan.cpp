// Host-side plan construction for the extractor (geometry only, no pixel work).
#include "extractor_plan.hpp"
#include "common.hpp"
#include <algorithm>
#include <cmath>
#include <cstdio>

namespace mcs {

namespace {

int16_t sat_s16_from_float(float v) {
  int i = cv_roundf(v);
  return (int16_t)std::min(std::max(i, -32768), 32767);
}

// cv::resize(INTER_LINEAR) coefficient tables for one src->dst level
// (OpenCV resize() + resizeGeneric_ table setup).
void linear_tables(int sw, int sh, int dw, int dh, Plan& pl) {
  const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
  for (int dx = 0; dx < dw; dx++) {
    float fx = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = cv_floorf(fx);
    fx -= sx;
    if (sx < 0) { fx = 0; sx = 0; }
    if (sx + 1 >= sw && sx >= sw - 1) { fx = 0; sx = sw - 1; }
    pl.xofs.push_back(sx);
    pl.alpha.push_back(sat_s16_from_float((1.f - fx) * 2048));
    pl.alpha.push_back(sat_s16_from_float(fx * 2048));
  }
  for (int dy = 0; dy < dh; dy++) {
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    int sy = cv_floorf(fy);
    fy -= sy;
    pl.yofs.push_back(sy);  // rows are clipped at use (resizeGeneric_ clip(sy, 0, h))
    pl.beta.push_back(sat_s16_from_float((1.f - fy) * 2048));
    pl.beta.push_back(sat_s16_from_float(fy * 2048));
  }
}

// Cells [c, e) of one cell row as k_fast_rows units: the fewest equal runs whose detection span
// (+3 px halo each side) fits one wave's lanes 0..62.
void split_runs(const std::vector<CellDesc>& cells, int c, int e, int level, int wcell,
                std::vector<FastUnit>& out) {
  const int n = e - c;
  auto fits = [&](int a, int b) {
    const int xa = (cells[a].wx0 - 3) & ~3;
    return cells[b - 1].wx1 + 3 <= xa + kFastUnitSpan;
  };
  for (int runs = 1; runs <= n; runs++) {
    const int per = (n + runs - 1) / runs;
    bool ok = true;
    for (int a = c; a < e && ok; a += per) ok = fits(a, std::min(e, a + per));
    if (!ok) continue;
    for (int a = c; a < e; a += per) {
      const int b = std::min(e, a + per);
      FastUnit u;
      u.level = (int16_t)level; u.ncells = (int16_t)(b - a);
      u.wy0 = cells[a].wy0; u.wy1 = cells[a].wy1;
      u.ux0 = cells[a].wx0; u.ux1 = cells[b - 1].wx1;
      u.xa = (int16_t)((u.ux0 - 3) & ~3);
      u.wcell = (int16_t)wcell;
      u.cell0 = a;
      out.push_back(u);
    }
    return;
  }
}

// Cells [c, e) as count-zeroing units (no rows: the wave writes 0 to each cell's count)
void zero_runs(const std::vector<CellDesc>& cells, int c, int e, int level, int wcell,
               std::vector<FastUnit>& out) {
  for (int a = c; a < e; a += 64) {
    const int b = std::min(e, a + 64);
    FastUnit u;
    u.level = (int16_t)level; u.ncells = (int16_t)(b - a);
    u.wy0 = u.wy1 = cells[a].wy0;
    u.ux0 = cells[a].wx0; u.ux1 = cells[b - 1].wx1;
    u.xa = (int16_t)((u.ux0 - 3) & ~3);
    u.wcell = (int16_t)wcell;
    u.cell0 = a;
    out.push_back(u);
  }
}

}  // namespace

int build_plan(const mcs_extractor_params& p, int W, int H, Plan& pl) {
  if (W <= 0 || H <= 0 || p.nlevels < 1 || p.nlevels > kMaxLevels || p.nfeatures < 0 ||
      !(p.scale_factor > 1.0f)) {
    set_error("invalid extractor parameters");
    return MCS_ERR_ARG;
  }
  if (p.desc_size != 16 && p.desc_size != 32 && p.desc_size != 64) {
    set_error("desc_size must be 16, 32 or 64 (src/cTracking.cpp:133)");
    return MCS_ERR_ARG;
  }
  // FastFeatureDetector types TYPE_5_8 = 0, TYPE_7_12 = 1, TYPE_9_16 = 2.  AGAST
  // (AgastFeatureDetector's generated decision trees, OpenCV) is not implemented.
  if (p.use_agast) {
    set_error("AGAST (useAgast != 0) is not implemented; FAST types 0, 1, 2 are");
    return MCS_ERR_UNSUPPORTED;
  }
  if (p.fast_agast_type < 0 || p.fast_agast_type > 2) {
    set_error("fastAgastType must be 0 (TYPE_5_8), 1 (TYPE_7_12) or 2 (TYPE_9_16)");
    return MCS_ERR_ARG;
  }
  pl.p = p;
  pl.W = W; pl.H = H; pl.nlevels = p.nlevels;
  pl.scale_factor = (double)p.scale_factor;

  // scale tables (ctor :153-162) and budgets (:167-179)
  double sf[kMaxLevels], isf[kMaxLevels];
  sf[0] = 1; isf[0] = 1;
  for (int i = 1; i < p.nlevels; i++) sf[i] = sf[i - 1] * pl.scale_factor;
  const double inv = 1.0 / pl.scale_factor;
  for (int i = 1; i < p.nlevels; i++) isf[i] = isf[i - 1] * inv;
  int nfl[kMaxLevels];
  {
    const double factor = 1.0 / pl.scale_factor;
    double nd = p.nfeatures * (1 - factor) / (1 - std::pow(factor, p.nlevels));
    int sum = 0;
    for (int l = 0; l < p.nlevels - 1; l++) { nfl[l] = cv_round(nd); sum += nfl[l]; nd *= factor; }
    nfl[p.nlevels - 1] = std::max(p.nfeatures - sum, 0);
  }

  int64_t pyr_off = 0, img_off = 0, mask_off = 0;
  auto align = [](int64_t v, int64_t a) { return (v + a - 1) / a * a; };
  int32_t slot = 0, sel = 0;
  pl.cells.clear(); pl.fast_units.clear(); pl.xofs.clear(); pl.yofs.clear(); pl.alpha.clear(); pl.beta.clear();
  pl.xtab_off.assign(p.nlevels, 0); pl.ytab_off.assign(p.nlevels, 0);
  pl.max_cells_level = 0;
  for (int l = 0; l < p.nlevels; l++) {
    LevelPlan& L = pl.lv[l];
    L.w = cv_round((double)W * isf[l]);
    L.h = cv_round((double)H * isf[l]);
    if (L.w > 4095 + 2 * kMinBorder || L.h > 4095 + 2 * kMinBorder) {
      set_error("level too large for 12-bit candidate packing");
      return MCS_ERR_UNSUPPORTED;
    }
    L.bpitch = (int32_t)align(L.w, 64);
    L.pitch = (l == 0) ? W : L.bpitch;
    L.pyr_off = (l == 0) ? 0 : pyr_off;
    if (l > 0) pyr_off = align(pyr_off + (int64_t)L.pitch * L.h, 256);
    L.img_off = img_off;
    img_off = align(img_off + (int64_t)L.bpitch * L.h, 256);
    L.mask_off = mask_off;
    mask_off = align(mask_off + (int64_t)L.bpitch * L.h, 256);
    L.nfeat = nfl[l];
    L.scale = (float)sf[l];
    L.patch_size_scaled = (int)(kPatchSize * sf[l]);

    if (l > 0) {
      const LevelPlan& S = pl.lv[l - 1];
      pl.xtab_off[l] = (int64_t)pl.xofs.size();
      pl.ytab_off[l] = (int64_t)pl.yofs.size();
      linear_tables(S.w, S.h, L.w, L.h, pl);
      // OpenCV 3.1 VResizeLinearVec_32s8u: 16-wide SSE2 loop (x <= w-16), then 4-wide
      // (x < w-4); the rest uses the scalar FixedPtCast form.
      int x = 0;
      for (; x <= L.w - 16; x += 16) {}
      for (; x < L.w - 4; x += 4) {}
      L.simd_end = x;
    } else {
      L.simd_end = 0;
    }

    // FAST cell grid (:876-948)
    const int maxBX = L.w - kEdgeThreshold + 3, maxBY = L.h - kEdgeThreshold + 3;
    const double width = maxBX - kMinBorder, height = maxBY - kMinBorder;
    const int nCols = (int)(width / 30.0), nRows = (int)(height / 30.0);
    if (nCols < 1 || nRows < 1) {
      set_error("pyramid level smaller than one 30px FAST cell (reference divides by zero)");
      return MCS_ERR_UNSUPPORTED;
    }
    const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
    if (wCell > kMaxCellDim || hCell > kMaxCellDim) {
      set_error("FAST cell larger than the kernel's 64px window bound");
      return MCS_ERR_UNSUPPORTED;
    }
    L.cell_begin = (int32_t)pl.cells.size();
    L.cand_off = slot;
    for (int i = 0; i < nRows; i++) {
      const double iniY = kMinBorder + i * hCell;
      double maxY = iniY + hCell + 6;
      if (iniY >= maxBY - 3) continue;
      if (maxY > maxBY) maxY = maxBY;
      for (int j = 0; j < nCols; j++) {
        const double iniX = kMinBorder + j * wCell;
        double maxX = iniX + wCell + 6;
        if (iniX >= maxBX - 6) continue;
        if (maxX > maxBX) maxX = maxBX;
        CellDesc c;
        c.level = l;
        c.wx0 = (int16_t)((int)iniX + 3); c.wx1 = (int16_t)((int)maxX - 3);
        c.wy0 = (int16_t)((int)iniY + 3); c.wy1 = (int16_t)((int)maxY - 3);
        const int ww = std::max(0, c.wx1 - c.wx0), wh = std::max(0, c.wy1 - c.wy0);
        pl.max_win_w = std::max(pl.max_win_w, ww);
        pl.max_win_h = std::max(pl.max_win_h, wh);
        c.slot_off = slot;
        c.slot_cap = ((ww + 1) / 2) * ((wh + 1) / 2);
        slot += c.slot_cap;
        pl.cells.push_back(c);
      }
    }
    L.cell_end = (int32_t)pl.cells.size();
    L.cand_cap = slot - L.cand_off;
    pl.unit_begin[l] = (int32_t)pl.fast_units.size();
    // k_fast_rows work units: every cell row split into the fewest equal runs of cells whose
    // detection span (+3 px halo each side) fits one wave's lanes 0..62
    L.wcell = wCell;
    for (int c = L.cell_begin; c < L.cell_end;) {
      int e = c;
      while (e < L.cell_end && pl.cells[e].wy0 == pl.cells[c].wy0) e++;
      split_runs(pl.cells, c, e, l, wCell, pl.fast_units);
      c = e;
    }
    pl.max_cells_level = std::max(pl.max_cells_level, L.cell_end - L.cell_begin);
    if (L.cell_end - L.cell_begin > kMaxCellsPerLevel) {
      set_error("too many FAST cells in one level");
      return MCS_ERR_UNSUPPORTED;
    }

    // octree domain (:954-957 -> :641-643)
    L.width_rel = maxBX - kMinBorder;
    L.height_rel = maxBY - kMinBorder;
    L.nini = cv_round((double)L.width_rel / L.height_rel);
    if (L.nini < 1) {
      set_error("octree nIni == 0 (level taller than 2x its width): reference indexes out of range");
      return MCS_ERR_UNSUPPORTED;
    }
    L.hx = (double)L.width_rel / L.nini;
    // even, so every level starts at an even selection index (k_orient_desc pairs keypoints
    // 2j, 2j+1 in one wave and needs them on one level)
    const int cap = (std::max(L.nfeat + 3, 4 * L.nini) + 1) & ~1;
    if (cap > kOctMaxL) {
      set_error("per-level feature budget exceeds the octree kernel's node bound (1024)");
      return MCS_ERR_UNSUPPORTED;
    }
    L.sel_off = sel;
    L.sel_cap = cap;
    sel += cap;
  }
  for (int l = p.nlevels; l <= kMaxLevels; l++) pl.unit_begin[l] = (int32_t)pl.fast_units.size();
  pl.pyr_frame_bytes = pyr_off;
  pl.img_frame_bytes = img_off;
  pl.mask_frame_bytes = mask_off;
  pl.slots_per_frame = slot;
  pl.cand_per_frame = slot;
  pl.sel_per_frame = sel;
  return MCS_OK;
}

void build_masked_units(const Plan& pl, const uint8_t* mask_pyr, std::vector<FastUnit>& live,
                        std::vector<FastUnit>& dead) {
  for (int l = 0; l < pl.nlevels; l++) {
    const LevelPlan& L = pl.lv[l];
    const uint8_t* m = mask_pyr + L.mask_off;
    auto cell_live = [&](const CellDesc& cd) {
      for (int y = cd.wy0; y < cd.wy1; y++)
        for (int x = cd.wx0; x < cd.wx1; x++)
          if (m[(int64_t)y * L.bpitch + x]) return true;
      return false;
    };
    for (int c = L.cell_begin; c < L.cell_end;) {
      int e = c;
      while (e < L.cell_end && pl.cells[e].wy0 == pl.cells[c].wy0) e++;
      int a0 = -1, a1 = -1;
      for (int k = c; k < e; k++)
        if (cell_live(pl.cells[k])) { if (a0 < 0) a0 = k; a1 = k + 1; }
      if (a0 < 0) {
        zero_runs(pl.cells, c, e, l, L.wcell, dead);
      } else {
        zero_runs(pl.cells, c, a0, l, L.wcell, dead);
        split_runs(pl.cells, a0, a1, l, L.wcell, live);
        zero_runs(pl.cells, a1, e, l, L.wcell, dead);
      }
      c = e;
    }
  }
}

}  // namespace mcs
