// Host orchestration of the MI355X feature extractor (C-ABI of include/mcs_extractor.h):
// pyramid+blur -> FAST cells -> octree -> orientation + rotated BRIEF, batched over many
// camera-frames resident in HBM.  Kernels: k_pyramid.hip, k_fast_rows.hip, k_octree.hip,
// k_desc.hip.
//
// Reference path (billamiable/MultiCol-SLAM-Annotation):
//   mdBRIEFextractorOct::operator()        src/mdBRIEFextractorOct.cpp:1244-1337
//   ComputePyramid                         :1158-1201   -> k_pyr_rows, k_mask_nearest
//   ComputeKeyPointsOctTree (FAST part)    :863-949     -> k_fast_rows
//   DistributeOctTree / DivideNode         :569-861     -> k_octree
//   computeOrientation / IC_Angle          :221-248     -> k_orient_desc (part 1)
//   boxFilter 5x5                          :1301        -> k_pyr_rows (fused)
//   compute_ORB / rotatePattern            :285-354     -> k_orient_desc (part 2)
#include "common.hpp"
#include "extractor_plan.hpp"
#include "extractor_kernels.hpp"
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

namespace mcs {

// ===========================================================================
// host side
// ===========================================================================
template <typename T>
static int dalloc(T** p, size_t count, size_t pad_bytes = 256) {
  *p = nullptr;
  MCS_HIP_CHECK(hipMalloc((void**)p, count * sizeof(T) + pad_bytes));
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
  mcs::FastUnit* d_units = nullptr;
  // workspace
  uint8_t* d_pyr = nullptr;      // [F][pyr_frame_bytes]   raw levels 1..L-1 (pitch align64)
  uint8_t* d_blur = nullptr;     // [F][img_frame_bytes]   blurred levels 0..L-1
  uint32_t* d_slots = nullptr;   // [F][slots_per_frame]   FAST survivors per cell
  int32_t* d_cell_counts = nullptr;  // [F][ncells]
  uint32_t* d_cand = nullptr;    // [F][cand_per_frame]    gathered candidates per level
  int32_t* d_cnode = nullptr;    // [F][cand_per_frame]
  uint32_t* d_sel = nullptr;     // [F][sel_per_frame]     octree selection per level
  int32_t* d_sel_count = nullptr;  // [F][nlevels]
  // masks: registered set + single-call slot, each with per-cell window bitmaps
  uint8_t* d_mask_pyr = nullptr; int n_masks = 0;
  mcs::FastUnit* d_munits = nullptr; int64_t munit_stride = 0;   // per-mask FAST units
  uint8_t* d_mask_single = nullptr;
  // single-frame staging
  uint8_t* d_in = nullptr;
  mcs_keypoint* d_kps = nullptr; uint8_t* d_desc = nullptr; int32_t* d_count = nullptr;
  uint8_t* d_dmask = nullptr;
  // camera models (dBRIEF / mdBRIEF)
  mcs_cam_model* d_cams = nullptr; int n_cams = 0;
  // side stream for the level-0 blur (overlaps the resize chain; see run_batch)
  hipStream_t side = nullptr; hipEvent_t ev_fork = nullptr, ev_join = nullptr;
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

static void fill_level_ptrs(const Plan& pl, LevelPtrs& lp) {
  for (int l = 0; l < kMaxLevels; l++) {
    const bool v = l < pl.nlevels;
    lp.w[l] = v ? pl.lv[l].w : 0; lp.h[l] = v ? pl.lv[l].h : 0;
    lp.pitch[l] = v ? pl.lv[l].pitch : 0; lp.bpitch[l] = v ? pl.lv[l].bpitch : 0;
    lp.pyr_off[l] = v ? pl.lv[l].pyr_off : 0; lp.img_off[l] = v ? pl.lv[l].img_off : 0;
    lp.mask_off[l] = v ? pl.lv[l].mask_off : 0;
  }
}

static inline void stage_mark(mcs_extractor* h, int stage, hipStream_t st) {
  if (!h->timing || h->ev_count >= mcs_extractor::kRing) return;
  (void)hipEventRecord(h->ev[h->ev_count * (MCS_EXTRACTOR_NSTAGES + 1) + stage], st);
}

// Core batched pipeline on device buffers.
static int run_batch(mcs_extractor* h, const uint8_t* d_images, int F, const uint8_t* mask_pyr,
                     const int32_t* d_mask_index, mcs_keypoint* d_kps,
                     int32_t* d_counts, uint8_t* d_desc, uint8_t* d_desc_masks,
                     const int32_t* d_cam_index, hipStream_t st) {
  const Plan& pl = h->plan;
  const int nl = pl.nlevels;
  const int64_t img0_fs = (int64_t)pl.W * pl.H;
  auto pyr_args = [&](int l) {
    PyrArgs a;
    const LevelPlan& D = pl.lv[l];
    if (l == 0) {
      a.src = d_images; a.src_fstride = img0_fs; a.sw = D.w; a.sh = D.h; a.spitch = D.pitch;
      a.dst = nullptr; a.dst_fstride = 0; a.dpitch = 0;
      a.xofs = nullptr; a.alpha = nullptr; a.yofs = nullptr; a.beta = nullptr; a.simd_end = 0;
    } else {
      const LevelPlan& S = pl.lv[l - 1];
      a.src = (l == 1) ? d_images : h->d_pyr + S.pyr_off;
      a.src_fstride = (l == 1) ? img0_fs : pl.pyr_frame_bytes;
      a.sw = S.w; a.sh = S.h; a.spitch = S.pitch;
      a.dst = h->d_pyr + D.pyr_off; a.dst_fstride = pl.pyr_frame_bytes; a.dpitch = D.pitch;
      a.xofs = h->d_xofs + pl.xtab_off[l]; a.alpha = h->d_alpha + 2 * pl.xtab_off[l];
      a.yofs = h->d_yofs + pl.ytab_off[l]; a.beta = h->d_beta + 2 * pl.ytab_off[l];
      a.simd_end = D.simd_end;
    }
    a.blur = h->d_blur + D.img_off; a.blur_fstride = pl.img_frame_bytes; a.bpitch = D.bpitch;
    a.dw = D.w; a.dh = D.h;
    pyr_strips(D.w, D.h, F, a);
    a.nframes = F;
    return a;
  };
  // K2 arguments (row-streaming FAST; one launch per level, units of a level are contiguous)
  FastRowArgs fa;
  fa.img0 = d_images; fa.img0_fstride = img0_fs;
  fa.pyr = h->d_pyr; fa.pyr_fstride = pl.pyr_frame_bytes;
  fa.mask_pyr = mask_pyr; fa.mask_fstride = pl.mask_frame_bytes;
  fa.mask_index = d_mask_index;
  fa.nmasks = (mask_pyr && mask_pyr == h->d_mask_pyr) ? h->n_masks : 1;
  fa.cells = h->d_cells; fa.ncells = (int)pl.cells.size();
  fa.slots = h->d_slots; fa.slots_fstride = pl.slots_per_frame;
  fa.cell_counts = h->d_cell_counts;
  fa.threshold = std::min(std::max(pl.p.fast_threshold, 0), 255);
  fa.pattern = pl.p.fast_agast_type == 2 ? 16 : pl.p.fast_agast_type == 1 ? 12 : 8;
  fa.frame_count = d_counts;
  fa.nframes = F;
  fill_level_ptrs(pl, fa.lp);
  const bool wide = pl.scale_factor > 1.5;
  // Schedule (one stream): the resize chain K1+K5 level by level, the level-0 blur, then FAST
  // of every level in one launch.  (FAST per level on a second stream beside the chain was
  // measured slower: 1.85 -> 2.0-2.1 ms per step; the chain then loses its Infinity-Cache
  // reuse of level l-1 and its CU slots.)
  // The level-0 blur depends on the input only: on the side stream it runs beside the chain
  // (sharing the chain's level-0 reads while level 1 streams them, and filling the CUs the
  // small levels 4..7 leave idle); FAST joins both.  With stage timing on, the serial order
  // (the stage events need one stream).
  const bool use_side = !h->timing;
  if (use_side && !h->side) {
    MCS_HIP_CHECK(hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking));
    MCS_HIP_CHECK(hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming));
    MCS_HIP_CHECK(hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming));
  }
  stage_mark(h, 0, st);
  if (use_side) {
    MCS_HIP_CHECK(hipEventRecord(h->ev_fork, st));
    MCS_HIP_CHECK(hipStreamWaitEvent(h->side, h->ev_fork, 0));
    launch_pyr_blur(pyr_args(0), false, false, h->side);   // blur of level 0 (the input frames)
    MCS_HIP_CHECK(hipEventRecord(h->ev_join, h->side));
  }
  for (int l = 1; l < nl; l++) launch_pyr_blur(pyr_args(l), true, wide, st);
  stage_mark(h, 1, st);
  if (use_side) MCS_HIP_CHECK(hipStreamWaitEvent(st, h->ev_join, 0));
  else launch_pyr_blur(pyr_args(0), false, false, st);  // blur of level 0 (the input frames)
  stage_mark(h, 2, st);
  {
    FastRowArgs fl = fa;
    const bool per_mask = mask_pyr && mask_pyr == h->d_mask_pyr && h->d_munits;
    fl.units = per_mask ? h->d_munits : h->d_units;
    fl.nunits = per_mask ? (int)h->munit_stride : (int)pl.fast_units.size();
    fl.unit_mstride = per_mask ? h->munit_stride : 0;
    launch_fast_rows(fl, st);   // also zeroes d_counts
  }
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
    oa.nframes = F;
    int maxl = 0;
    for (int l = 0; l < nl; l++) maxl = std::max(maxl, pl.lv[l].sel_cap);
    launch_octree(oa, maxl, st);
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
    da.nframes = F;
    da.mode = pl.p.learn_masks ? 2 : (pl.p.do_dbrief ? 1 : 0);
    da.do_dbrief = pl.p.do_dbrief ? 1 : 0;
    da.cams = h->d_cams; da.cam_index = d_cam_index;
    da.desc_masks = d_desc_masks;
    if (da.mode != 0 && !h->d_cams) {
      set_error("dBRIEF / mdBRIEF need camera models (mcs_extractor_set_cam_models)");
      return MCS_ERR_ARG;
    }
    if (d_desc_masks && da.mode != 2)   // Mat::zeros (:1213-1215)
      MCS_HIP_CHECK(hipMemsetAsync(d_desc_masks, 0, (size_t)F * pl.sel_per_frame * pl.p.desc_size, st));
    launch_orient_desc(da, st);
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
  if (!(pl.scale_factor <= kMaxScaleFactor)) {
    delete h; set_error("scale_factor > 2.2 exceeds the pyramid kernel's source tile"); return MCS_ERR_UNSUPPORTED;
  }
  static bool consts_done[64] = {false};
  if (device < 64 && !consts_done[device]) {
    if ((rc = upload_desc_constants()) != MCS_OK) { delete h; return rc; }
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
  ALLOC(h->d_units, pl.fast_units.size());
  ALLOC(h->d_pyr, F * pl.pyr_frame_bytes);
  ALLOC(h->d_blur, F * pl.img_frame_bytes);
  ALLOC(h->d_slots, F * pl.slots_per_frame);
  ALLOC(h->d_cell_counts, F * pl.cells.size());
  ALLOC(h->d_cand, F * pl.cand_per_frame);
  ALLOC(h->d_cnode, F * pl.cand_per_frame);
  ALLOC(h->d_sel, F * pl.sel_per_frame);
  ALLOC(h->d_sel_count, F * pl.nlevels);
  ALLOC(h->d_mask_single, pl.mask_frame_bytes);
  ALLOC(h->d_in, (size_t)width * height);
  ALLOC(h->d_kps, pl.sel_per_frame);
  ALLOC(h->d_desc, (size_t)pl.sel_per_frame * pl.p.desc_size);
  ALLOC(h->d_count, 1);
  ALLOC(h->d_dmask, (size_t)pl.sel_per_frame * pl.p.desc_size);
#undef ALLOC
  hipError_t e = hipSuccess;
  if (e == hipSuccess) e = hipMemcpy(h->d_xofs, pl.xofs.data(), pl.xofs.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(h->d_alpha, pl.alpha.data(), pl.alpha.size() * 2, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(h->d_yofs, pl.yofs.data(), pl.yofs.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(h->d_beta, pl.beta.data(), pl.beta.size() * 2, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(h->d_cells, pl.cells.data(), pl.cells.size() * sizeof(CellDesc), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(h->d_units, pl.fast_units.data(), pl.fast_units.size() * sizeof(FastUnit), hipMemcpyHostToDevice);
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
  void* ptrs[] = {h->d_xofs, h->d_alpha, h->d_yofs, h->d_beta, h->d_cells, h->d_units, h->d_pyr, h->d_blur,
                  h->d_slots, h->d_cell_counts, h->d_cand, h->d_cnode, h->d_sel, h->d_sel_count,
                  h->d_mask_pyr, h->d_munits, h->d_mask_single, h->d_in,
                  h->d_kps, h->d_desc, h->d_count, h->d_dmask, h->d_cams};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (h->side) (void)hipStreamDestroy(h->side);
  if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
  if (h->ev_join) (void)hipEventDestroy(h->ev_join);
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
  if (h->d_munits) { MCS_HIP_CHECK(hipFree(h->d_munits)); h->d_munits = nullptr; }
  h->n_masks = 0;
  h->munit_stride = 0;
  if (n_masks == 0) return MCS_OK;
  const Plan& pl = h->plan;
  int rc = dalloc(&h->d_mask_pyr, (size_t)n_masks * pl.mask_frame_bytes);
  if (rc) return rc;
  launch_mask_pyramids(pl, d_masks, n_masks, h->d_mask_pyr, (hipStream_t)stream);
  MCS_HIP_CHECK(hipGetLastError());
  // FAST units per mask (registration time, once per camera): cells without a mask pixel only
  // zero their count, and every wave of the batch kernel covers live cells
  std::vector<uint8_t> hm((size_t)n_masks * pl.mask_frame_bytes);
  MCS_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
  MCS_HIP_CHECK(hipMemcpy(hm.data(), h->d_mask_pyr, hm.size(), hipMemcpyDeviceToHost));
  std::vector<std::vector<FastUnit>> lists(n_masks);
  size_t stride = 0;
  for (int m = 0; m < n_masks; m++) {
    std::vector<FastUnit> dead;
    build_masked_units(pl, hm.data() + (size_t)m * pl.mask_frame_bytes, lists[m], dead);
    lists[m].insert(lists[m].end(), dead.begin(), dead.end());   // heavy units first
    stride = std::max(stride, lists[m].size());
  }
  stride = std::max<size_t>(stride, 1);
  FastUnit pad{};   // no cells, no rows: the wave exits without a store
  std::vector<FastUnit> all((size_t)n_masks * stride, pad);
  for (int m = 0; m < n_masks; m++) std::copy(lists[m].begin(), lists[m].end(), all.begin() + (size_t)m * stride);
  if ((rc = dalloc(&h->d_munits, all.size())) != MCS_OK) return rc;
  MCS_HIP_CHECK(hipMemcpy(h->d_munits, all.data(), all.size() * sizeof(FastUnit), hipMemcpyHostToDevice));
  h->munit_stride = (int64_t)stride;
  h->n_masks = n_masks;
  return MCS_OK;
}

int mcs_extractor_set_cam_models(mcs_extractor* h, const mcs_cam_model* models, int32_t n) {
  if (!h || n < 0 || (n > 0 && !models)) return MCS_ERR_ARG;
  for (int i = 0; i < n; i++)
    if (models[i].p_deg < 1 || models[i].p_deg > 16 || models[i].invp_deg < 1 ||
        models[i].invp_deg > 16) {
      set_error("camera polynomial length must be 1..16");
      return MCS_ERR_ARG;
    }
  MCS_HIP_CHECK(hipSetDevice(h->device));
  if (h->d_cams) { MCS_HIP_CHECK(hipFree(h->d_cams)); h->d_cams = nullptr; }
  h->n_cams = 0;
  if (n == 0) return MCS_OK;
  int rc = dalloc(&h->d_cams, (size_t)n);
  if (rc) return rc;
  MCS_HIP_CHECK(hipMemcpy(h->d_cams, models, sizeof(mcs_cam_model) * n, hipMemcpyHostToDevice));
  h->n_cams = n;
  return MCS_OK;
}

int mcs_extract_batch_device_ex(mcs_extractor* h, const uint8_t* d_images, int32_t n_frames,
                                const int32_t* d_cam_index, mcs_keypoint* d_kps,
                                int32_t* d_counts, uint8_t* d_desc, uint8_t* d_desc_masks,
                                void* stream) {
  if (!h || !d_images || !d_kps || !d_counts || !d_desc || n_frames < 1) {
    set_error("null argument"); return MCS_ERR_ARG;
  }
  if (n_frames > h->max_frames) { set_error("n_frames > max_frames"); return MCS_ERR_CAPACITY; }
  MCS_HIP_CHECK(hipSetDevice(h->device));
  const uint8_t* mp = h->n_masks > 0 ? h->d_mask_pyr : nullptr;
  return run_batch(h, d_images, n_frames, mp, mp ? d_cam_index : nullptr, d_kps, d_counts,
                   d_desc, d_desc_masks, h->n_cams > 1 ? d_cam_index : nullptr,
                   (hipStream_t)stream);
}

int mcs_extract_batch_device(mcs_extractor* h, const uint8_t* d_images, int32_t n_frames,
                             const int32_t* d_mask_index, mcs_keypoint* d_kps,
                             int32_t* d_counts, uint8_t* d_desc, void* stream) {
  return mcs_extract_batch_device_ex(h, d_images, n_frames, d_mask_index, d_kps, d_counts,
                                     d_desc, nullptr, stream);
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
    // level 0 of the single-call mask pyramid doubles as the upload buffer
    MCS_HIP_CHECK(hipMemcpy2D(h->d_mask_single, pl.lv[0].bpitch, mask, mask_stride, pl.W, pl.H,
                              hipMemcpyHostToDevice));
    launch_mask_pyramids(pl, h->d_mask_single, 1, h->d_mask_single, st);
    MCS_HIP_CHECK(hipGetLastError());
    mp = h->d_mask_single;
  }
  const bool learn = pl.p.learn_masks != 0;
  int rc = run_batch(h, h->d_in, 1, mp, nullptr, h->d_kps, h->d_count, h->d_desc,
                     learn ? h->d_dmask : nullptr, nullptr, st);
  if (rc) return rc;
  int32_t n = 0;
  MCS_HIP_CHECK(hipMemcpy(&n, h->d_count, sizeof(n), hipMemcpyDeviceToHost));
  *n_out = n;
  if (n > kps_cap) { set_error("kps_cap too small"); return MCS_ERR_CAPACITY; }
  if (n > 0) {
    if (kps) MCS_HIP_CHECK(hipMemcpy(kps, h->d_kps, sizeof(mcs_keypoint) * n, hipMemcpyDeviceToHost));
    if (desc) MCS_HIP_CHECK(hipMemcpy(desc, h->d_desc, (size_t)n * pl.p.desc_size, hipMemcpyDeviceToHost));
    if (desc_masks) {
      if (learn)
        MCS_HIP_CHECK(hipMemcpy(desc_masks, h->d_dmask, (size_t)n * pl.p.desc_size, hipMemcpyDeviceToHost));
      else
        std::memset(desc_masks, 0, (size_t)n * pl.p.desc_size);
    }
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
    int sp;
    if (stage == 0) {
      src = level == 0 ? h->last_img0 + (int64_t)frame * pl.W * pl.H
                       : h->d_pyr + (int64_t)frame * pl.pyr_frame_bytes + L.pyr_off;
      sp = L.pitch;
    } else {
      src = h->d_blur + (int64_t)frame * pl.img_frame_bytes + L.img_off;
      sp = L.bpitch;
    }
    MCS_HIP_CHECK(hipMemcpy2D(dst, L.w, src, sp, L.w, L.h, hipMemcpyDeviceToHost));
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
