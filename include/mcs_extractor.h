/*
 * mcs_extractor.h -- C-ABI drop-in boundary for the MultiCol-SLAM feature extractor.
 *
 * Replaces (reference paths relative to billamiable/MultiCol-SLAM-Annotation):
 *   mdBRIEFextractorOct::mdBRIEFextractorOct(...)      include/mdBRIEFextractorOct.h:339-351
 *   mdBRIEFextractorOct::operator()(image, mask, kps,   include/mdBRIEFextractorOct.h:355-361
 *        camModel, desc, descMasks)                     src/mdBRIEFextractorOct.cpp:1244-1337
 *   the per-camera OpenMP loop of cMultiFrame::cMultiFrame  src/cMultiFrame.cpp:128-139
 *     (-> mcs_extract_batch_device: all cameras of many multi-frames in one call)
 *
 * Conventions: plain pointers and sizes, no exceptions, every entry point returns an
 * mcs_status (0 == MCS_OK).  Host buffers are caller-allocated (the reference callee
 * allocated via OutputArray::create, src/mdBRIEFextractorOct.cpp:1277-1280; here the
 * caller asks mcs_extractor_capacity() first).  An extractor handle owns mutable device
 * workspace and is NOT re-entrant (same as the reference object, which owns its
 * pyramid): use one handle per camera thread, or the batch entry point.
 */
#ifndef MCS_EXTRACTOR_H
#define MCS_EXTRACTOR_H

#include <stdint.h>
#include "mcs_common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Constructor arguments of mdBRIEFextractorOct, same order and meaning
 * (include/mdBRIEFextractorOct.h:339-351).  edge_threshold, first_level, score_type and
 * patch_size are accepted but, as in the reference, unused (the compile-time constants
 * EDGE_THRESHOLD=25 / PATCH_SIZE=32 of src/mdBRIEFextractorOct.cpp:84-86 apply). */
typedef struct mcs_extractor_params {
  int32_t nfeatures;       /* 1000 default */
  float scale_factor;      /* 1.2 default; stored as double((float)x) like the reference */
  int32_t nlevels;         /* 8 */
  int32_t edge_threshold;  /* 25 (unused) */
  int32_t first_level;     /* 0 (unused) */
  int32_t score_type;      /* 0 HARRIS / 1 FAST: only logged by the reference (unused) */
  int32_t patch_size;      /* 32 (unused) */
  int32_t fast_threshold;  /* 20 (5 for the initialisation extractor) */
  int32_t use_agast;       /* must be 0 (AGAST: MCS_ERR_UNSUPPORTED) */
  int32_t fast_agast_type; /* FastFeatureDetector type: 2 TYPE_9_16 (default), 1 TYPE_7_12,
                              0 TYPE_5_8 (mdBRIEFextractorOct.cpp:871-872, 916-917) */
  int32_t do_dbrief;       /* 1 = dBRIEF (needs mcs_extractor_set_cam_models) */
  int32_t learn_masks;     /* 1 = mdBRIEF: 3 rotated patterns -> descriptor + stability mask
                              (src/mdBRIEFextractorOct.cpp:410-554; needs camera models) */
  int32_t desc_size;       /* bytes: 16, 32 or 64 */
} mcs_extractor_params;

/* Field order and layout of cv::KeyPoint (pt.x, pt.y, size, angle, response, octave,
 * class_id), 28 bytes. */
typedef struct mcs_keypoint {
  float x, y, size, angle, response;
  int32_t octave, class_id;
} mcs_keypoint;

/* Scaramuzza omni camera model (cCamModelGeneral_, include/cam_model_omni.h:36-147,
 * src/cam_model_omni.cpp:49-163), needed by the dBRIEF / mdBRIEF descriptors: keypoints are
 * undistorted with ImgToWorld (undistortPointsOcam, scale p[0]) and the rotated pattern is
 * re-distorted with WorldToImg at z = -p[0] (distortPointsOcam). */
typedef struct mcs_cam_model {
  double c, d, e, u0, v0;        /* affine parameters and principal point */
  int32_t p_deg, invp_deg;       /* number of coefficients in p / invp (<= 16 each) */
  double p[16];                  /* forward polynomial (ImgToWorld); p[0] = p1 */
  double invp[16];               /* inverse polynomial (WorldToImg), Horner in theta */
} mcs_cam_model;

typedef struct mcs_extractor mcs_extractor;

/* Fill *p with the reference constructor defaults (include/mdBRIEFextractorOct.h:339-351). */
void mcs_extractor_default_params(mcs_extractor_params* p);

/* Create an extractor for width x height 8-bit frames; reserves device workspace for up
 * to max_frames camera-frames per batch call.  device = HIP device ordinal. */
int mcs_extractor_create(const mcs_extractor_params* p, int32_t width, int32_t height,
                         int32_t max_frames, int32_t device, mcs_extractor** out);
void mcs_extractor_destroy(mcs_extractor* h);

/* Upper bound on keypoints one frame can produce (sum over levels of
 * max(N_l + 3, 4 * nIni_l)); size kps/desc buffers with it. */
int32_t mcs_extractor_capacity(const mcs_extractor* h);
/* Per-level geometry: wh[2*l] = width, wh[2*l+1] = height; nfeat[l] = level budget. */
int mcs_extractor_levels(const mcs_extractor* h, int32_t* nlevels, int32_t* wh, int32_t* nfeat);

/* Single frame, host memory: drop-in for mdBRIEFextractorOct::operator().
 * image: height rows of `stride` bytes; mask: NULL (no mask, like an empty cv::Mat) or
 * height rows of `mask_stride` bytes (nonzero == usable).  On return *n_out keypoints in
 * level order with desc_size-byte descriptors (row-major).  desc_masks (nullable) is
 * zero-filled like the reference ORB path.  If *n_out > kps_cap -> MCS_ERR_CAPACITY. */
int mcs_extract(mcs_extractor* h, const uint8_t* image, int32_t stride, const uint8_t* mask,
                int32_t mask_stride, mcs_keypoint* kps, int32_t kps_cap, int32_t* n_out,
                uint8_t* desc, uint8_t* desc_masks);

/* Register static per-camera masks (device memory, n_masks x height x width, pitch =
 * width).  Their pyramids are built once (the reference rebuilds them per frame,
 * src/mdBRIEFextractorOct.cpp:1182-1197).  n_masks = 0 clears. */
int mcs_extractor_set_masks_device(mcs_extractor* h, const uint8_t* d_masks, int32_t n_masks,
                                   void* stream);

/* Batch, device-resident (HBM in, HBM out), asynchronous on `stream` (hipStream_t, NULL =
 * default).  d_images: n_frames x height x width (pitch = width).  d_mask_index: per
 * frame index into the registered masks, or NULL => mask 0 if masks are registered, no
 * mask otherwise.  Outputs: d_kps [n_frames][cap], d_counts [n_frames],
 * d_desc [n_frames][cap][desc_size], cap = mcs_extractor_capacity(). */
int mcs_extract_batch_device(mcs_extractor* h, const uint8_t* d_images, int32_t n_frames,
                             const int32_t* d_mask_index, mcs_keypoint* d_kps,
                             int32_t* d_counts, uint8_t* d_desc, void* stream);

/* Camera models for the dBRIEF / mdBRIEF descriptors (do_dbrief / learn_masks), one per
 * camera; a frame uses the model of its mask index (model 0 for mcs_extract).  Host memory,
 * copied.  Required before extracting with do_dbrief or learn_masks set. */
int mcs_extractor_set_cam_models(mcs_extractor* h, const mcs_cam_model* models, int32_t n);

/* mcs_extract_batch_device with the descriptor masks of mdBRIEF (learn_masks; all-zero for
 * ORB and dBRIEF, as the reference's Mat::zeros): d_desc_masks [n_frames][cap][desc_size]
 * (nullable).  d_cam_index doubles as mask and camera-model index. */
int mcs_extract_batch_device_ex(mcs_extractor* h, const uint8_t* d_images, int32_t n_frames,
                                const int32_t* d_cam_index, mcs_keypoint* d_kps,
                                int32_t* d_counts, uint8_t* d_desc, uint8_t* d_desc_masks,
                                void* stream);

/* Stage read-back for parity tests (synchronous; reads the workspace of the LAST batch
 * or single-frame call).  stage 0: pyramid level image (w*h bytes, row-major);
 * stage 1: 5x5-blurred level image; stage 2: FAST candidates of the level in reference
 * order as int32 triples (x_rel, y_rel, score), coordinates relative to minBorder=22
 * (src/mdBRIEFextractorOct.cpp:876-945); stage 3: octree selection of the level as int32
 * triples in output order.  *n_out = element count (bytes for 0/1, triples for 2/3). */
int mcs_extractor_read_stage(mcs_extractor* h, int32_t stage, int32_t frame, int32_t level,
                             void* dst, int64_t cap, int64_t* n_out);

/* Live per-stage device timing (hipEvents recorded on the call's stream around each
 * stage of every batch call; no host synchronisation inside the call).  Stages:
 * 0 pyramid = resize + blur of levels 1..L-1 (k_pyr_rows<true> x L-1), 1 blur of level 0
 * (k_pyr_rows<false>), 2 FAST (k_fast_rows), 3 octree (k_octree),
 * 4 orientation + descriptor (k_orient_desc).
 * read_timing synchronises, returns the summed milliseconds per stage over the recorded
 * calls and their number, and optionally resets.  At most 256 calls are kept. */
#define MCS_EXTRACTOR_NSTAGES 5
int mcs_extractor_enable_timing(mcs_extractor* h, int32_t enable);
int mcs_extractor_read_timing(mcs_extractor* h, float* ms_per_stage, int32_t* ncalls,
                              int32_t reset);

/* HarrisResponses (src/mdBRIEFextractorOct.cpp:86-132), opt-in: the reference never calls it
 * from ComputeKeyPointsOctTree (scoreType is stored, unused), so it is not part of
 * mcs_extract*; callers that want Harris responses compute them here.  d_level_ptrs
 * [n_levels] device addresses of u8 level images, d_level_geom [n_levels][3] = {w, h, pitch};
 * d_kps [n] in LEVEL coordinates with octave = level; reads outside a level use its
 * BORDER_REFLECT_101 mirror (the reference's padded levels).  Out: d_response [n] floats with
 * the reference's float expression order.  block_size in [1, 45]. */
int mcs_harris_responses_device(const uint64_t* d_level_ptrs, const int32_t* d_level_geom,
                                int32_t n_levels, const mcs_keypoint* d_kps, int32_t n,
                                int32_t block_size, float harris_k, float* d_response,
                                void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MCS_EXTRACTOR_H */
