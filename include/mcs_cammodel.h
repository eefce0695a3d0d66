/*
 * mcs_cammodel.h -- mirror masks of the omnidirectional camera model (libmcs_amd.so).
 *
 * Replaces:
 *   CreateMirrorMask(cCamModelGeneral_ camera, int pyrLevel, vector<Mat>& mirror_masks)
 *       reference src/cam_model_omni.cpp:183-222, decl include/cam_model_omni.h:252;
 *       called from cSystem::LoadMCS src/cSystem.cpp:164-172 with pyrLevel = 4 when
 *       Camera.mirrorMask == 1 (otherwise a single all-ones Iw x Ih mask).
 *   cCamModelGeneral_::isPointInMirrorMask(u, v, pyr)
 *       reference src/cam_model_omni.cpp:165-180, decl include/cam_model_omni.h:169;
 *       called by the matchers (src/cORBmatcher.cpp:513,1204,1300,...) and
 *       cMultiFrame::isInFrustum (src/cMultiFrame.cpp:230).
 *
 * Layout: the masks of all levels are packed level after level (row-major u8, 255 inside the
 * mirror circle, 0 outside); level l has widths[l] x heights[l] pixels starting at offsets[l].
 * Level sizes follow cv::buildPyramid: ((w+1)/2, (h+1)/2) per step.
 */
#ifndef MCS_CAMMODEL_H
#define MCS_CAMMODEL_H

#include <stdint.h>
#include "mcs_common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Level sizes and byte offsets of the packed mask pyramid (levels in 1..4, the reference's
 * offset table has 4 entries). Any output pointer may be NULL. */
int mcs_mirror_mask_layout(int32_t width, int32_t height, int32_t levels, int32_t* widths,
                           int32_t* heights, int64_t* offsets, int64_t* total_bytes);

/* CreateMirrorMask on the device: writes the packed pyramid into d_masks (total_bytes from
 * mcs_mirror_mask_layout). cam_u0/cam_v0 are the camera's Camera.u0/Camera.v0 (the reference
 * swaps them: row centre and radius base = (float)v0, column centre = (float)u0, see
 * src/cam_model_omni.cpp:189-190, 212-213). Asynchronous on `stream` (hipStream_t, NULL = default). */
int mcs_create_mirror_mask_device(double cam_u0, double cam_v0, int32_t width, int32_t height,
                                  int32_t levels, uint8_t* d_masks, void* stream);

/* isPointInMirrorMask against one level's HOST mask (cols x rows): 1 inside, 0 outside. */
int mcs_is_point_in_mirror_mask(const uint8_t* mask, int32_t cols, int32_t rows, double u,
                                double v);

#ifdef __cplusplus
}
#endif
#endif /* MCS_CAMMODEL_H */
