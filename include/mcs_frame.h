/*
 * mcs_frame.h -- C-ABI of the cMultiFrame work around the extractor, on the device.
 *
 * Replaces (reference paths relative to billamiable/MultiCol-SLAM-Annotation):
 *   cMultiFrame::cMultiFrame bearing rays: cCamModelGeneral_::ImgToWorld per keypoint
 *       src/cMultiFrame.cpp:143-152, src/cam_model_omni.cpp:49-67     -> mcs_keypoint_rays_device
 *   cMultiFrame::cMultiFrame concatenation of the cameras (mvKeys, mvKeysRays, descriptors,
 *       keypoint_to_cam, cont_idx_to_local_cam_idx) and PosInGrid
 *       src/cMultiFrame.cpp:166-184, :342-353                         -> mcs_multiframe_concat_device
 *   cMultiFrame::isInFrustum src/cMultiFrame.cpp:218-270 (WorldToCamHom_fast
 *       src/cam_system_omni.cpp:92-112, isPointInMirrorMask src/cam_model_omni.cpp:165-180,
 *       distance invariance src/cMapPoint.cpp:498-508)              -> mcs_is_in_frustum_device
 *
 * All pointers are device memory; calls are asynchronous on `stream` (hipStream_t, NULL =
 * default).  Double precision throughout with the reference's operation order (no FMA).
 */
#ifndef MCS_FRAME_H
#define MCS_FRAME_H

#include <stdint.h>
#include "mcs_common.h"
#include "mcs_extractor.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Bearing ray (unit 3-vector) of every keypoint of a batch: ray = ImgToWorld((double)kp.x,
 * (double)kp.y) with the frame's camera model.  d_kps [n_frames][cap], d_counts [n_frames],
 * d_cam_index [n_frames] (nullable = camera 0), d_cams [n_cams] camera models.
 * Out: d_rays [n_frames][cap][3] (slots >= count untouched). */
int mcs_keypoint_rays_device(const mcs_keypoint* d_kps, const int32_t* d_counts, int32_t n_frames,
                             int32_t cap, const int32_t* d_cam_index, const mcs_cam_model* d_cams,
                             double* d_rays, void* stream);

/* Concatenate the cameras of n_mf multi-frames in camera order (c = 0..n_cams-1).  Inputs per
 * multi-frame m and camera c: d_counts [n_mf][n_cams], d_kps [n_mf][n_cams][cap], d_rays
 * [..][cap][3] (nullable), d_desc [..][cap][desc_bytes] (nullable); d_grid_params [n_cams][4]
 * = {mnMinX, mnMinY, mfGridElementWidthInv, mfGridElementHeightInv}.  Outputs per multi-frame
 * (row stride n_cams * cap): d_keys (mvKeys), d_keys_rays (nullable), d_descs (nullable),
 * d_kp_to_cam (keypoint_to_cam), d_cont_to_local (cont_idx_to_local_cam_idx), d_grid_pos
 * (posX | posY << 8, or -1 when PosInGrid fails, nullable), d_total [n_mf] (totalN). */
int mcs_multiframe_concat_device(const int32_t* d_counts, int32_t n_mf, int32_t n_cams, int32_t cap,
                                 const mcs_keypoint* d_kps, const double* d_rays,
                                 const uint8_t* d_desc, int32_t desc_bytes,
                                 const double* d_grid_params, mcs_keypoint* d_keys,
                                 double* d_keys_rays, uint8_t* d_descs, int32_t* d_kp_to_cam,
                                 int32_t* d_cont_to_local, int32_t* d_grid_pos, int32_t* d_total,
                                 void* stream);

/* isInFrustum for every (map point, camera) of one frame: project with (M_t M_c)^-1 and
 * WorldToImg, reject outside the level-0 mirror mask, outside [0.8 minDist, 1.2 maxDist] of
 * the camera centre, predict the scale level by lower_bound over the scale factors.
 * d_pose [6] frame M_t (Cayley + t), d_mc [n_cams][6], d_cam [n_cams][17] (c,d,e,u0,v0,invP
 * [12]), d_masks [n_cams][mask_h][mask_w] (level-0 mirror masks, pitch mask_w), d_pts
 * [n][3], d_normals [n][3], d_dist [n][2] (mfMinDistance, mfMaxDistance), d_scale [n_levels]
 * (mvScaleFactors).  Outputs [n][n_cams]: d_in_view (mbTrackInView), d_proj [..][2]
 * (mTrackProjX/Y), d_level (mnTrackScaleLevel), d_view_cos (mTrackViewCos); the last three
 * are written only where in view. */
int mcs_is_in_frustum_device(const double* d_pose, const double* d_mc, const double* d_cam,
                             int32_t n_cams, const uint8_t* d_masks, int32_t mask_w,
                             int32_t mask_h, const double* d_pts, const double* d_normals,
                             const double* d_dist, int32_t n, const double* d_scale,
                             int32_t n_levels, uint8_t* d_in_view, double* d_proj,
                             int32_t* d_level, double* d_view_cos, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MCS_FRAME_H */
