/*
 * mcs_mappoint.h -- C-ABI of the map-point refresh LocalBundleAdjustment runs after its
 * write-back (src/cOptimizer.cpp:885-902: for every local point with >= 2 edges,
 * SetWorldPos, then UpdateNormalAndDepth and ComputeDistinctiveDescriptors), batched over
 * points on the device.
 *
 * Replaces (billamiable/MultiCol-SLAM-Annotation):
 *   cMapPoint::ComputeDistinctiveDescriptors(bool havingMasks)   src/cMapPoint.cpp:297-390,
 *       decl include/cMapPoint.h:80 (median: include/misc.h:97-105)
 *   cMapPoint::UpdateNormalAndDepth()                           src/cMapPoint.cpp:453-496,
 *       decl include/cMapPoint.h:90 (GetCameraCenter: src/cMultiKeyFrame.cpp:159-165)
 *
 * Observations are given per point as CSR lists in the order the reference visits its
 * std::map<cMultiKeyFrame*, ...> (the caller's map order; bad keyframes already dropped for
 * ComputeDistinctiveDescriptors, as the reference skips them).  All pointers are device
 * memory; calls are asynchronous on `stream` (hipStream_t, NULL = default).
 */
#ifndef MCS_MAPPOINT_H
#define MCS_MAPPOINT_H

#include <stdint.h>
#include "mcs_common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ComputeDistinctiveDescriptors for n_points points: point p's descriptors are rows
 * d_obs_row[d_obs_ptr[p] .. d_obs_ptr[p+1]) of d_desc ([rows][bytes], bytes = 16, 32 or 64);
 * d_masks (nullable, same layout) = havingMasks (DescriptorDistance64Masked).  Among the
 * N descriptors the one whose median distance to the LATER ones (row i of the upper triangle,
 * j > i; median = element N-1-i >> 1 in sorted order) is smallest wins, the first on ties;
 * N <= 2 -> 0; N = 0 -> -1 (the reference returns without touching the point).
 * Out: d_best[p] (index within the point's list); d_out_desc / d_out_mask (nullable,
 * [n_points][bytes]) = the chosen descriptor / mask (rows of points with N = 0 untouched). */
int mcs_distinctive_descriptors_device(const uint8_t* d_desc, const uint8_t* d_masks, int32_t bytes,
                                       const int32_t* d_obs_ptr, const int32_t* d_obs_row,
                                       int32_t n_points, int32_t* d_best, uint8_t* d_out_desc,
                                       uint8_t* d_out_mask, void* stream);

/* UpdateNormalAndDepth for n_points points at positions d_points [n][3]: observing keyframes
 * d_obs_kf[d_obs_ptr[p] .. d_obs_ptr[p+1]) (map order), keyframe centres d_kf_center
 * [n_kf][3] (the translation of M_t, GetCameraCenter), reference keyframe d_ref_kf[p] and
 * d_ref_level[p] = octave of the reference keyframe's first observation of the point, or -1
 * when it holds none (the reference then uses level 1); d_scale [n_levels] = mvScaleFactors.
 * Out: d_normal [n][3] (mean of the unit viewing rays), d_min_dist, d_max_dist [n]
 * (mfMinDistance, mfMaxDistance).  Points with no observation are left untouched. */
int mcs_update_normal_depth_device(const double* d_points, int32_t n_points,
                                   const int32_t* d_obs_ptr, const int32_t* d_obs_kf,
                                   const double* d_kf_center, const int32_t* d_ref_kf,
                                   const int32_t* d_ref_level, const double* d_scale,
                                   int32_t n_levels, double* d_normal, double* d_min_dist,
                                   double* d_max_dist, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MCS_MAPPOINT_H */
