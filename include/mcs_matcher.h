/*
 * mcs_matcher.h -- C-ABI drop-in boundary for the binary-descriptor matcher.
 *
 * Replaces (billamiable/MultiCol-SLAM-Annotation):
 *   int DescriptorDistance64(const uint64_t*, const uint64_t*, const int& dim)
 *                                                include/cORBmatcher.h:43-45, src/cORBmatcher.cpp:2443-2455
 *   int DescriptorDistance64Masked(...)          include/cORBmatcher.h:48-52, src/cORBmatcher.cpp:2457-2477
 *   the O(N1*N2) Hamming loop + selection of cORBmatcher::SearchForTriangulationRaw
 *                                                include/cORBmatcher.h:111-117, src/cORBmatcher.cpp:968-1156
 *   the best / second-best Hamming scans of the windowed matchers (SearchByProjection
 *   src/cORBmatcher.cpp:67-163, WindowSearch :326-475) -> mcs_hamming_top2_*.
 *
 * `dim` / `bytes` is the descriptor length in BYTES (the reference passes featDim = 32
 * and loops dim/8 uint64 words).  Device entry points are asynchronous on `stream`.
 */
#ifndef MCS_MATCHER_H
#define MCS_MATCHER_H

#include <stdint.h>
#include "mcs_common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Exact reference semantics; returns the distance (not a status). */
int mcs_descriptor_distance64(const uint64_t* d1, const uint64_t* d2, int32_t dim);
int mcs_descriptor_distance64_masked(const uint64_t* d1, const uint64_t* d2, const uint64_t* m1,
                                     const uint64_t* m2, int32_t dim);

/* Dense distances D[i*nb + j] = Hamming(A_i, B_j) (uint16), device buffers. */
int mcs_hamming_dense_device(const uint8_t* d_a, int32_t na, const uint8_t* d_b, int32_t nb,
                             int32_t bytes, uint16_t* d_dist, void* stream);

/* For each query i: best = min distance over all train rows (ties -> lowest train index),
 * second = second smallest distance counting multiplicity (ORB-SLAM bestDist/bestDist2
 * update rule), second_idx its train index.  nt == 0 -> best_idx = -1, dists = 256*8+1. */
int mcs_hamming_top2_device(const uint8_t* d_q, int32_t nq, const uint8_t* d_t, int32_t nt,
                            int32_t bytes, int32_t* d_best_idx, int32_t* d_best_dist,
                            int32_t* d_second_idx, int32_t* d_second_dist, void* stream);

/* Batched top-2 straight on the extractor's batch output: descriptor sets are
 * d_desc[set][cap][bytes] with d_counts[set] valid rows; pair p matches set
 * d_pairs[2p] (queries) against set d_pairs[2p+1] (train).  Outputs [n_pairs][cap]. */
int mcs_hamming_top2_batch_device(const uint8_t* d_desc, const int32_t* d_counts,
                                  const int32_t* d_pairs, int32_t n_pairs, int32_t cap,
                                  int32_t bytes, int32_t* d_best_idx, int32_t* d_best_dist,
                                  int32_t* d_second_idx, int32_t* d_second_dist, void* stream);

/* SearchForTriangulationRaw, match-list part (src/cORBmatcher.cpp:968-1156, with
 * mbCheckOrientation = false as constructed by the reference, include/cORBmatcher.h:40):
 * for each unmatched keypoint of KF1 (in index order), brute-force over unmatched
 * keypoints of KF2 of the SAME camera, keep dist <= th_low, visit candidates in
 * (dist, idx2) order up to cvRound(2*best), accept the first passing
 * CheckDistEpipolarLine(ray1, ray2, E[cam1][cam2], epi_thresh) (src/misc.cpp:54-70).
 * Host buffers: desc1 n1 x bytes, cam1 n1, has_mp1 n1 (nonzero = already has a map point),
 * rays1 n1 x 3 doubles; same for KF2; E = ncams*ncams 3x3 row-major doubles (E[c1][c2]).
 * Output matches12[n1] (-1 = none); *n_matches.  Distances are computed on the GPU. */
int mcs_search_for_triangulation_raw(const uint8_t* desc1, const int32_t* cam1,
                                     const uint8_t* has_mp1, const double* rays1, int32_t n1,
                                     const uint8_t* desc2, const int32_t* cam2,
                                     const uint8_t* has_mp2, const double* rays2, int32_t n2,
                                     int32_t ncams, const double* E, int32_t bytes,
                                     int32_t th_low, double epi_thresh, int32_t* matches12,
                                     int32_t* n_matches);

/* Same with mdBRIEF descriptor masks (cORBmatcher built with havingMasks = true, whose
 * TH_LOW is floor(featDim), src/cORBmatcher.cpp:52-65): distances are
 * DescriptorDistance64Masked(d1, d2, m1, m2) (src/cORBmatcher.cpp:1052-1056, 2457-2477).
 * mask1 [n1][bytes], mask2 [n2][bytes] host, both required.  Both entries reject
 * n2 >= 2^19 and cameras outside [0, ncams) with MCS_ERR_ARG (the device search keeps a
 * vbMatched2 bitmap of KF2 in LDS). */
int mcs_search_for_triangulation_raw_masked(const uint8_t* desc1, const uint8_t* mask1,
                                            const int32_t* cam1, const uint8_t* has_mp1,
                                            const double* rays1, int32_t n1,
                                            const uint8_t* desc2, const uint8_t* mask2,
                                            const int32_t* cam2, const uint8_t* has_mp2,
                                            const double* rays2, int32_t n2, int32_t ncams,
                                            const double* E, int32_t bytes, int32_t th_low,
                                            double epi_thresh, int32_t* matches12,
                                            int32_t* n_matches);

/* Device-resident SearchForTriangulationRaw for CreateNewMapPoints' neighbour loop
 * (src/cLocalMapping.cpp:223-266 -> src/cORBmatcher.cpp:968-1156): the same match list as
 * the two host entries above, on device buffers and stream-ordered (no host synchronisation),
 * so a caller keeps KF descriptors, rays and has-map-point flags resident and runs one call per
 * neighbour keyframe, updating d_has_mp1 between calls as the reference's triangulation does.
 * d_mask1 / d_mask2: both null (ORB, DescriptorDistance64) or both set (mdBRIEF, ...Masked).
 * d_E [ncams][ncams][9] (mcs_compute_e_rig).  Out: d_matches12[n1] (-1 = none), *d_n_matches.
 * Keypoints whose camera lies outside [0, ncams) never match (the host entries reject them).
 * The workspace holds per-query candidate slots; n1 <= max_n1, n2 <= max_n2 < 2^19, ncams <= 8. */
typedef struct mcs_tri_workspace mcs_tri_workspace;
int mcs_tri_workspace_create(int32_t device, int32_t max_n1, int32_t max_n2, mcs_tri_workspace** out);
void mcs_tri_workspace_destroy(mcs_tri_workspace* ws);
int mcs_search_for_triangulation_raw_device(mcs_tri_workspace* ws, const uint8_t* d_desc1,
                                            const uint8_t* d_mask1, const int32_t* d_cam1,
                                            const uint8_t* d_has_mp1, const double* d_rays1,
                                            int32_t n1, const uint8_t* d_desc2,
                                            const uint8_t* d_mask2, const int32_t* d_cam2,
                                            const uint8_t* d_has_mp2, const double* d_rays2,
                                            int32_t n2, int32_t ncams, const double* d_E,
                                            int32_t bytes, int32_t th_low, double epi_thresh,
                                            int32_t* d_matches12, int32_t* d_n_matches,
                                            void* stream);

/* The essential matrices SearchForTriangulationRaw precomputes per camera pair
 * (src/cORBmatcher.cpp:985-998): E[i][j] = ComputeE(KF1.Get_MtMc_inv(i), KF2.Get_MtMc(j))
 * (src/misc.cpp:72-86), the rig poses given as the Cayley 6-vectors the keyframes hold
 * (cMultiCamSys_::Set_M_t_from_min, src/cam_system_omni.cpp:170-183): mt1, mt2 [6],
 * mc [ncams][6].  Out: E [ncams][ncams][9] row-major, the `E` input of the two entries above.
 * Host math in the reference's cv::Matx operation order. */
int mcs_compute_e_rig(const double* mt1, const double* mt2, const double* mc, int32_t ncams,
                      double* E);

/* CheckDistEpipolarLine(ray1, ray2, E12, thresh) (src/misc.cpp:54-70): 1 = passes (squared
 * epipolar distance < thresh), 0 = fails (or den == 0), < 0 = argument error.  The check the
 * triangulation entries apply to every candidate. */
int mcs_check_dist_epipolar_line(const double* ray1, const double* ray2, const double* E12,
                                 double thresh);

/* ---- Projection-guided (windowed) matching -------------------------------------------
 * cMultiFrame feature grid (src/cMultiFrame.cpp:154-184, PosInGrid :342-353; 64 x 48 cells
 * per camera, include/cMultiFrame.h FRAME_GRID_COLS / FRAME_GRID_ROWS) and
 * GetFeaturesInArea (:272-340), feeding the best / second-best Hamming scans of
 *   SearchByProjection(F, vpMapPoints, th)          src/cORBmatcher.cpp:67-166   (rule 0)
 *   SearchByProjection(CurrentFrame, LastFrame, th) src/cORBmatcher.cpp:1991-2123 (rule 1)
 *   SearchForInitialization(F1, F2, ...)            src/cORBmatcher.cpp:579-726  (rule 2)
 *   WindowSearch(F1, F2, windowSize, ...)           src/cORBmatcher.cpp:326-473  (rule 3)
 * with checkOrientation = false (include/cORBmatcher.h:40).
 * Split: the grid is built on the host (it is part of the cMultiFrame constructor); the
 * device enumerates every query's window candidates in the reference's order (cells ix-major,
 * then iy, then insertion order) and computes their Hamming distances; the host applies the
 * reference's sequential selection rule (it depends on earlier queries' assignments). */
#define MCS_GRID_COLS 64
#define MCS_GRID_ROWS 48

/* grid_params[cam] = {min_x, min_y, grid_w_inv, grid_h_inv} (mnMinX, mnMinY,
 * mfGridElementWidthInv, mfGridElementHeightInv).  kp_xy [n_kp][2] float (cv::KeyPoint.pt),
 * kp_cam [n_kp].  Out: cell_ptr [n_cams*64*48 + 1] (cell = (cam*64 + ix)*48 + iy), cell_kp
 * [n_kp] (keypoints outside the grid are dropped; *n_in_grid entries used).  Host memory. */
int mcs_frame_grid_build(const float* kp_xy, const int32_t* kp_cam, int32_t n_kp, int32_t n_cams,
                         const double* grid_params, int32_t* cell_ptr, int32_t* cell_kp,
                         int32_t* n_in_grid);

/* Device window search.  Queries: q_xyr [nq][3] doubles (x, y, r), q_cam_lvl [nq][3]
 * (cam, minLevel, maxLevel; -1/-1 = any level), q_desc [nq][bytes] (+ q_mask nullable).
 * Keypoints: kp_xy [n][2] float, kp_octave [n], kp_desc [n][bytes] (+ kp_mask nullable; with
 * masks the distance is DescriptorDistance64Masked).  Grid: device copies of the
 * mcs_frame_grid_build outputs and grid_params.  Out: cand_ptr [nq+1], cand_kp / cand_dist
 * [cap]; *total = number of candidates (MCS_ERR_CAPACITY if > cap; nothing else written).
 * Synchronises `stream` once to read the total. */
int mcs_window_search_device(const int32_t* d_cell_ptr, const int32_t* d_cell_kp,
                             const double* d_grid_params, int32_t n_cams, const float* d_kp_xy,
                             const int32_t* d_kp_octave, const uint8_t* d_kp_desc,
                             const uint8_t* d_kp_mask, int32_t bytes, int32_t nq,
                             const double* d_q_xyr, const int32_t* d_q_cam_lvl,
                             const uint8_t* d_q_desc, const uint8_t* d_q_mask,
                             int32_t* d_cand_ptr, int32_t* d_cand_kp, int32_t* d_cand_dist,
                             int64_t cap, int64_t* total, void* stream);

/* Host selection over the candidate lists (queries in the reference's loop order).
 * rule 0: SearchByProjection(F, MPs): skip assigned keypoints, best / second with octaves,
 *         accept best <= th unless (same octave and best > nnratio * second), assign.
 * rule 1: SearchByProjection(Current, Last): skip assigned keypoints, best only,
 *         accept best <= th, assign.
 * rule 2: SearchForInitialization: skip candidates whose vMatchedDistance <= dist, accept
 *         best <= th and best < second * nnratio, a re-matched train keypoint drops its
 *         previous query.
 * rule 3: WindowSearch: skip keypoints matched earlier in the call, accept
 *         best <= second * nnratio and best <= th, assign.
 * th = TH_HIGH (rules 0, 1, 3) or TH_LOW (rule 2) of cORBmatcher (src/cORBmatcher.cpp:46-65).
 * kp_assigned [n_kp] in/out (rules 0, 1, 3: keypoint already holds a map point).  match [nq]
 * out (keypoint index or -1; rule 2: vnMatches12).  *n_matches = match count. */
int mcs_window_select(int32_t rule, int32_t nq, const int32_t* cand_ptr, const int32_t* cand_kp,
                      const int32_t* cand_dist, const int32_t* kp_octave, int32_t n_kp,
                      int32_t th, double nnratio, uint8_t* kp_assigned, int32_t* match,
                      int32_t* n_matches);

/* Host-buffer entry point for the reference's call sites (cv::Mat / std::vector data): builds
 * the grid, uploads the frame and the queries, runs mcs_window_search_device and
 * mcs_window_select on `device` (no CPU fallback).  kp_assigned may be NULL (= none). */
typedef struct mcs_window_frame {
  int32_t n_cams, n_kp, bytes;
  const double* grid_params;     /* [n_cams][4], as above */
  const float* kp_xy;            /* [n_kp][2] mvKeys pt */
  const int32_t* kp_cam;         /* [n_kp] keypoint_to_cam */
  const int32_t* kp_octave;      /* [n_kp] */
  const uint8_t* desc;           /* [n_kp][bytes] mDescriptors in camera order */
  const uint8_t* desc_mask;      /* nullable [n_kp][bytes] mDescriptorMasks (mdBRIEF) */
} mcs_window_frame;
int mcs_window_match(int32_t device, int32_t rule, const mcs_window_frame* frame, int32_t nq,
                     const double* q_xyr, const int32_t* q_cam_lvl, const uint8_t* q_desc,
                     const uint8_t* q_mask, int32_t th, double nnratio, uint8_t* kp_assigned,
                     int32_t* match, int32_t* n_matches);

#ifdef __cplusplus
}
#endif
#endif /* MCS_MATCHER_H */
