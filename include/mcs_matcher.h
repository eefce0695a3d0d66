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

#ifdef __cplusplus
}
#endif
#endif /* MCS_MATCHER_H */
