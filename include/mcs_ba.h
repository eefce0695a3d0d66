/*
 * mcs_ba.h -- C-ABI drop-in boundary for the MultiCol bundle adjustment.
 *
 * Replaces (billamiable/MultiCol-SLAM-Annotation):
 *   cOptimizer::LocalBundleAdjustment(pKF, pMap, nrIters, getCovMats, pbStopFlag)
 *       include/cOptimizer.h:61-65, src/cOptimizer.cpp:489-908   -> mcs_local_ba_select + mcs_local_ba_ex
 *   cOptimizer::BundleAdjustment / GlobalBundleAdjustment
 *       include/cOptimizer.h:50-59, src/cOptimizer.cpp:59-261     -> mcs_global_ba_select + mcs_global_ba
 *   cOptimizer::PoseOptimization(pFrame, inliers, huberMultiplier)
 *       include/cOptimizer.h:67-69, src/cOptimizer.cpp:264-486    -> mcs_pose_optimization_select
 *                                                                    + mcs_pose_optimization
 *   g2o::SparseOptimizer::initializeOptimization(0) + optimize(n) with
 *       OptimizationAlgorithmLevenberg + BlockSolver_6_3 + LinearSolverEigen and a
 *       SparseOptimizerTerminateAction        (ThirdParty/g2o/g2o/core)        -> mcs_ba_optimize
 *   EdgeProjectXYZ2MCS::computeError / linearizeOplus (+ mcsJacs1), VertexMt_cayley,
 *       VertexPointXYZ, VertexMc_cayley, VertexOmniCameraParameters
 *       include/g2o_MultiCol_vertices_edges.h:42-216, src/g2o_MultiCol_vertices_edges.cpp
 *
 * The host keeps the map traversal that builds the problem (local / fixed keyframe
 * selection, one edge per observation, :503-769) and the write-back (:859-903); this ABI
 * takes the resulting graph as flat SoA arrays.  Mc and IO vertices are fixed, as in
 * LocalBundleAdjustment (:636-664).  All doubles.  Status codes as mcs_common.h.
 */
#ifndef MCS_BA_H
#define MCS_BA_H

#include <stdint.h>
#include "mcs_common.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mcs_ba_problem {
  int32_t n_poses, n_points, n_edges, n_cams;
  const double* poses;        /* [n_poses][6] M_t as (r1,r2,r3,t1,t2,t3): Cayley + t, body->world */
  const uint8_t* pose_fixed;  /* [n_poses] 1 = fixed vertex */
  const double* points;       /* [n_points][3] world coordinates (marginalised vertices) */
  const double* mc;           /* [n_cams][6] M_c camera->body (Cayley + t), fixed */
  const double* cam;          /* [n_cams][17] c,d,e,u0,v0,invP[0..11] (VertexOmniCameraParameters) */
  const int32_t* edge_pose;   /* [n_edges] vertex 0 (Mt) */
  const int32_t* edge_point;  /* [n_edges] vertex 1 (point) */
  const int32_t* edge_cam;    /* [n_edges] vertices 2/3 (Mc, IO) */
  const double* edge_meas;    /* [n_edges][2] measured (distorted) pixel, kp.pt */
  const double* edge_info;    /* [n_edges] information = edge_info * I2 (invSigma2(octave)) */
  double huber_delta;         /* RobustKernelHuber delta: 1.345*2 (LocalBA), sqrt(5.991) (global) */
} mcs_ba_problem;

typedef struct mcs_ba_options {
  int32_t max_iterations;       /* optimize(n): 10 (LocalBA round 1), 15 (round 2) */
  double gain_threshold;        /* SparseOptimizerTerminateAction gain threshold: 1e-6 */
  int32_t terminate_max_iter;   /* SparseOptimizerTerminateAction max iterations: 15 */
  int32_t max_trials;           /* LM maxTrialsAfterFailure: 10 */
  double tau;                   /* LM lambda init factor: 1e-5 */
} mcs_ba_options;

typedef struct mcs_ba_report {
  int32_t iterations;           /* optimize() return value (iterations run) */
  int32_t stop_flag;            /* value of the (caller's or auxiliary) stop flag afterwards */
  double chi2_initial;          /* robust chi2 before the first iteration */
  double chi2_final;            /* robust chi2 at the final estimate */
  double lambda_final;
  int32_t n_active_edges;
  int32_t n_active_poses;       /* non-fixed poses with >= 1 active edge */
  int32_t n_active_points;
  double* trace_chi2;           /* nullable [trace_cap]: robust chi2 after each iteration */
  int32_t trace_cap;
} mcs_ba_report;

typedef struct mcs_ba_ctx mcs_ba_ctx;

void mcs_ba_default_options(mcs_ba_options* o);
/* Device context sized for problems up to the given counts (grown on demand). */
int mcs_ba_create(int32_t device, mcs_ba_ctx** out);
void mcs_ba_destroy(mcs_ba_ctx* c);

/* One initializeOptimization(0) + optimize(max_iterations) on the GPU.
 * poses/points: in/out (n_poses*6 / n_points*3 doubles), updated in place.
 * edge_level: in [n_edges], 0 = active edge (level 0), nonzero = disabled (level 1).
 * edge_chi2: out (nullable) unrobust chi2 e^T*Omega*e of every edge at the final estimate.
 * stop_flag: the caller's force-stop flag (nullable, like pbStopFlag); polled between LM
 * trials and written by the terminate action exactly as g2o does
 * (sparse_optimizer_terminate_action.cpp:21-72). */
int mcs_ba_optimize(mcs_ba_ctx* c, const mcs_ba_problem* p, const mcs_ba_options* o,
                    double* poses, double* points, const uint8_t* edge_level,
                    double* edge_chi2, volatile int32_t* stop_flag, mcs_ba_report* rep);

/* cOptimizer::LocalBundleAdjustment after graph construction (src/cOptimizer.cpp:771-903):
 * round 1 optimize(10); if the stop flag is set afterwards -> return (no write-back);
 * else disable edges with chi2 > delta^2, round 2 optimize(15), cull again.  stop_flag NULL
 * (pbStopFlag == NULL): the terminate action's auxiliary flag persists from round 1 into
 * round 2, as in g2o.  An empty active graph (optimize() == -1) returns without write-back.
 * Outputs: poses/points (in/out; only meaningful when *write_back == 1), edge_inlier[n_edges]
 * (0 = observation erased), write_back (bDoMore of the reference), reports of both rounds. */
int mcs_local_ba(mcs_ba_ctx* c, const mcs_ba_problem* p, double* poses, double* points,
                 uint8_t* edge_inlier, int32_t* write_back, volatile int32_t* stop_flag,
                 mcs_ba_report* rep_round1, mcs_ba_report* rep_round2);

/* mcs_local_ba with the reference's point bookkeeping (src/cOptimizer.cpp:798-903,
 * cMapPoint::EraseObservation src/cMapPoint.cpp:120-152, TotalNrObservations :166-178):
 * both culling passes walk the edges in order and skip edges of a point that has turned bad;
 * erasing an observation turns its point bad once fewer than 2 observations remain,
 * counting point_extra_obs[i] observations of point i from bad keyframes (edges exist only for
 * good keyframes; nullable = 0).  Edges of a point that turned bad stay active in round 2, as in
 * the reference.  point_write[i] (out) = the point is written back: write_back, not bad, more
 * than one remaining observation from good keyframes and >= 2 edges (:885-902). */
int mcs_local_ba_ex(mcs_ba_ctx* c, const mcs_ba_problem* p, const int32_t* point_extra_obs,
                    double* poses, double* points, uint8_t* edge_inlier, uint8_t* point_write,
                    int32_t* write_back, volatile int32_t* stop_flag, mcs_ba_report* rep_round1,
                    mcs_ba_report* rep_round2);

/* ---- LocalBundleAdjustment graph assembly (src/cOptimizer.cpp:503-769) ---------------------
 * The map as flat arrays (indices, not pointers).  Observation order per point is the
 * reference's std::map<cMultiKeyFrame*, vector<size_t>> iteration order (keyframe, then the
 * image points of that keyframe); map-point matches per keyframe are GetMapPointMatches(). */
typedef struct mcs_lba_map {
  int32_t n_kf;
  const int64_t* kf_id;       /* [n_kf] mnId */
  const uint8_t* kf_bad;      /* [n_kf] isBad() */
  const int32_t* kf_mp_off;   /* [n_kf + 1] CSR offsets into kf_mp */
  const int32_t* kf_mp;       /* map point matches (point index, -1 = NULL) */
  int32_t n_points;
  const uint8_t* pt_bad;      /* [n_points] isBad() */
  const int32_t* pt_obs_off;  /* [n_points + 1] CSR offsets into obs_kf */
  const int32_t* obs_kf;      /* observing keyframe of every observation */
} mcs_lba_map;

/* Outputs (caller-allocated arrays, counts written back).  Pose slots: the local keyframes
 * first (pKF, then its covisibles in order), then the fixed keyframes. */
typedef struct mcs_lba_graph {
  int32_t* local_kf;          /* [n_kf] */
  int32_t n_local;
  int32_t* fixed_kf;          /* [n_kf] */
  int32_t n_fixed;
  uint8_t* pose_fixed;        /* [n_kf] per pose slot: setFixed of the vertex */
  int32_t* points;            /* [n_points] local map points (vertex order) */
  int32_t n_points;
  int32_t* point_extra_obs;   /* [n_points] per local point: observations from bad keyframes */
  int32_t* edge_obs;          /* [edge_cap] observation index of every edge (vpEdges order) */
  int32_t* edge_pose;         /* [edge_cap] pose slot */
  int32_t* edge_point;        /* [edge_cap] local point slot */
  int32_t n_edges;
  int32_t edge_cap;
} mcs_lba_graph;

/* Local keyframes = pKF + every non-bad covisible keyframe (GetVectorCovisibleKeyFrames order,
 * :503-517); local points = first appearance over their map-point matches, non-bad (:521-537);
 * fixed keyframes = observers of local points that are neither local (bad covisibles count as
 * local) nor already fixed, non-bad (:540-558); vertex fixed flags follow the reference exactly:
 * a local keyframe is fixed iff mnId == 0, and `oneFixed` keeps only the LAST local keyframe's
 * test, so when that is false and there is no fixed keyframe pKF is fixed too (:585-612); one
 * edge per observation of a local point from a non-bad keyframe (:688-766).  cur_kf = pKF.
 * Returns MCS_OK, MCS_LBA_EMPTY when there is at most one local keyframe (the reference
 * returns without optimising, :519-520), or MCS_ERR_CAPACITY (n_edges > edge_cap; counts are
 * still written). */
#define MCS_LBA_EMPTY 1
int mcs_local_ba_select(const mcs_lba_map* m, int32_t cur_kf, const int32_t* covis,
                        int32_t n_covis, mcs_lba_graph* g);

/* ---- BundleAdjustment graph assembly (src/cOptimizer.cpp:101-234, write-back :240-259) -----
 * cOptimizer::GlobalBundleAdjustment (:59-69) calls BundleAdjustment(pMap->GetAllKeyFrames(),
 * pMap->GetAllMapPoints(), ...).  The two lists as flat arrays, in the caller's order (the
 * reference's std::set pointer order); each point's observations in its std::map<cMultiKeyFrame*,
 * vector<size_t>> iteration order (keyframe, then the image points of that keyframe). */
typedef struct mcs_gba_map {
  int32_t n_kf;               /* vpKFs.size() */
  const int64_t* kf_id;       /* [n_kf] mnId */
  const uint8_t* kf_bad;      /* [n_kf] isBad() */
  int32_t n_points;           /* vpMP.size() */
  const int64_t* pt_id;       /* [n_points] mnId (the key of mapPointId_to_cont_g2oId, :163-176) */
  const uint8_t* pt_bad;      /* [n_points] isBad() */
  const int32_t* pt_obs_off;  /* [n_points + 1] CSR offsets into obs_kf */
  const int32_t* obs_kf;      /* observing keyframe of every observation: index into vpKFs */
  int32_t n_cams;             /* vpKFs[0]->camSystem.GetNrCams() */
} mcs_gba_map;

/* Outputs (caller-allocated; counts written back).  Vertex ids are g2o's: keyframe mnId, then
 * the Mc, IO and point vertices from currVertexIdx = maxKF + 1 on (:103-176). */
typedef struct mcs_gba_graph {
  int32_t* pose_kf;           /* [n_kf] vpKFs index of every pose vertex (addVertex order) */
  uint8_t* pose_fixed;        /* [n_kf] setFixed: mnId == 0 (:119-120) */
  int32_t n_poses;
  int32_t* points;            /* [n_points] vpMP index of every point vertex (addVertex order) */
  int64_t* point_vertex_id;   /* [n_points] nullable: the g2o id of every point vertex */
  int32_t n_points;
  int64_t mc_vertex_id0;      /* id of camera 0's Mc vertex (maxMcid - nrCams); IO follows */
  int64_t io_vertex_id0;      /* id of camera 0's IO vertex (maxIOid - nrCams) */
  int32_t* kf_slot;           /* [n_kf] write-back (:242-249): pose slot of vpKFs[i], -1 if it has
                                 no pose vertex (a bad keyframe: the reference dereferences NULL) */
  int32_t* pt_slot;           /* [n_points] write-back (:252-259): point slot of vpMP[i] via
                                 mapPointId_to_cont_g2oId[mnId] (the last good point of that mnId),
                                 -1 if none (a bad point: the reference dereferences end()) */
  int32_t* edge_obs;          /* [edge_cap] observation index of every edge (addEdge order) */
  int32_t* edge_pose;         /* [edge_cap] pose slot */
  int32_t* edge_point;        /* [edge_cap] point slot */
  int32_t n_edges;
  int32_t edge_cap;
  int64_t collision_id;       /* out: first vertex id registered twice, -1 = none */
} mcs_gba_graph;

/* Pose vertices: every non-bad keyframe, in list order, id = mnId, fixed iff mnId == 0.  The
 * reference's `maxKF` rule (:104-132): `if (pKF->mnId > maxKFid) maxKF = pKF->mnId;` with
 * maxKFid never updated (0), so maxKF is the mnId of the LAST non-bad keyframe with mnId > 0
 * (0 if none) and the Mc / IO / point ids start at maxKF + 1 -- not at max(mnId) + 1.  When the
 * list is not id-ordered these ids can equal a keyframe's mnId; g2o's addVertex then refuses
 * the second vertex ("FATAL, a vertex with ID .. has already been registered", optimizable_
 * graph.cpp:243-250) and the edges bind whatever vertex holds the id: this returns
 * MCS_ERR_ARG with collision_id set and the message, and builds no edges.  Point vertices:
 * every non-bad point in list order (one id each, also for points without an edge), Huber
 * delta sqrt(5.991) and information I are the caller's (:161, :209).  Edges: one per
 * observation from a non-bad keyframe (:189-231); an observing keyframe without a pose vertex
 * is rejected (the reference would bind a NULL vertex).  An empty vpKFs is rejected
 * (the reference reads vpKFs[0]).  MCS_ERR_CAPACITY when n_edges > edge_cap (counts written). */
int mcs_global_ba_select(const mcs_gba_map* m, mcs_gba_graph* g);

/* ---- PoseOptimization graph assembly (src/cOptimizer.cpp:294-430) --------------------------
 * The frame's mvpMapPoints as indices: key_mp[i] = the map point of keypoint i (index into
 * pt_id) or -1 (NULL).  Vertex 0 = the frame pose, ids 1..nrCams the Mc vertices, then the IO
 * vertices, then one fixed point vertex per distinct map-point mnId in order of first
 * appearance (mapPt_2_obs_idx, :373-392).  One edge per non-NULL keypoint, in keypoint order
 * (:364-430), bad map points included (the reference does not test isBad here).  The caller
 * fills edge_meas = mvKeys[i].pt, edge_cam = keypoint_to_cam[i], edge_info =
 * mvInvLevelSigma2[mvKeys[i].octave] and huber_delta = 1.345 * huberMultiplier (:344, :398-406)
 * and passes the problem to mcs_pose_optimization; keypoints without an edge keep
 * mvbOutlier = false (:367). */
typedef struct mcs_po_frame {
  int32_t n_keys;             /* N = mvpMapPoints.size() */
  const int32_t* key_mp;      /* [n_keys] map point index or -1 */
  int32_t n_mp;
  const int64_t* pt_id;       /* [n_mp] mnId */
  int32_t n_cams;
} mcs_po_frame;

typedef struct mcs_po_graph {
  int32_t* points;            /* [n_mp] map point index of every point vertex */
  int64_t* point_vertex_id;   /* [n_mp] nullable */
  int32_t n_points;
  int32_t* edge_obs;          /* [edge_cap] keypoint index i of every edge (vnIndexEdge) */
  int32_t* edge_point;        /* [edge_cap] point slot */
  int32_t n_edges;
  int32_t edge_cap;
} mcs_po_graph;

int mcs_pose_optimization_select(const mcs_po_frame* f, mcs_po_graph* g);

/* cOptimizer::PoseOptimization (src/cOptimizer.cpp:264-486) after graph construction:
 * p->n_poses == 1 (the frame's M_t, optimised; pose_fixed is ignored), every map point fixed
 * (:382), Mc / IO fixed, Huber delta = p->huber_delta (1.345 * huberMultiplier, :344),
 * edge_info = invSigma2(octave) (:405-406).  optimize(10), edges with chi2 > delta^2 become
 * outliers and are disabled, optimize(10) again, the remaining edges are classified
 * (:432-474).  No force-stop flag is set, so the terminate action's auxiliary flag carries
 * over from round 1 to round 2 (a converged round 1 leaves round 2 without iterations).
 * pose: in/out [6]; outlier: out [n_edges] (mvbOutlier of the observations);
 * *n_good = nInitialCorrespondences - nBad (the reference's return value);
 * *bad_ratio = nBad / nInitialCorrespondences (its `inliers` output, nullable). */
int mcs_pose_optimization(mcs_ba_ctx* c, const mcs_ba_problem* p, double* pose, uint8_t* outlier,
                          int32_t* n_good, double* bad_ratio, mcs_ba_report* rep_round1,
                          mcs_ba_report* rep_round2);

/* Per-edge error and Jacobians (vertex order Mt, point) at the given estimate, for tests:
 * err [n][2], jac_pose [n][2][6], jac_point [n][2][3] (g2o sign: d(meas - proj)/d(param)). */
int mcs_ba_linearize(mcs_ba_ctx* c, const mcs_ba_problem* p, double* err, double* jac_pose,
                     double* jac_point);

/* ---- Global BA and point-sharded BA (config E) ------------------------------------------
 * cOptimizer::GlobalBundleAdjustment / BundleAdjustment (src/cOptimizer.cpp:59-261): every
 * MultiKeyFrame and map point, information = I (:209), Huber delta = sqrt(5.991) (:161),
 * keyframe mnId 0 fixed (:119-120, the caller sets pose_fixed), Mc / IO fixed, one
 * optimize(15) (:241; the nIterations argument is ignored by the reference), poseOnly fixes
 * every point (:178), results always written back (:244-261).
 *
 * Sharding: each rank holds a subset of the points with ALL of their edges;
 * poses are replicated.  Per LM trial every rank forms its partial Schur complement
 * S_r = Hpp_r - sum_{own points} Hpl Hll^-1 Hpl^T (lambda added by rank 0 only) and the
 * partial rhs; one in-place SUM all-reduce of [S tiles | b_schur] gives every rank the same
 * reduced camera system, which each rank factors redundantly (identical bits, no broadcast).
 * Points are back-substituted locally; chi2 and the model-decrease terms are all-reduced as
 * three scalars, so every rank takes the same LM decisions (lock step).
 *
 * The library never talks to the interconnect itself: `allreduce` (e.g. torch.distributed /
 * RCCL on the caller's side) reduces xchg[offset, offset + count) in place across ranks.  It is
 * called with the library's stream (hipStream_t) and returns 0 on success:
 *   stream_ordered == 0: the library synchronises its stream before every call and reads the
 *       buffer only after the callback returned (the callback completes the reduction);
 *   stream_ordered != 0: the library does NOT synchronise; the callback enqueues the
 *       reduction so that it starts after all work already on `stream` and completes before
 *       any work enqueued on `stream` after the call (RCCL on that stream, or a side stream
 *       joined by events) and may return before it has run.  The per-iteration exchanges of
 *       the reduced camera system then cost no host round trip; the LM-control scalars are
 *       reduced on the device too and read back once per trial.
 * Every rank issues the same sequence of calls (same offsets and counts). */
enum { MCS_REDUCE_SUM = 0, MCS_REDUCE_MAX = 1 };
typedef int32_t (*mcs_ba_allreduce_fn)(void* user, int32_t op, int64_t offset, int64_t count,
                                       void* stream);
typedef struct mcs_ba_shard {
  int32_t rank, world;
  double* xchg;                  /* device buffer of >= mcs_ba_xchg_doubles(n_poses) doubles */
  int64_t xchg_cap;              /* its size in doubles */
  mcs_ba_allreduce_fn allreduce;
  void* user;
  int32_t stream_ordered;        /* see above */
} mcs_ba_shard;

/* Exchange-buffer size (doubles) for problems with up to n_poses pose vertices. */
int64_t mcs_ba_xchg_doubles(int32_t n_poses);

/* mcs_ba_optimize over this rank's shard (shard == NULL or world == 1: single GPU). */
int mcs_ba_optimize_sharded(mcs_ba_ctx* c, const mcs_ba_problem* p, const mcs_ba_options* o,
                            double* poses, double* points, const uint8_t* edge_level,
                            double* edge_chi2, volatile int32_t* stop_flag, mcs_ba_report* rep,
                            const mcs_ba_shard* shard);

/* cOptimizer::BundleAdjustment after graph construction: optimize(15) with the terminate
 * action (gain 1e-6, max 15), pose_only = 1 fixes every point.  p->huber_delta and
 * p->edge_info are taken as given (the reference uses sqrt(5.991) and 1). */
int mcs_global_ba(mcs_ba_ctx* c, const mcs_ba_problem* p, int32_t pose_only, double* poses,
                  double* points, volatile int32_t* stop_flag, mcs_ba_report* rep,
                  const mcs_ba_shard* shard);

/* Stage timing (device time from HIP events on the context's stream; the exchange stage is
 * the stream time of the reduced-system all-reduce when the shard is stream_ordered, else the
 * host wall time around the callback).  Stages: 0 linearize (errors, Jacobians,
 * Hpp / Hll / b), 1 Schur (Hll^-1, Y = Hpl Hll^-1, reduced camera system), 2 exchange
 * (all-reduce of the reduced system, sharded runs only), 3 dense LDL^T solve, 4 update
 * (back-substitution, oplus, chi2).  ms[] accumulates over calls until read with reset. */
#define MCS_BA_NSTAGES 5
int mcs_ba_enable_timing(mcs_ba_ctx* c, int32_t on);
int mcs_ba_read_timing(mcs_ba_ctx* c, double* ms, int32_t* n_iterations, int32_t* n_trials,
                       int32_t* last_n, int32_t reset);

/* Host wall time of the host-side phases of the calls on this context (always accumulated):
 * 0 argument checks + active counts, 1 structure build (initializeOptimization +
 * buildStructure), 2 packing + upload of the problem, 3 waiting for the device + result
 * download, 4 LocalBA bookkeeping between the rounds (culling, re-masking).  ms[] accumulates
 * until read with reset. */
#define MCS_BA_NHOST 5
int mcs_ba_read_host_timing(mcs_ba_ctx* c, double* ms, int32_t* n_calls, int32_t reset);

/* Test hook: the structure of `p` (edges with edge_level != 0 inactive; NULL = all active)
 * built by the product (Schur pair lists and k_schur items on the device) against the host
 * restatement of BlockSolver::buildStructure's pairs (block pointers, every (e1, e2) pair in
 * order, every work item).  Returns the number of differing entries (0 = identical) or a
 * negative status. */
int mcs_ba_check_structure(mcs_ba_ctx* c, const mcs_ba_problem* p, const uint8_t* edge_level);

/* Test hook: the device Levenberg-Marquardt control of the product (the function the device-
 * driven optimisation runs after every trial: OptimizationAlgorithmLevenberg::solve's accept /
 * reject and lambda schedule, optimization_algorithm_levenberg.cpp:99-189, Raul's nBad stop,
 * and SparseOptimizerTerminateAction, sparse_optimizer_terminate_action.cpp:43-72) replayed on
 * scripted trial outcomes.  in3 = {initial robust chi2, max |diag Hll|, max |diag Hpp|};
 * trials [n][4] = {trial robust chi2, points' model decrease, poses' model decrease, solve
 * failed (0/1)}; out [n][10] per consumed trial = {lambda used, lambda after, ni, accepted,
 * qmax, nBad, iterations done, done, terminate flag, currentChi}; *n_out = trials consumed
 * (the replay stops when the optimisation is done). */
int mcs_ba_lm_replay(int32_t device, const mcs_ba_options* o, const double* in3, const double* trials,
                     int32_t n, double* out, int32_t* n_out);
/* Test hook: the per-landmark block of BlockSolver::solve (block_solver.hpp:381-403) through the
 * product's device helpers -- Dinv = (H + lambda I).inverse() in Eigen 3.2.10's fixed 3x3 order,
 * db = Dinv b, Y = Hpl Dinv -- for n independent (H[9], b[3], Hpl[18]) inputs, row-major.  Out:
 * Dinv[n][9], db[n][3], Y[n][18].  Pinned by tests/golden/g2o_schur.npz. */
int mcs_ba_point_block_eval(int32_t device, const double* H, double lambda, const double* b, const double* hpl,
                            int32_t n, double* Dinv, double* db, double* Y);
/* Test hook: the product's robust kernel (RobustKernelHuber::robustify,
 * robust_kernel_impl.cpp:78-91, delta^2 held as float as robust_kernel_impl.h:84 declares it) on
 * n squared errors: rho0 = rho(e), rho1 = rho'(e). */
int mcs_ba_huber_eval(int32_t device, const double* e, int32_t n, double delta, double* rho0, double* rho1);

/* Test hook for the dense reduced-camera solve (LinearSolverEigen::solve,
 * ThirdParty/g2o/g2o/solvers/linear_solver_eigen.h:94-126): S is n x n row-major (lower
 * triangle read), b and x length n.  *zero_pivot = 1 when the LDL^T meets an exact zero. */
int mcs_dense_ldlt_solve(int32_t device, const double* S, int32_t n, const double* b, double* x,
                         int32_t* zero_pivot);
/* Same, choosing the kernels: path 0 = what the BA uses (n <= 64: the fused one-tile solve,
 * else pad + the pipelined factorisation (one launch) over the tile band of S -- tiles below the
 * widest tile diagonal holding a non-zero are skipped, as the BA skips the pose pairs no point
 * connects -- + backward; banded systems of any size the pipeline's task bound takes, e.g.
 * n > 12288), path 1 = always pad + one
 * panel launch per step + the multi-workgroup backward, path 2 = always pad + pipelined
 * factorisation + backward (bitwise equal to path 1), path 3 = pad + one panel launch per step
 * + the one-workgroup backward substitution (dense systems above 96 tiles, n > 6144, run this
 * path; it takes n <= 12288).  Paths 0-2 give bitwise equal x
 * (tests/test_global_ba.py::test_gpu_one_tile_solve_matches_tiled).  A timed-out hand-off wait
 * of the pipelined kernels returns MCS_ERR_HIP (never a zero pivot). */
int mcs_dense_ldlt_solve_ex(int32_t device, const double* S, int32_t n, const double* b, double* x,
                            int32_t* zero_pivot, int32_t path);
/* Test hook: the pipelined LDL^T's hand-off wait bound in ticks of the 100 MHz real-time counter
 * (<= 0 restores the default 25,000,000 = 0.25 s).  Process-wide; tests lower it to force the
 * timeout path, which must surface as MCS_ERR_HIP from the solve and the BA entries. */
int mcs_ldlt_set_wait_ticks(int64_t ticks);

#ifdef __cplusplus
}
#endif
#endif /* MCS_BA_H */
