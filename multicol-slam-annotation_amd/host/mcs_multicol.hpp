// Header-only C++ host mirror of the reference operator surface, implemented on top of the
// C-ABI of libmcs_amd.so (include/mcs_extractor.h, mcs_matcher.h, mcs_ba.h).  A MultiCol-SLAM
// build keeps its call sites and swaps the types:
//
//   reference                                        here
//   mdBRIEFextractorOct(nfeatures, scaleFactor, ...)  mcs::mdBRIEFextractorOct(same args, w, h)
//     include/mdBRIEFextractorOct.h:339-351
//   operator()(image, mask, kps, camModel, desc,      operator()(image, stride, mask, mstride,
//              descMasks)  :355-361                      kps, camModel, desc, descMasks)
//   DescriptorDistance64 (include/cORBmatcher.h:43)   mcs::DescriptorDistance64
//   cOptimizer::LocalBundleAdjustment (cOptimizer.h:61) mcs::LocalBA::run(problem, ...)
//   cOptimizer::BundleAdjustment / GlobalBundleAdjustment (cOptimizer.h:50-59)
//                                                     mcs::GlobalBA::run(map, poseOnly, pbStopFlag)
//   cOptimizer::PoseOptimization (cOptimizer.h:67-69) mcs::PoseOptimizer::run(frame, inliers,
//                                                                        huberMultiplier)
//
// cv::KeyPoint-compatible: mcs_keypoint has cv::KeyPoint's field order and size (28 B), so a
// std::vector<mcs_keypoint> can be copied into std::vector<cv::KeyPoint> member-wise.
#pragma once
#include <cstdint>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/mcs_ba.h"
#include "../../include/mcs_extractor.h"
#include "../../include/mcs_matcher.h"

namespace mcs {

inline void check(int rc, const char* what) {
  if (rc != MCS_OK)
    throw std::runtime_error(std::string(what) + ": " + mcs_last_error() + " (" + std::to_string(rc) + ")");
}

class mdBRIEFextractorOct {
 public:
  mdBRIEFextractorOct(int nfeatures, float scaleFactor, int nlevels, int edgeThreshold,
                      int firstLevel, int scoreType, int patchSize, int fastThreshold,
                      bool useAgast, int fastAgastType, bool do_dBrief, bool learnMasks,
                      int descSize, int width, int height, int device = 0) {
    mcs_extractor_params p;
    p.nfeatures = nfeatures; p.scale_factor = scaleFactor; p.nlevels = nlevels;
    p.edge_threshold = edgeThreshold; p.first_level = firstLevel; p.score_type = scoreType;
    p.patch_size = patchSize; p.fast_threshold = fastThreshold; p.use_agast = useAgast;
    p.fast_agast_type = fastAgastType; p.do_dbrief = do_dBrief; p.learn_masks = learnMasks;
    p.desc_size = descSize;
    check(mcs_extractor_create(&p, width, height, 1, device, &h_), "mcs_extractor_create");
    desc_size_ = descSize;
    do_dbrief_ = do_dBrief;
    learn_masks_ = learnMasks;
    nlevels_ = nlevels;
    scale_factor_ = scaleFactor;
  }
  ~mdBRIEFextractorOct() { mcs_extractor_destroy(h_); }
  mdBRIEFextractorOct(const mdBRIEFextractorOct&) = delete;
  mdBRIEFextractorOct& operator=(const mdBRIEFextractorOct&) = delete;

  // operator()(image, mask, kps, camModel, desc, descMasks) (:355-361).  The camera model is
  // read only by the dBRIEF / mdBRIEF branches (keypoint undistortion :1304-1316 and the
  // re-distorted pattern :250-283); it is forwarded to the device when it changes.
  void operator()(const uint8_t* image, int stride, const uint8_t* mask, int mask_stride,
                  std::vector<mcs_keypoint>& kps, const mcs_cam_model& camModel,
                  std::vector<uint8_t>& desc, std::vector<uint8_t>& descMasks) {
    if ((do_dbrief_ || learn_masks_) &&
        (!cam_set_ || std::memcmp(&cam_, &camModel, sizeof(cam_)) != 0)) {
      check(mcs_extractor_set_cam_models(h_, &camModel, 1), "mcs_extractor_set_cam_models");
      cam_ = camModel;
      cam_set_ = true;
    }
    const int cap = mcs_extractor_capacity(h_);
    kps.resize(cap);
    desc.resize((size_t)cap * desc_size_);
    descMasks.resize((size_t)cap * desc_size_);
    int32_t n = 0;
    check(mcs_extract(h_, image, stride, mask, mask_stride, kps.data(), cap, &n, desc.data(),
                      descMasks.data()),
          "mcs_extract");
    kps.resize(n);
    desc.resize((size_t)n * desc_size_);
    descMasks.resize((size_t)n * desc_size_);
  }

  int GetLevels() const { return nlevels_; }
  double GetScaleFactor() const { return (double)scale_factor_; }
  bool GetMasksLearned() const { return learn_masks_; }   // mdBRIEFextractorOct.h:367
  int GetDescriptorSize() const { return desc_size_; }
  mcs_extractor* handle() { return h_; }

 private:
  mcs_extractor* h_ = nullptr;
  int desc_size_ = 32, nlevels_ = 8;
  float scale_factor_ = 1.2f;
  bool do_dbrief_ = false, learn_masks_ = false, cam_set_ = false;
  mcs_cam_model cam_{};
};

inline int DescriptorDistance64(const uint64_t* d1, const uint64_t* d2, const int& dim) {
  return mcs_descriptor_distance64(d1, d2, dim);
}
inline int DescriptorDistance64Masked(const uint64_t* d1, const uint64_t* d2, const uint64_t* m1,
                                      const uint64_t* m2, const int& dim) {
  return mcs_descriptor_distance64_masked(d1, d2, m1, m2, dim);
}

// LocalBundleAdjustment after the host has collected local/fixed keyframes and observations
// (src/cOptimizer.cpp:503-769) into an mcs_ba_problem.
class LocalBA {
 public:
  explicit LocalBA(int device = 0) { check(mcs_ba_create(device, &c_), "mcs_ba_create"); }
  ~LocalBA() { mcs_ba_destroy(c_); }
  LocalBA(const LocalBA&) = delete;
  LocalBA& operator=(const LocalBA&) = delete;

  struct Result {
    std::vector<double> poses, points;
    std::vector<uint8_t> edge_inlier;
    bool write_back = false;
    mcs_ba_report round1{}, round2{};
  };

  Result run(const mcs_ba_problem& p, volatile int32_t* pbStopFlag) {
    Result r;
    r.poses.assign(p.poses, p.poses + 6 * (size_t)p.n_poses);
    r.points.assign(p.points, p.points + 3 * (size_t)p.n_points);
    r.edge_inlier.assign(p.n_edges, 1);
    int32_t wb = 0;
    check(mcs_local_ba(c_, &p, r.poses.data(), r.points.data(), r.edge_inlier.data(), &wb,
                       pbStopFlag, &r.round1, &r.round2),
          "mcs_local_ba");
    r.write_back = wb != 0;
    return r;
  }

 private:
  mcs_ba_ctx* c_ = nullptr;
};


// cOptimizer::BundleAdjustment (src/cOptimizer.cpp:73-261): the keyframe / map-point lists of
// GlobalBundleAdjustment (pMap->GetAllKeyFrames(), GetAllMapPoints(), :64-68) as flat arrays,
// graph assembly by mcs_global_ba_select (vertex ids, maxKF rule, bad skips), one optimize(15)
// by mcs_global_ba, and the write-back of :240-259 through the select's slots.
class GlobalBA {
 public:
  explicit GlobalBA(int device = 0) { check(mcs_ba_create(device, &c_), "mcs_ba_create"); }
  ~GlobalBA() { mcs_ba_destroy(c_); }
  GlobalBA(const GlobalBA&) = delete;
  GlobalBA& operator=(const GlobalBA&) = delete;

  struct Map {
    std::vector<int64_t> kf_id;       // vpKFs: mnId
    std::vector<uint8_t> kf_bad;      //        isBad()
    std::vector<double> kf_pose;      //        [n_kf][6] hom2cayley(GetPose())
    std::vector<int64_t> pt_id;       // vpMP:  mnId
    std::vector<uint8_t> pt_bad;      //        isBad()
    std::vector<double> pt_pos;       //        [n_points][3] GetWorldPos()
    std::vector<int32_t> pt_obs_off;  // [n_points + 1]: GetObservations() in std::map order
    std::vector<int32_t> obs_kf;      // vpKFs index of the observing keyframe
    std::vector<int32_t> obs_cam;     // keypoint_to_cam[obsIdx]
    std::vector<double> obs_meas;     // [n_obs][2] GetKeyPoint(obsIdx).pt
    std::vector<double> mc;           // [n_cams][6] vpKFs[0]->camSystem.Get_M_c_min(c)
    std::vector<double> cam;          // [n_cams][17] GetCamModelObj(c).toVector()
  };
  struct Result {
    std::vector<double> kf_pose, pt_pos;      // the lists' poses / positions after the write-back
    std::vector<uint8_t> kf_written, pt_written;
    mcs_ba_report report{};
  };

  // Throws on an id collision (g2o's addVertex FATAL) or any other error.
  Result run(const Map& m, bool poseOnly, volatile int32_t* pbStopFlag = nullptr) {
    const int nk = (int)m.kf_id.size(), np = (int)m.pt_id.size(), nc = (int)m.mc.size() / 6;
    mcs_gba_map gm{nk, m.kf_id.data(), m.kf_bad.data(), np, m.pt_id.data(), m.pt_bad.data(),
                   m.pt_obs_off.data(), m.obs_kf.data(), nc};
    const int nobs = (int)m.obs_kf.size();
    std::vector<int32_t> pose_kf(nk), points(np), kf_slot(nk), pt_slot(np), eo(nobs), ep(nobs), eq(nobs);
    std::vector<uint8_t> pose_fixed(nk);
    mcs_gba_graph g{pose_kf.data(), pose_fixed.data(), 0, points.data(), nullptr, 0, -1, -1,
                    kf_slot.data(), pt_slot.data(), eo.data(), ep.data(), eq.data(), 0, nobs, -1};
    check(mcs_global_ba_select(&gm, &g), "mcs_global_ba_select");
    std::vector<double> poses(6 * (size_t)g.n_poses), pts(3 * (size_t)g.n_points), meas(2 * (size_t)g.n_edges);
    std::vector<int32_t> ecam(g.n_edges);
    std::vector<double> info(g.n_edges, 1.0);                       // Identity (:209)
    for (int i = 0; i < g.n_poses; i++) std::memcpy(&poses[6 * i], &m.kf_pose[6 * (size_t)pose_kf[i]], 48);
    for (int i = 0; i < g.n_points; i++) std::memcpy(&pts[3 * i], &m.pt_pos[3 * (size_t)points[i]], 24);
    for (int e = 0; e < g.n_edges; e++) {
      ecam[e] = m.obs_cam[eo[e]];
      meas[2 * e] = m.obs_meas[2 * (size_t)eo[e]];
      meas[2 * e + 1] = m.obs_meas[2 * (size_t)eo[e] + 1];
    }
    mcs_ba_problem p{g.n_poses, g.n_points, g.n_edges, nc, poses.data(), pose_fixed.data(), pts.data(),
                     m.mc.data(), m.cam.data(), ep.data(), eq.data(), ecam.data(), meas.data(), info.data(),
                     std::sqrt(5.991)};                             // thHuber (:161)
    Result r;
    check(mcs_global_ba(c_, &p, poseOnly ? 1 : 0, poses.data(), pts.data(), pbStopFlag, &r.report, nullptr),
          "mcs_global_ba");
    r.kf_pose = m.kf_pose;
    r.pt_pos = m.pt_pos;
    r.kf_written.assign(nk, 0);
    r.pt_written.assign(np, 0);
    for (int i = 0; i < nk; i++)
      if (kf_slot[i] >= 0) { std::memcpy(&r.kf_pose[6 * (size_t)i], &poses[6 * (size_t)kf_slot[i]], 48); r.kf_written[i] = 1; }
    for (int i = 0; i < np; i++)
      if (pt_slot[i] >= 0) { std::memcpy(&r.pt_pos[3 * (size_t)i], &pts[3 * (size_t)pt_slot[i]], 24); r.pt_written[i] = 1; }
    return r;
  }

 private:
  mcs_ba_ctx* c_ = nullptr;
};

// cOptimizer::PoseOptimization(pFrame, inliers, huberMultiplier) (src/cOptimizer.cpp:264-486):
// the frame's map-point matches as indices, graph assembly by mcs_pose_optimization_select,
// both rounds and the outlier classification by mcs_pose_optimization.
class PoseOptimizer {
 public:
  explicit PoseOptimizer(int device = 0) { check(mcs_ba_create(device, &c_), "mcs_ba_create"); }
  ~PoseOptimizer() { mcs_ba_destroy(c_); }
  PoseOptimizer(const PoseOptimizer&) = delete;
  PoseOptimizer& operator=(const PoseOptimizer&) = delete;

  struct Frame {
    std::vector<int32_t> key_mp;      // mvpMapPoints[i]: index into pt_id / pt_pos, -1 = NULL
    std::vector<int32_t> key_cam;     // keypoint_to_cam[i]
    std::vector<double> key_pt;       // [N][2] mvKeys[i].pt
    std::vector<int32_t> key_octave;  // mvKeys[i].octave
    std::vector<double> inv_level_sigma2;   // mvInvLevelSigma2
    std::vector<int64_t> pt_id;       // map points: mnId
    std::vector<double> pt_pos;       //             [n][3] GetWorldPos()
    std::vector<double> pose;         // [6] GetPoseMin()
    std::vector<double> mc, cam;      // camSystem: [n_cams][6], [n_cams][17]
  };
  struct Result {
    int n_good = 0;                   // the reference's return value
    double inliers = 0.0;             // its `inliers` output (nBad / nInitialCorrespondences)
    std::vector<uint8_t> outlier;     // mvbOutlier
    std::vector<double> pose;         // Set_M_t_from_min
    mcs_ba_report round1{}, round2{};
  };

  Result run(const Frame& f, double huberMultiplier = 2) {
    const int N = (int)f.key_mp.size(), nmp = (int)f.pt_id.size(), nc = (int)f.mc.size() / 6;
    mcs_po_frame pf{N, f.key_mp.data(), nmp, f.pt_id.data(), nc};
    std::vector<int32_t> points(nmp), eo(N), eq(N);
    mcs_po_graph g{points.data(), nullptr, 0, eo.data(), eq.data(), 0, N};
    check(mcs_pose_optimization_select(&pf, &g), "mcs_pose_optimization_select");
    std::vector<double> pts(3 * (size_t)g.n_points), meas(2 * (size_t)g.n_edges), info(g.n_edges);
    std::vector<int32_t> ecam(g.n_edges), epose(g.n_edges, 0);
    for (int i = 0; i < g.n_points; i++) std::memcpy(&pts[3 * i], &f.pt_pos[3 * (size_t)points[i]], 24);
    for (int e = 0; e < g.n_edges; e++) {
      const int k = eo[e];
      ecam[e] = f.key_cam[k];
      meas[2 * e] = f.key_pt[2 * (size_t)k];
      meas[2 * e + 1] = f.key_pt[2 * (size_t)k + 1];
      info[e] = f.inv_level_sigma2[f.key_octave[k]];               // :405-406
    }
    const uint8_t not_fixed = 0;
    mcs_ba_problem p{1, g.n_points, g.n_edges, nc, f.pose.data(), &not_fixed, pts.data(), f.mc.data(),
                     f.cam.data(), epose.data(), eq.data(), ecam.data(), meas.data(), info.data(),
                     1.345 * huberMultiplier};                     // :344
    Result r;
    r.pose = f.pose;
    std::vector<uint8_t> eout(std::max(1, g.n_edges));
    int32_t good = 0;
    check(mcs_pose_optimization(c_, &p, r.pose.data(), eout.data(), &good, &r.inliers, &r.round1, &r.round2),
          "mcs_pose_optimization");
    r.n_good = good;
    r.outlier.assign(N, 0);                                        // :367
    for (int e = 0; e < g.n_edges; e++) r.outlier[eo[e]] = eout[e];
    return r;
  }

 private:
  mcs_ba_ctx* c_ = nullptr;
};

}  // namespace mcs
