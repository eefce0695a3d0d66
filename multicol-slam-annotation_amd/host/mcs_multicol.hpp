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
//
// cv::KeyPoint-compatible: mcs_keypoint has cv::KeyPoint's field order and size (28 B), so a
// std::vector<mcs_keypoint> can be copied into std::vector<cv::KeyPoint> member-wise.
#pragma once
#include <cstdint>
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

}  // namespace mcs
