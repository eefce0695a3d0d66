// DBoW2 vocabulary transform (bag of words) for ORB descriptors on gfx950.
//
// Reference (billamiable/MultiCol-SLAM-Annotation, ThirdParty/DBoW2/DBoW2):
//   load(const cv::FileStorage&)                       TemplatedVocabulary.h:1568-1616
//   transform(feature, word_id, weight, nid, levelsup) TemplatedVocabulary.h:1217-1261
//   transform(features, BowVector, FeatureVector, up)  TemplatedVocabulary.h:1126-1196
//   BowVector::addWeight / addIfNotExist / normalize   BowVector.cpp:34-86
//   FeatureVector::addFeature                          FeatureVector.cpp:31-45
//   FORB::distance (32-byte popcount)                  FORB.cpp:82-101
//   mustNormalize per scoring type                     ScoringObject.h:53-91
//
// Device layout (HBM, built once per vocabulary): the children of every node are stored
// contiguously in CSR order (node -> [child_begin, child_begin + child_count)), and the
// children's 32-byte descriptors are stored in that same CSR order, so one descent step of a
// lane reads one contiguous k x 32 B block.  Per node: child_begin (i32), child_count (i32),
// word_id (u32), weight (f64).  The whole small Lafida vocabulary (15 821 nodes) is 0.5 MB of
// descriptors and stays resident in each XCD's L2 while a batch is transformed.
//
// Kernel: one lane per descriptor, the descriptor held in 8 VGPRs; per level the lane scans
// the k children (first strict minimum wins, as `d < best_d` in the reference) and moves to
// the winner; the ancestor at level L - levelsup is recorded on the way down.  The descent is
// integer VALU work (v_xor + v_bcnt per dword) on L2-resident gathers; roofline: the
// descriptor stream (32 B in, 16 B out per feature) from HBM.
#include "common.hpp"
#include "../../include/mcs_vocab.h"
#include <algorithm>
#include <cmath>
#include <map>
#include <vector>

struct mcs_vocab {
  int k = 0, L = 0, scoring = 0, weighting = 0, n_nodes = 0, n_words = 0, device = 0;
  int32_t* d_child_begin = nullptr;
  int32_t* d_child_count = nullptr;
  uint32_t* d_child_id = nullptr;
  uint4* d_child_desc = nullptr;   // 2 x uint4 per child
  uint32_t* d_word = nullptr;
  double* d_weight = nullptr;
};

namespace mcs {
namespace voc {

constexpr int kBlock = 256;
constexpr int kMaxDepth = 64;      // host validation guarantees depth <= this

__device__ __forceinline__ int ham32(const uint32_t (&a)[8], uint4 lo, uint4 hi) {
  return __popc(a[0] ^ lo.x) + __popc(a[1] ^ lo.y) + __popc(a[2] ^ lo.z) + __popc(a[3] ^ lo.w) +
         __popc(a[4] ^ hi.x) + __popc(a[5] ^ hi.y) + __popc(a[6] ^ hi.z) + __popc(a[7] ^ hi.w);
}

__global__ __launch_bounds__(kBlock) void k_descend(
    const uint4* __restrict__ desc, int n, const int32_t* __restrict__ child_begin,
    const int32_t* __restrict__ child_count, const uint32_t* __restrict__ child_id,
    const uint4* __restrict__ child_desc, const uint32_t* __restrict__ node_word,
    const double* __restrict__ node_weight, int nid_level, uint32_t* __restrict__ out_word,
    double* __restrict__ out_weight, uint32_t* __restrict__ out_node) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint4 lo = desc[2 * i], hi = desc[2 * i + 1];
  const uint32_t f[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  uint32_t nid = 0;          // nid_level <= 0 -> root (TemplatedVocabulary.h:1229)
  uint32_t cur = 0;
  for (int level = 1; level <= kMaxDepth; ++level) {
    const int b = child_begin[cur], c = child_count[cur];
    if (c == 0) break;       // only reachable for a childless root
    int best = b;
    int best_d = ham32(f, child_desc[2 * b], child_desc[2 * b + 1]);
    for (int j = b + 1; j < b + c; ++j) {
      const int d = ham32(f, child_desc[2 * j], child_desc[2 * j + 1]);
      if (d < best_d) { best_d = d; best = j; }
    }
    cur = child_id[best];
    if (level == nid_level) nid = cur;
    if (child_count[cur] == 0) break;  // isLeaf()
  }
  out_word[i] = node_word[cur];
  out_weight[i] = node_weight[cur];
  out_node[i] = nid;
}

// L2 scoring normalises with L2, DOT_PRODUCT not at all, every other scoring with L1
// (ScoringObject.h:74-89).
inline bool must_normalize(int scoring, bool* l2) {
  *l2 = scoring == 1;
  return scoring != 5;
}

}  // namespace voc
}  // namespace mcs

using namespace mcs;

extern "C" {

int mcs_vocab_create(int32_t k, int32_t L, int32_t scoring, int32_t weighting, int32_t n_nodes,
                     const int32_t* node_id, const int32_t* parent_id, const double* weight,
                     const uint8_t* desc, int32_t n_words, const int32_t* word_node,
                     int32_t device, mcs_vocab** out) {
  if (!out) return MCS_ERR_ARG;
  *out = nullptr;
  if (n_nodes < 0 || n_words < 0 || scoring < 0 || scoring > 5 || weighting < 0 || weighting > 3)
    return MCS_ERR_ARG;
  if (n_nodes > 0 && (!node_id || !parent_id || !weight || !desc)) return MCS_ERR_ARG;
  if (n_words > 0 && !word_node) return MCS_ERR_ARG;
  const int nn = n_nodes + 1;   // + root (load(): m_nodes.resize(fn.size() + 1))
  std::vector<int32_t> parent(nn, -1), pos(nn, -1);
  std::vector<std::vector<int32_t>> children(nn);
  for (int i = 0; i < n_nodes; ++i) {
    const int id = node_id[i], p = parent_id[i];
    if (id < 1 || id >= nn || p < 0 || p >= nn || id == p || pos[id] >= 0) {
      set_error("vocabulary node ids must be a permutation of 1..n_nodes with valid parents");
      return MCS_ERR_ARG;
    }
    pos[id] = i;
    parent[id] = p;
    children[p].push_back(id);   // file order (push_back in load())
  }
  // acyclic and not deeper than the kernel's bound
  std::vector<int32_t> depth(nn, -1);
  depth[0] = 0;
  for (int v = 1; v < nn; ++v) {
    std::vector<int32_t> chain;
    int u = v;
    while (depth[u] < 0) {
      chain.push_back(u);
      if ((int)chain.size() > voc::kMaxDepth + 1) {
        set_error("vocabulary tree has a cycle or is deeper than 64 levels");
        return MCS_ERR_ARG;
      }
      u = parent[u];
    }
    for (int j = (int)chain.size() - 1; j >= 0; --j) depth[chain[j]] = depth[parent[chain[j]]] + 1;
    if (depth[v] > voc::kMaxDepth) {
      set_error("vocabulary tree deeper than 64 levels");
      return MCS_ERR_ARG;
    }
  }
  std::vector<uint32_t> word(nn, 0);     // Node(): word_id(0)
  for (int w = 0; w < n_words; ++w) {
    if (word_node[w] < 0 || word_node[w] >= nn) return MCS_ERR_ARG;
    word[word_node[w]] = (uint32_t)w;
  }
  std::vector<int32_t> cb(nn), cc(nn);
  std::vector<uint32_t> cid;
  std::vector<uint8_t> cdesc;
  std::vector<double> wt(nn, 0.0);
  cid.reserve(n_nodes);
  cdesc.reserve((size_t)n_nodes * 32);
  for (int v = 0; v < nn; ++v) {
    cb[v] = (int32_t)cid.size();
    cc[v] = (int32_t)children[v].size();
    for (int c : children[v]) {
      cid.push_back((uint32_t)c);
      cdesc.insert(cdesc.end(), desc + (size_t)pos[c] * 32, desc + (size_t)pos[c] * 32 + 32);
    }
    if (v > 0) wt[v] = weight[pos[v]];
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    set_error("no HIP device visible (no CPU fallback)");
    return MCS_ERR_NO_DEVICE;
  }
  if (device < 0 || device >= ndev) return MCS_ERR_ARG;
  MCS_HIP_CHECK(hipSetDevice(device));
  mcs_vocab* V = new mcs_vocab();
  V->k = k; V->L = L; V->scoring = scoring; V->weighting = weighting;
  V->n_nodes = nn; V->n_words = n_words; V->device = device;
  hipError_t e = hipSuccess;
  auto up = [&](auto** d, const auto* h, size_t bytes) {
    if (e == hipSuccess) e = hipMalloc((void**)d, std::max<size_t>(bytes, 16));
    if (e == hipSuccess && bytes) e = hipMemcpy(*d, h, bytes, hipMemcpyHostToDevice);
  };
  up(&V->d_child_begin, cb.data(), 4 * (size_t)nn);
  up(&V->d_child_count, cc.data(), 4 * (size_t)nn);
  up(&V->d_child_id, cid.data(), 4 * cid.size());
  up(&V->d_child_desc, reinterpret_cast<const uint4*>(cdesc.data()), cdesc.size());
  up(&V->d_word, word.data(), 4 * (size_t)nn);
  up(&V->d_weight, wt.data(), 8 * (size_t)nn);
  if (e != hipSuccess) {
    set_hip_error(e, "vocabulary upload", __FILE__, __LINE__);
    mcs_vocab_destroy(V);
    return MCS_ERR_HIP;
  }
  *out = V;
  return MCS_OK;
}

int mcs_vocab_destroy(mcs_vocab* V) {
  if (!V) return MCS_OK;
  void* ps[] = {V->d_child_begin, V->d_child_count, V->d_child_id, V->d_child_desc, V->d_word,
                V->d_weight};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  delete V;
  return MCS_OK;
}

int mcs_vocab_info(const mcs_vocab* V, int32_t* info) {
  if (!V || !info) return MCS_ERR_ARG;
  info[0] = V->k; info[1] = V->L; info[2] = V->scoring; info[3] = V->weighting;
  info[4] = V->n_nodes; info[5] = V->n_words;
  return MCS_OK;
}

int mcs_vocab_transform_words_device(const mcs_vocab* V, const uint8_t* d_desc, int32_t n,
                                     int32_t levelsup, uint32_t* d_word, double* d_weight,
                                     uint32_t* d_node, void* stream) {
  if (!V || n < 0 || (n > 0 && (!d_desc || !d_word || !d_weight || !d_node))) return MCS_ERR_ARG;
  if (((uintptr_t)d_desc & 15) || ((uintptr_t)d_weight & 7) || ((uintptr_t)d_word & 3) ||
      ((uintptr_t)d_node & 3)) {
    set_error("vocab transform: descriptor buffer must be 16-byte aligned");
    return MCS_ERR_ARG;
  }
  if (n == 0) return MCS_OK;
  hipStream_t s = (hipStream_t)stream;
  if (V->n_words == 0) {   // empty(): transform() returns word 0 / weight 0 (:1053-1056)
    MCS_HIP_CHECK(hipMemsetAsync(d_word, 0, 4 * (size_t)n, s));
    MCS_HIP_CHECK(hipMemsetAsync(d_weight, 0, 8 * (size_t)n, s));
    MCS_HIP_CHECK(hipMemsetAsync(d_node, 0, 4 * (size_t)n, s));
    return MCS_OK;
  }
  const int grid = (n + voc::kBlock - 1) / voc::kBlock;
  hipLaunchKernelGGL(voc::k_descend, dim3(grid), dim3(voc::kBlock), 0, s,
                     reinterpret_cast<const uint4*>(d_desc), n, V->d_child_begin, V->d_child_count,
                     V->d_child_id, V->d_child_desc, V->d_word, V->d_weight, V->L - levelsup,
                     d_word, d_weight, d_node);
  MCS_HIP_CHECK(hipGetLastError());
  return MCS_OK;
}

int mcs_vocab_transform(const mcs_vocab* V, const uint8_t* desc, int32_t n, int32_t levelsup,
                        uint32_t* bow_word, double* bow_value, int32_t* bow_n, uint32_t* fv_node,
                        int32_t* fv_ptr, uint32_t* fv_feat, int32_t* fv_n) {
  if (!V || n < 0 || !bow_n || !fv_n || (n > 0 && !desc)) return MCS_ERR_ARG;
  if (n > 0 && (!bow_word || !bow_value || !fv_node || !fv_ptr || !fv_feat)) return MCS_ERR_ARG;
  *bow_n = 0;
  *fv_n = 0;
  if (fv_ptr) fv_ptr[0] = 0;
  if (V->n_words == 0 || n == 0) return MCS_OK;   // v.clear(); fv.clear(); empty() -> return
  MCS_HIP_CHECK(hipSetDevice(V->device));
  uint8_t* d = nullptr;
  const size_t nn = (size_t)n;
  MCS_HIP_CHECK(hipMalloc(&d, nn * 48 + 64));
  uint8_t* d_desc = d;
  double* d_weight = reinterpret_cast<double*>(d + nn * 32);
  uint32_t* d_word = reinterpret_cast<uint32_t*>(d + nn * 40);
  uint32_t* d_node = reinterpret_cast<uint32_t*>(d + nn * 44);
  std::vector<uint32_t> word(nn), node(nn);
  std::vector<double> w(nn);
  hipError_t e = hipMemcpy(d_desc, desc, nn * 32, hipMemcpyHostToDevice);
  int rc = MCS_OK;
  if (e == hipSuccess)
    rc = mcs_vocab_transform_words_device(V, d_desc, n, levelsup, d_word, d_weight, d_node, nullptr);
  if (e == hipSuccess && rc == MCS_OK) e = hipMemcpy(word.data(), d_word, nn * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess && rc == MCS_OK) e = hipMemcpy(node.data(), d_node, nn * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess && rc == MCS_OK) e = hipMemcpy(w.data(), d_weight, nn * 8, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) { set_hip_error(e, "vocab transform", __FILE__, __LINE__); return MCS_ERR_HIP; }
  if (rc) return rc;
  // BowVector / FeatureVector assembly in feature order (:1142-1193)
  std::map<uint32_t, double> bow;
  std::map<uint32_t, std::vector<uint32_t>> fv;
  const bool tf = V->weighting == 0 || V->weighting == 1;
  for (size_t i = 0; i < nn; ++i) {
    if (!(w[i] > 0)) continue;   // stopped word
    auto it = bow.lower_bound(word[i]);
    if (it != bow.end() && it->first == word[i]) {
      if (tf) it->second += w[i];                     // addWeight
    } else {
      bow.emplace_hint(it, word[i], w[i]);            // insert / addIfNotExist
    }
    fv[node[i]].push_back((uint32_t)i);
  }
  bool l2 = false;
  const bool must = voc::must_normalize(V->scoring, &l2);
  if (tf && !bow.empty() && !must) {
    const double nd = (double)bow.size();
    for (auto& kv : bow) kv.second /= nd;
  }
  if (must) {   // BowVector::normalize
    double norm = 0.0;
    if (!l2) {
      for (auto& kv : bow) norm += std::fabs(kv.second);
    } else {
      for (auto& kv : bow) norm += kv.second * kv.second;
      norm = std::sqrt(norm);
    }
    if (norm > 0.0)
      for (auto& kv : bow) kv.second /= norm;
  }
  int j = 0;
  for (auto& kv : bow) { bow_word[j] = kv.first; bow_value[j] = kv.second; ++j; }
  *bow_n = j;
  j = 0;
  int f = 0;
  for (auto& kv : fv) {
    fv_node[j] = kv.first;
    fv_ptr[j] = f;
    for (uint32_t x : kv.second) fv_feat[f++] = x;
    ++j;
  }
  fv_ptr[j] = f;
  *fv_n = j;
  return MCS_OK;
}

}  // extern "C"
