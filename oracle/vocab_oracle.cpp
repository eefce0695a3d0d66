// ORACLE (test infrastructure only -- imported by tests/, __graft_entry__.smoke() and the
// bench.py cpu_baseline leg as the CHECKER, never shipped or measured as the product).
//
// CPU restatement of the DBoW2 vocabulary transform used by MultiCol-SLAM's ComputeBoW
// (src/cMultiFrame.cpp:356-363, src/cMultiKeyFrame.cpp:105-119):
//   TemplatedVocabulary::load(FileStorage)            ThirdParty/DBoW2/DBoW2/TemplatedVocabulary.h:1568-1616
//   TemplatedVocabulary::transform(feature, ...)      TemplatedVocabulary.h:1217-1261
//   TemplatedVocabulary::transform(features, v, fv)   TemplatedVocabulary.h:1126-1196
//   BowVector::addWeight/addIfNotExist/normalize      BowVector.cpp:34-86
//   FeatureVector::addFeature                         FeatureVector.cpp:31-45
//   FORB::distance (SWAR popcount over 8 int32)       FORB.cpp:82-101
//   ScoringObject mustNormalize table                 ScoringObject.h:74-89
// The reference cannot be compiled here (DBoW2 needs OpenCV, absent), so this restatement is
// pinned by the reference's own vocabulary file (Examples/small_orb_omni_voc_9_6.yml: node
// count, word count, k, L, weights) and by exhaustive-descent cross-checks in tests/; the
// transform outputs themselves are "parity unpinned" against a reference binary.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <vector>

namespace {

struct Node {
  int id = 0, parent = 0;
  double weight = 0;
  unsigned word_id = 0;
  std::vector<int> children;
  uint8_t desc[32] = {0};
  bool isLeaf() const { return children.empty(); }
};

struct Voc {
  int k = 0, L = 0, scoring = 0, weighting = 0;
  std::vector<Node> nodes;
  std::vector<int> words;
  bool empty() const { return words.empty(); }
};

// FORB::distance: bit-parallel popcount of the XOR, 32 bits at a time (FORB.cpp:88-98)
int forb_distance(const uint8_t* a, const uint8_t* b) {
  int dist = 0;
  for (int i = 0; i < 8; i++) {
    uint32_t x, y;
    std::memcpy(&x, a + 4 * i, 4);
    std::memcpy(&y, b + 4 * i, 4);
    uint32_t v = x ^ y;
    v = v - ((v >> 1) & 0x55555555u);
    v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
    dist += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
  }
  return dist;
}

Voc make_voc(int k, int L, int scoring, int weighting, int n_nodes, const int* node_id,
             const int* parent_id, const double* weight, const uint8_t* desc, int n_words,
             const int* word_node) {
  Voc v;
  v.k = k; v.L = L; v.scoring = scoring; v.weighting = weighting;
  v.nodes.resize(n_nodes + 1);
  for (int i = 0; i < n_nodes; ++i) {   // load(): :1585-1600
    Node& nd = v.nodes[node_id[i]];
    nd.id = node_id[i];
    nd.parent = parent_id[i];
    nd.weight = weight[i];
    v.nodes[parent_id[i]].children.push_back(node_id[i]);
    std::memcpy(nd.desc, desc + 32 * (size_t)i, 32);
  }
  v.words.resize(n_words);
  for (int w = 0; w < n_words; ++w) {   // :1603-1613
    v.nodes[word_node[w]].word_id = (unsigned)w;
    v.words[w] = word_node[w];
  }
  return v;
}

// transform(feature, word_id, weight, nid, levelsup)  :1217-1261
void transform_one(const Voc& v, const uint8_t* f, unsigned* word_id, double* weight, int* nid,
                   int levelsup) {
  const int nid_level = v.L - levelsup;
  if (nid_level <= 0) *nid = 0;
  int final_id = 0, current_level = 0;
  do {
    ++current_level;
    const std::vector<int>& nodes = v.nodes[final_id].children;
    if (nodes.empty()) break;   // childless root (malformed); the reference would index nodes[0]
    final_id = nodes[0];
    int best_d = forb_distance(f, v.nodes[final_id].desc);
    for (size_t j = 1; j < nodes.size(); ++j) {
      int d = forb_distance(f, v.nodes[nodes[j]].desc);
      if (d < best_d) { best_d = d; final_id = nodes[j]; }
    }
    if (current_level == nid_level) *nid = final_id;
  } while (!v.nodes[final_id].isLeaf());
  *word_id = v.nodes[final_id].word_id;
  *weight = v.nodes[final_id].weight;
}

}  // namespace

extern "C" {

// Per-feature descent: word, weight and the level-(L - levelsup) ancestor of every descriptor.
int oracle_vocab_words(int k, int L, int scoring, int weighting, int n_nodes, const int* node_id,
                       const int* parent_id, const double* weight, const uint8_t* desc,
                       int n_words, const int* word_node, const uint8_t* feats, int n,
                       int levelsup, uint32_t* word, double* w, uint32_t* node) {
  Voc v = make_voc(k, L, scoring, weighting, n_nodes, node_id, parent_id, weight, desc, n_words,
                   word_node);
  for (int i = 0; i < n; ++i) {
    if (v.empty()) { word[i] = 0; w[i] = 0; node[i] = 0; continue; }
    unsigned wid = 0; double wt = 0; int nid = 0;
    transform_one(v, feats + 32 * (size_t)i, &wid, &wt, &nid, levelsup);
    word[i] = wid; w[i] = wt; node[i] = (uint32_t)nid;
  }
  return 0;
}

// transform(features, BowVector, FeatureVector, levelsup) with the reference containers
// (std::map keyed by word / node id), flattened like mcs_vocab_transform.
int oracle_vocab_transform(int k, int L, int scoring, int weighting, int n_nodes,
                           const int* node_id, const int* parent_id, const double* weight,
                           const uint8_t* desc, int n_words, const int* word_node,
                           const uint8_t* feats, int n, int levelsup, uint32_t* bow_word,
                           double* bow_value, int* bow_n, uint32_t* fv_node, int* fv_ptr,
                           uint32_t* fv_feat, int* fv_n) {
  Voc v = make_voc(k, L, scoring, weighting, n_nodes, node_id, parent_id, weight, desc, n_words,
                   word_node);
  std::map<unsigned, double> bv;
  std::map<unsigned, std::vector<unsigned>> fv;
  *bow_n = 0; *fv_n = 0; fv_ptr[0] = 0;
  if (v.empty()) return 0;
  // LNorm + mustNormalize (ScoringObject.h:74-89)
  const bool must = scoring != 5;
  const bool l2 = scoring == 1;
  const bool tf = weighting == 0 || weighting == 1;
  for (int i = 0; i < n; ++i) {
    unsigned id; double w; int nid = 0;
    transform_one(v, feats + 32 * (size_t)i, &id, &w, &nid, levelsup);
    if (w > 0) {
      if (tf) {
        auto it = bv.find(id);          // addWeight
        if (it != bv.end()) it->second += w; else bv[id] = w;
      } else {
        if (!bv.count(id)) bv[id] = w;  // addIfNotExist
      }
      fv[(unsigned)nid].push_back((unsigned)i);
    }
  }
  if (tf && !bv.empty() && !must) {
    const double nd = bv.size();
    for (auto& e : bv) e.second /= nd;
  }
  if (must) {
    double norm = 0.0;
    if (!l2) for (auto& e : bv) norm += std::fabs(e.second);
    else { for (auto& e : bv) norm += e.second * e.second; norm = std::sqrt(norm); }
    if (norm > 0.0) for (auto& e : bv) e.second /= norm;
  }
  int j = 0;
  for (auto& e : bv) { bow_word[j] = e.first; bow_value[j] = e.second; ++j; }
  *bow_n = j;
  j = 0;
  int f = 0;
  for (auto& e : fv) {
    fv_node[j] = e.first; fv_ptr[j] = f;
    for (unsigned x : e.second) fv_feat[f++] = x;
    ++j;
  }
  fv_ptr[j] = f;
  *fv_n = j;
  return 0;
}

}  // extern "C"
