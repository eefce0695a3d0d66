/*
 * mcs_vocab.h -- C-ABI drop-in boundary for the DBoW2 vocabulary transform (bag of words).
 *
 * Replaces (billamiable/MultiCol-SLAM-Annotation, ThirdParty/DBoW2, ORBVocabulary =
 * TemplatedVocabulary<FORB::TDescriptor, FORB>, include/cORBVocabulary.h):
 *   TemplatedVocabulary::load(const cv::FileStorage&, name)   TemplatedVocabulary.h:1568-1616
 *     -> mcs_vocab_create (the caller parses the YAML node list; mcs_amd/vocab.py does it)
 *   TemplatedVocabulary::transform(feature, word_id, weight, nid, levelsup)
 *                                                              TemplatedVocabulary.h:1217-1261
 *     -> mcs_vocab_transform_words_device (one call for every descriptor of a batch)
 *   TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup)
 *                                                              TemplatedVocabulary.h:1126-1196
 *     -> mcs_vocab_transform (host descriptors in, sparse BowVector / FeatureVector out)
 *   FORB::distance                                             FORB.cpp:82-101
 * Callers: cMultiFrame::ComputeBoW (src/cMultiFrame.cpp:356-363) and
 * cMultiKeyFrame::ComputeBoW (src/cMultiKeyFrame.cpp:105-119), both with levelsup = 4 over the
 * camera-concatenated descriptors (cConverter::toDescriptorVector, src/cConverter.cpp:58-67).
 *
 * Descriptors are FORB's 32 bytes.  Enumerations follow DBoW2 (BowVector.h):
 * weighting TF_IDF = 0, TF = 1, IDF = 2, BINARY = 3; scoring L1_NORM = 0, L2_NORM = 1,
 * CHI_SQUARE = 2, KL = 3, BHATTACHARYYA = 4, DOT_PRODUCT = 5.
 */
#ifndef MCS_VOCAB_H
#define MCS_VOCAB_H

#include <stdint.h>
#include "mcs_common.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mcs_vocab mcs_vocab;

/* Build a vocabulary on `device` from the YAML node list in file order (the order fixes each
 * parent's children order, exactly as load() push_backs them): node_id / parent_id / weight /
 * desc (n_nodes x 32 bytes) per entry, root (id 0) not listed; word_node[w] = node id of word w.
 * Node ids must be 1..n_nodes (load() sizes m_nodes to n_nodes + 1). */
int mcs_vocab_create(int32_t k, int32_t L, int32_t scoring, int32_t weighting, int32_t n_nodes,
                     const int32_t* node_id, const int32_t* parent_id, const double* weight,
                     const uint8_t* desc, int32_t n_words, const int32_t* word_node,
                     int32_t device, mcs_vocab** out);
int mcs_vocab_destroy(mcs_vocab* voc);
/* k, L, scoring, weighting, number of nodes (incl. root), number of words */
int mcs_vocab_info(const mcs_vocab* voc, int32_t* info6);

/* Per-descriptor tree descent (device buffers, async on `stream`): d_word[i] = word id,
 * d_weight[i] = that word's weight, d_node[i] = the ancestor at level L - levelsup (0 = root
 * when L - levelsup <= 0).  An empty vocabulary writes word 0 / weight 0 / node 0. */
int mcs_vocab_transform_words_device(const mcs_vocab* voc, const uint8_t* d_desc, int32_t n,
                                     int32_t levelsup, uint32_t* d_word, double* d_weight,
                                     uint32_t* d_node, void* stream);

/* transform(features, BowVector, FeatureVector, levelsup) on host buffers.
 * BowVector: bow_n entries (bow_word ascending, bow_value), capacity n.
 * FeatureVector: fv_n node entries (fv_node ascending), features of entry j are
 * fv_feat[fv_ptr[j] .. fv_ptr[j+1]) in feature order; fv_ptr has capacity n + 1, fv_node and
 * fv_feat capacity n.  Stopped words (weight <= 0) appear in neither, as in the reference. */
int mcs_vocab_transform(const mcs_vocab* voc, const uint8_t* desc, int32_t n, int32_t levelsup,
                        uint32_t* bow_word, double* bow_value, int32_t* bow_n, uint32_t* fv_node,
                        int32_t* fv_ptr, uint32_t* fv_feat, int32_t* fv_n);

#ifdef __cplusplus
}
#endif
#endif /* MCS_VOCAB_H */
