"""DBoW2 ORB vocabulary on the GPU (include/mcs_vocab.h).

Host mirror of ORBVocabulary = DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB>
(reference include/cORBVocabulary.h, ThirdParty/DBoW2/DBoW2/TemplatedVocabulary.h):

  load_yaml(path)              ~ TemplatedVocabulary::load(cv::FileStorage)   :1568-1616
                                  (the FileStorage YAML written by save() :1475-1564; parsed
                                  here without OpenCV)
  Vocabulary.transform_words   ~ transform(feature, word_id, weight, nid, levelsup) :1217-1261,
                                  for a whole device batch in one launch
  Vocabulary.transform         ~ transform(features, BowVector, FeatureVector, levelsup)
                                  :1126-1196; called by cMultiFrame::ComputeBoW
                                  (src/cMultiFrame.cpp:356-363) with levelsup = 4

There is no CPU fallback: without the library or a GPU the calls raise.
"""
import ctypes
import re

import numpy as np

from . import McsError, _check, lib

TF_IDF, TF, IDF, BINARY = 0, 1, 2, 3                                   # BowVector.h:36-42
L1_NORM, L2_NORM, CHI_SQUARE, KL, BHATTACHARYYA, DOT_PRODUCT = range(6)  # BowVector.h:45-53



def _lib():
    return lib()   # signatures registered in mcs_amd.SIGNATURES


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


_NODE_RE = re.compile(r'\{\s*nodeId:\s*(\d+),\s*parentId:\s*(\d+),\s*weight:\s*([^,\s]+),\s*'
                      r'descriptor:\s*"([^"]*)"\s*\}')
_WORD_RE = re.compile(r'\{\s*wordId:\s*(\d+),\s*nodeId:\s*(\d+)\s*\}')


def _scalar(text, key):
    m = re.search(r'^\s*%s:\s*(-?\d+)\s*$' % key, text, re.M)
    if not m:
        raise ValueError("vocabulary file has no '%s'" % key)
    return int(m.group(1))


def parse_yaml(text):
    """Parse a DBoW2 FileStorage vocabulary (save() format, TemplatedVocabulary.h:1475-1564).

    Returns a dict of flat arrays in FILE order (which fixes the children order of load()).
    """
    nodes = _NODE_RE.findall(text)
    words = _WORD_RE.findall(text)
    n = len(nodes)
    desc = np.array(" ".join(d for _, _, _, d in nodes).split(), dtype=np.int64)
    if desc.size != 32 * n or (desc.size and (desc.min() < 0 or desc.max() > 255)):
        raise ValueError("vocabulary descriptors are not 32 bytes each")
    word_node = np.zeros(len(words), np.int32)
    for wid, nid in words:
        word_node[int(wid)] = int(nid)
    return {
        "k": _scalar(text, "k"), "L": _scalar(text, "L"),
        "scoring": _scalar(text, "scoringType"), "weighting": _scalar(text, "weightingType"),
        "node_id": np.array([int(a) for a, _, _, _ in nodes], np.int32),
        "parent_id": np.array([int(b) for _, b, _, _ in nodes], np.int32),
        "weight": np.array([float(w) for _, _, w, _ in nodes], np.float64),
        "desc": desc.astype(np.uint8).reshape(n, 32),
        "word_node": word_node,
    }


def load_yaml(path):
    with open(path, "r") as f:
        return parse_yaml(f.read())


def load_npz(path):
    z = np.load(path)   # allow_pickle=False
    d = {k: z[k] for k in ("node_id", "parent_id", "weight", "desc", "word_node")}
    for k in ("k", "L", "scoring", "weighting"):
        d[k] = int(z[k])
    return d


def save_npz(path, voc):
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in voc.items()})


class Vocabulary:
    """ORBVocabulary resident on one GPU."""

    def __init__(self, voc, device=0):
        self.voc = voc
        h = ctypes.c_void_p()
        self._arrays = [np.ascontiguousarray(voc[k]) for k in
                        ("node_id", "parent_id", "weight", "desc", "word_node")]
        nid, pid, w, d, wn = self._arrays
        _check(_lib().mcs_vocab_create(voc["k"], voc["L"], voc["scoring"], voc["weighting"],
                                       len(nid), _p(nid), _p(pid), _p(w), _p(d), len(wn), _p(wn),
                                       device, ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            _lib().mcs_vocab_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self):
        out = np.zeros(6, np.int32)
        _check(_lib().mcs_vocab_info(self._h, _p(out)))
        return dict(zip(("k", "L", "scoring", "weighting", "n_nodes", "n_words"), out.tolist()))

    def transform_words_device(self, d_desc, n, levelsup, d_word, d_weight, d_node, stream=None):
        """Raw device pointers (ints) -> per-descriptor word / weight / ancestor node."""
        _check(_lib().mcs_vocab_transform_words_device(self._h, d_desc, int(n), int(levelsup),
                                                       d_word, d_weight, d_node, stream))

    def transform_words(self, desc, levelsup=4):
        """torch uint8 [n, 32] on cuda -> (word u32, weight f64, node u32) torch tensors."""
        import torch
        n = desc.shape[0]
        word = torch.empty(n, dtype=torch.int32, device=desc.device)
        weight = torch.empty(n, dtype=torch.float64, device=desc.device)
        node = torch.empty(n, dtype=torch.int32, device=desc.device)
        stream = torch.cuda.current_stream(desc.device).cuda_stream
        self.transform_words_device(desc.data_ptr(), n, levelsup, word.data_ptr(),
                                    weight.data_ptr(), node.data_ptr(), stream)
        return word, weight, node

    def transform(self, desc, levelsup=4):
        """Host uint8 [n, 32] -> (BowVector dict word->value, FeatureVector dict node->[i])."""
        desc = np.ascontiguousarray(desc, dtype=np.uint8).reshape(-1, 32)
        n = desc.shape[0]
        m = max(n, 1)
        bw, bv = np.zeros(m, np.uint32), np.zeros(m, np.float64)
        fn, fp, ff = np.zeros(m, np.uint32), np.zeros(m + 1, np.int32), np.zeros(m, np.uint32)
        bn, fvn = ctypes.c_int32(), ctypes.c_int32()
        _check(_lib().mcs_vocab_transform(self._h, _p(desc), n, levelsup, _p(bw), _p(bv),
                                          ctypes.byref(bn), _p(fn), _p(fp), _p(ff),
                                          ctypes.byref(fvn)))
        bow = {int(bw[i]): float(bv[i]) for i in range(bn.value)}
        fv = {int(fn[j]): ff[fp[j]:fp[j + 1]].tolist() for j in range(fvn.value)}
        return bow, fv


def synthetic(k=9, L=3, seed=0, stop_frac=0.1, weighting=TF_IDF, scoring=L1_NORM, ragged=False):
    """A random k-ary vocabulary of depth L in save()'s DFS-stack node order.

    ragged=True gives nodes 1..k children and ends some branches early (as k-means trees
    with few descriptors per cluster do, e.g. the reference's small_orb_omni_voc_9_6.yml)."""
    rng = np.random.default_rng(seed)
    node_id, parent_id, weight, leaves = [], [], [], []
    next_id = [1]
    stack = [(0, 0)]
    while stack:                      # save(): parents.pop_back(), children in order
        pid, depth = stack.pop()
        nk = int(rng.integers(1, k + 1)) if ragged else k
        kids = list(range(next_id[0], next_id[0] + nk))
        next_id[0] += nk
        for c in kids:
            node_id.append(c)
            parent_id.append(pid)
            if depth + 1 == L or (ragged and depth >= 1 and rng.random() < 0.2):
                leaves.append(c)
                weight.append(0.0 if rng.random() < stop_frac else float(rng.uniform(0.5, 3.0)))
            else:
                weight.append(0.0)
                stack.append((c, depth + 1))
    n = len(node_id)
    desc = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    return {"k": k, "L": L, "scoring": scoring, "weighting": weighting,
            "node_id": np.array(node_id, np.int32), "parent_id": np.array(parent_id, np.int32),
            "weight": np.array(weight, np.float64), "desc": desc,
            "word_node": np.array(sorted(leaves), np.int32)}


__all__ = ["Vocabulary", "parse_yaml", "load_yaml", "load_npz", "save_npz", "synthetic",
           "McsError"]
