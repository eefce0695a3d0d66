"""DBoW2 vocabulary transform (bag of words): oracle pinning on CPU, GPU parity vs the oracle.

Reference: ThirdParty/DBoW2/DBoW2/TemplatedVocabulary.h:1126-1261 (transform), :1568-1616
(load), BowVector.cpp:34-86, FeatureVector.cpp:31-45, FORB.cpp:82-101; call sites
src/cMultiFrame.cpp:356-363 and src/cMultiKeyFrame.cpp:105-119 (levelsup = 4).
The reference has no tests for this path and cannot be compiled here (OpenCV absent); the
oracle is pinned by the reference's own vocabulary file (tests/golden/small_orb_omni_voc_9_6.npz,
made by tools/make_vocab_fixture.py) and by a pure-Python restatement of the descent on small
cases.  Integer outputs (word / node ids, feature lists) must be equal, weights bit-exact.
"""
import os

import numpy as np
import pytest

from tests import oracle_bind as ob

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "golden", "small_orb_omni_voc_9_6.npz")
REF_YML = "/root/reference/Examples/small_orb_omni_voc_9_6.yml"


def _vocab():
    from mcs_amd import vocab
    return vocab


def _real():
    return _vocab().load_npz(FIXTURE)


def _features(voc, n, seed, flip_bits=12):
    """Half random descriptors, half vocabulary leaves with a few flipped bits (deep descents)."""
    rng = np.random.default_rng(seed)
    rnd = rng.integers(0, 256, size=(n - n // 2, 32), dtype=np.uint8)
    src = voc["desc"][rng.integers(0, len(voc["desc"]), size=n // 2)].copy()
    bits = np.unpackbits(src, axis=1)
    for r in range(bits.shape[0]):
        bits[r, rng.integers(0, 256, size=flip_bits)] ^= 1
    return np.concatenate([rnd, np.packbits(bits, axis=1)], axis=0)


def _py_descend(voc, f, levelsup):
    """Pure-Python restatement of transform(feature, ...) (TemplatedVocabulary.h:1217-1261)."""
    children = {}
    for i, (nid, pid) in enumerate(zip(voc["node_id"].tolist(), voc["parent_id"].tolist())):
        children.setdefault(pid, []).append((nid, i))
    word_of = {int(nd): w for w, nd in enumerate(voc["word_node"].tolist())}
    pos = {int(nid): i for i, nid in enumerate(voc["node_id"].tolist())}
    fb = np.unpackbits(f)
    nid_level = voc["L"] - levelsup
    nid, cur, level = 0, 0, 0
    while True:
        level += 1
        kids = children[cur]
        best, best_d = None, None
        for c, i in kids:
            d = int(np.count_nonzero(fb != np.unpackbits(voc["desc"][i])))
            if best_d is None or d < best_d:
                best, best_d = c, d
        cur = best
        if level == nid_level:
            nid = cur
        if cur not in children:
            break
    return word_of.get(cur, 0), float(voc["weight"][pos[cur]]), nid


# ----------------------------------------------------------------------------- CPU


def test_fixture_matches_reference_file():
    v = _real()
    assert (v["k"], v["L"], v["scoring"], v["weighting"]) == (9, 6, 0, 0)   # TF_IDF, L1
    assert len(v["node_id"]) == 8822 and len(v["word_node"]) == 6999
    assert sorted(v["node_id"].tolist()) == list(range(1, 8823))
    parents = set(v["parent_id"].tolist())
    assert not parents & set(v["word_node"].tolist())          # every word is a leaf
    if os.path.exists(REF_YML):                                 # build container only
        y = _vocab().load_yaml(REF_YML)
        for k in ("node_id", "parent_id", "weight", "desc", "word_node"):
            assert np.array_equal(y[k], v[k]), k


def test_oracle_descent_matches_python_restatement(built):
    v = _real()
    feats = _features(v, 24, seed=3)
    for levelsup in (4, 0, 6):
        word, w, node = ob.vocab_words(v, feats, levelsup)
        for i in range(len(feats)):
            assert (int(word[i]), float(w[i]), int(node[i])) == _py_descend(v, feats[i], levelsup)


def test_oracle_bow_properties(built):
    v = _real()
    feats = _features(v, 2000, seed=5)
    word, w, node = ob.vocab_words(v, feats, 4)
    bow, fv = ob.vocab_transform(v, feats, 4)
    kept = w > 0
    assert set(bow) == set(word[kept].tolist())
    assert abs(sum(bow.values()) - 1.0) < 1e-12                   # L1-normalised
    allf = sorted(i for lst in fv.values() for i in lst)
    assert allf == np.nonzero(kept)[0].tolist()
    for nd, lst in fv.items():
        assert all(int(node[i]) == nd for i in lst) and lst == sorted(lst)


def test_vocab_symbols_exported(built):
    import ctypes
    import mcs_amd
    L = ctypes.CDLL(mcs_amd.LIB_PATH)
    for s in ("mcs_vocab_create", "mcs_vocab_destroy", "mcs_vocab_info",
              "mcs_vocab_transform_words_device", "mcs_vocab_transform"):
        assert hasattr(L, s), s


# ----------------------------------------------------------------------------- GPU


def _check_transform(voc, feats, levelsup):
    vocab = _vocab()
    V = vocab.Vocabulary(voc)
    try:
        bow, fv = V.transform(feats, levelsup)
        obow, ofv = ob.vocab_transform(voc, feats, levelsup)
        assert list(bow) == list(obow)
        assert all(bow[k] == obow[k] for k in bow)                 # bit-exact doubles
        assert fv == ofv
    finally:
        V.close()


@pytest.mark.gpu
def test_gpu_words_real_vocab(gpu):
    import torch
    vocab = _vocab()
    v = _real()
    V = vocab.Vocabulary(v)
    info = V.info()
    assert info["n_nodes"] == 8823 and info["n_words"] == 6999
    feats = _features(v, 50000, seed=11)
    d = torch.from_numpy(feats).cuda()
    for levelsup in (4, 0, 2, 6, 7):
        word, w, node = V.transform_words(d, levelsup)
        torch.cuda.synchronize()
        ow, oww, on = ob.vocab_words(v, feats, levelsup)
        assert np.array_equal(word.cpu().numpy().view(np.uint32), ow), levelsup
        assert np.array_equal(w.cpu().numpy(), oww), levelsup
        assert np.array_equal(node.cpu().numpy().view(np.uint32), on), levelsup
    V.close()


@pytest.mark.gpu
@pytest.mark.parametrize("levelsup", [4, 1])
def test_gpu_transform_real_vocab(gpu, levelsup):
    v = _real()
    _check_transform(v, _features(v, 6000, seed=17 + levelsup), levelsup)


@pytest.mark.gpu
@pytest.mark.parametrize("weighting,scoring", [(0, 0), (1, 1), (1, 5), (2, 0), (3, 2), (0, 5)])
@pytest.mark.parametrize("ragged", [False, True])
def test_gpu_transform_synthetic(gpu, weighting, scoring, ragged):
    vocab = _vocab()
    v = vocab.synthetic(k=9, L=4, seed=7 + weighting, weighting=weighting, scoring=scoring,
                        ragged=ragged)
    _check_transform(v, _features(v, 3000, seed=23, flip_bits=20), 2)


@pytest.mark.gpu
def test_gpu_edge_cases(gpu):
    vocab = _vocab()
    v = vocab.synthetic(k=3, L=2, seed=1)
    V = vocab.Vocabulary(v)
    assert V.transform(np.zeros((0, 32), np.uint8)) == ({}, {})  # no features
    V.close()
    empty = dict(v, word_node=np.zeros(0, np.int32))              # empty(): no words
    V = vocab.Vocabulary(empty)
    assert V.transform(_features(v, 10, seed=2)) == ({}, {})
    V.close()
    bad = dict(v, parent_id=v["node_id"].copy())                  # self-parent -> error
    with pytest.raises(vocab.McsError):
        vocab.Vocabulary(bad)
    allstop = dict(v, weight=np.zeros_like(v["weight"]))          # every word stopped
    _check_transform(allstop, _features(v, 50, seed=4), 1)
