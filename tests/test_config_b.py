"""GPU parity of the exact batch the headline number is measured on (bench.py config B).

171 multi-frames x 3 Lafida cameras = 513 camera-frames, per-camera mirror masks, 2000
features per camera, ONE `extract_batch_device` call (the bench's launch sequence: XCD frame
mapping, per-frame slot offsets, the k_octree LDS/global switch, every level), then ONE
`mcs_hamming_top2_batch_device` call over the 510 consecutive same-camera pairs.  Frames 0..2,
every 16th, and the last three are compared bit-exactly with the oracle (all keypoint fields
and descriptors), and the first, middle and last match pairs with the oracle top-2.

Reference: cMultiFrame ctor, per-camera extraction (src/cMultiFrame.cpp:128-139);
mdBRIEFextractorOct::operator() (src/mdBRIEFextractorOct.cpp:1244-1337); the O(N1*N2)
Hamming part of SearchForTriangulationRaw (src/cORBmatcher.cpp:968-1156).
"""
import numpy as np
import pytest

from tests import oracle_bind as ob

pytestmark = pytest.mark.gpu

M, NC, W, H, NFEAT = 171, 3, 754, 480, 2000


@pytest.fixture(scope="module")
def batch(gpu):
    import torch
    import mcs_amd
    from mcs_amd import synth
    uimgs, imgs, masks, midx, pairs = synth.config_b_batch(M)
    F = M * NC
    p = mcs_amd.ExtractorParams(nfeatures=NFEAT, fast_threshold=20)
    ex = mcs_amd.Extractor(p, W, H, max_frames=F)
    cap = ex.capacity
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    d_img = torch.from_numpy(imgs).to(dev)
    d_mask = torch.from_numpy(masks).to(dev)
    ex.set_masks_device(d_mask.data_ptr(), NC, s)
    d_midx = torch.from_numpy(midx).to(dev)
    d_kps = torch.full((F, cap * 7), -1, dtype=torch.int32, device=dev)
    d_cnt = torch.full((F,), -1, dtype=torch.int32, device=dev)
    d_desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
    ex.extract_batch_device(d_img.data_ptr(), F, d_midx.data_ptr(), d_kps.data_ptr(),
                            d_cnt.data_ptr(), d_desc.data_ptr(), s)
    d_pairs = torch.from_numpy(pairs).to(dev)
    NP = len(pairs)
    d_m = [torch.full((NP, cap), -7, dtype=torch.int32, device=dev) for _ in range(4)]
    rc = mcs_amd.lib().mcs_hamming_top2_batch_device(
        d_desc.data_ptr(), d_cnt.data_ptr(), d_pairs.data_ptr(), NP, cap, 32,
        *[t.data_ptr() for t in d_m], s)
    assert rc == 0
    torch.cuda.synchronize()
    out = {
        "imgs": imgs, "masks": masks, "pairs": pairs, "cap": cap,
        "cnt": d_cnt.cpu().numpy(),
        "kps": d_kps.cpu().numpy().view(mcs_amd.KEYPOINT_DTYPE).reshape(F, cap),
        "desc": d_desc.cpu().numpy(),
        "m": [t.cpu().numpy() for t in d_m],
    }
    ex.close()
    return out


def _checked_frames():
    F = M * NC
    return sorted(set([0, 1, 2] + list(range(0, F, 16)) + [F - 3, F - 2, F - 1]))


_ORACLE = {}


def _oracle(b, f):
    if f not in _ORACLE:
        _ORACLE[f] = ob.extract(b["imgs"][f], b["masks"][f % NC], nfeatures=NFEAT, fast_th=20)
    return _ORACLE[f]


def test_config_b_counts_plausible(batch):
    cnt = batch["cnt"]
    assert (cnt > 0).all() and (cnt <= batch["cap"]).all()
    # frames repeat every n_unique multi-frames: identical inputs give identical outputs
    U = 12
    for f in range(U * NC, M * NC):
        g = f - U * NC
        assert cnt[f] == cnt[g]


@pytest.mark.parametrize("f", _checked_frames())
def test_config_b_frame_bitexact(batch, f):
    okps, odesc = _oracle(batch, f)
    n = batch["cnt"][f]
    assert n == len(okps), (f, n, len(okps))
    kp = batch["kps"][f, :n]
    for name in okps.dtype.names:
        assert np.array_equal(kp[name], okps[name]), "frame %d field %s differs" % (f, name)
    assert np.array_equal(batch["desc"][f, :n], odesc), "frame %d descriptors differ" % f


def test_config_b_repeated_frames_identical(batch):
    """Every repeat of a rendered multi-frame in the batch gives the identical output block
    (slot offsets / XCD mapping cannot leak between frames)."""
    U = 12
    cnt, kps, desc = batch["cnt"], batch["kps"], batch["desc"]
    for f in range(U * NC, M * NC):
        g = f % (U * NC)
        n = cnt[g]
        assert np.array_equal(kps[f, :n], kps[g, :n]), f
        assert np.array_equal(desc[f, :n], desc[g, :n]), f


@pytest.mark.parametrize("p", [0, 1, 2, 254, 255, 256, 507, 508, 509])
def test_config_b_match_pairs(batch, p):
    qf, tf = batch["pairs"][p]
    _, qd = _oracle(batch, int(qf))
    _, td = _oracle(batch, int(tf))
    bi, bd, sd = ob.hamming_top2(qd, td)
    n = len(qd)
    m = batch["m"]
    assert np.array_equal(m[0][p, :n], bi), "pair %d best idx" % p
    assert np.array_equal(m[1][p, :n], bd), "pair %d best dist" % p
    assert np.array_equal(m[3][p, :n], sd), "pair %d second dist" % p
