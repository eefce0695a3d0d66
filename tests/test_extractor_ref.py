"""The extractor against the reference's OWN text.

tests/golden/extractor_ref.npz holds the output of mdBRIEFextractorOct's constructor,
ComputePyramid, ComputeKeyPointsOctTree (cell grid + skip rules), DistributeOctTree /
DivideNode, IC_Angle, rotatePattern / compute_ORB, rotateAndDistortPattern / compute_dBRIEF /
compute_mdBRIEF with the keypoint undistortion on the Lafida camera models (undistortPointsOcam /
distortPointsOcam, include/cam_model_omni.h:129-147), computeDescriptors and operator()
(src/mdBRIEFextractorOct.cpp:134-1337) evaluated from the reference's text by
tests/golden/gen_extractor_ref.py (tests/golden/cxx_eval.py translator), with OpenCV's calls as
stand-ins over this project's OpenCV restatement (the part that stays
unpinned).  Pointer ties of DistributeOctTree's (size, Node*) sort follow the list-node
allocation order (the fixture's `tie_convention`).

  * CPU: the oracle (oracle/extractor_oracle.cpp) reproduces the fixture bit for bit, so the
    oracle's restatement of the reference's own loops is pinned to the reference text;
  * GPU: the HIP extractor (single frame, and the three config-B cameras as one device batch
    with registered masks; the mdBRIEF cameras as one batch with per-frame camera models)
    reproduces it bit for bit: every keypoint field, every descriptor byte and every mdBRIEF
    stability-mask byte (integer / byte / index work: no tolerance).
Inputs are regenerated (mcs_amd.synth) and checked against the fixture's SHA-256.
"""
import hashlib
import os

import numpy as np
import pytest

from tests import oracle_bind as ob

FIX = os.path.join(os.path.dirname(__file__), "golden", "extractor_ref.npz")
FIELDS = ("x", "y", "size", "angle", "response", "octave", "class_id")


def _fix():
    return np.load(FIX, allow_pickle=False)


def _names():
    return [str(n) for n in _fix()["case_names"]]


def _case(name):
    from mcs_amd import synth
    z = _fix()
    meta = [int(v) for v in z[name + "_meta"]]
    w, h, seed, cam, nf, th, ds = meta[:7]
    db, lm = meta[7:9] if len(meta) > 7 else (0, 0)
    img, mask = synth.fisheye_frame(w, h, seed=seed, cam_index=cam)
    assert hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest() == str(z[name + "_img_sha"])
    assert hashlib.sha256(np.ascontiguousarray(mask).tobytes()).hexdigest() == str(z[name + "_mask_sha"])
    return dict(img=img, mask=mask, w=w, h=h, nf=nf, th=th, ds=ds, db=db, lm=lm, cam=cam,
                kps=z[name + "_kps"], desc=z[name + "_desc"], dmask=z[name + "_dmask"],
                nfl=z[name + "_nfl"])


def _cam_model(c):
    from mcs_amd import CamModel, synth
    return CamModel.from_dict(synth.LAFIDA_CAMS[c["cam"]])


def _names_of(kind):
    """ORB cases, or the dBRIEF / mdBRIEF cases (do_dBrief or learnMasks set)."""
    z = _fix()
    out = []
    for n in _names():
        m = z[n + "_meta"]
        distorted = len(m) > 7 and (int(m[7]) or int(m[8]))
        if (kind == "orb") != bool(distorted):
            out.append(n)
    return out


def _check(kps, desc, c, what):
    k = c["kps"]
    assert len(kps) == len(k), "%s: %d keypoints, reference text %d" % (what, len(kps), len(k))
    for i, f in enumerate(FIELDS):
        got = np.asarray(kps[f], np.float64)
        bad = np.nonzero(got != k[:, i])[0]
        assert len(bad) == 0, "%s: field %s differs at %d keypoints (first %s)" % (what, f, len(bad), bad[:5])
    bad = np.nonzero((np.asarray(desc) != c["desc"]).any(1))[0] if len(k) else []
    assert len(bad) == 0, "%s: descriptors differ at %d keypoints (first %s)" % (what, len(bad), bad[:5])


def _check_masks(dmask, c, what):
    bad = np.nonzero((np.asarray(dmask) != c["dmask"]).any(1))[0] if len(c["kps"]) else []
    assert len(bad) == 0, "%s: descriptor masks differ at %d keypoints (first %s)" % (what, len(bad), bad[:5])


def test_fixture_tables():
    """The constructor's tables as the reference text computes them (:153-202)."""
    z = _fix()
    assert np.array_equal(z["umax"], ob.umax())
    assert str(z["tie_convention"]).startswith("pointer order")
    assert int(z["n_statements"]) > 300
    for name in _names():
        nf = int(z[name + "_meta"][4])
        assert np.array_equal(z[name + "_nfl"], ob.features_per_level(nf)), name


@pytest.mark.parametrize("name", _names_of("orb"))
def test_oracle_matches_reference_text(name):
    c = _case(name)
    okps, odesc = ob.extract(c["img"], c["mask"], nfeatures=c["nf"], fast_th=c["th"], desc_size=c["ds"])
    _check(okps, odesc, c, "oracle " + name)
    assert not c["dmask"].any()          # ORB: the descriptor masks stay zero (:1216)


@pytest.mark.parametrize("name", _names_of("distorted"))
def test_oracle_dbrief_matches_reference_text(name):
    """dBRIEF / mdBRIEF: rotateAndDistortPattern, compute_dBRIEF, compute_mdBRIEF and the
    keypoint undistortion of operator() (:250-283, :356-554, :1304-1317) on the Lafida camera
    models (undistortPointsOcam / distortPointsOcam, include/cam_model_omni.h:129-147)."""
    c = _case(name)
    okps, odesc, omask = ob.extract_ex(c["img"], _cam_model(c), c["mask"], nfeatures=c["nf"],
                                       fast_th=c["th"], desc_size=c["ds"], do_dbrief=c["db"],
                                       learn_masks=c["lm"])
    _check(okps, odesc, c, "oracle " + name)
    _check_masks(omask, c, "oracle " + name)
    if not c["lm"]:
        assert not c["dmask"].any()      # dBRIEF: Mat::zeros masks (:1216)
    else:
        assert 0.2 < np.unpackbits(c["dmask"], axis=1).mean() < 0.98


@pytest.mark.gpu
@pytest.mark.parametrize("name", _names())
def test_gpu_extract_matches_reference_text(gpu, name):
    import mcs_amd
    c = _case(name)
    p = mcs_amd.ExtractorParams(nfeatures=c["nf"], fast_threshold=c["th"], desc_size=c["ds"],
                                do_dbrief=c["db"], learn_masks=c["lm"])
    ex = mcs_amd.Extractor(p, c["w"], c["h"])
    try:
        if c["db"] or c["lm"]:
            ex.set_cam_models([_cam_model(c)])
        kps, desc, dm = ex.extract_with_masks(c["img"], c["mask"])
    finally:
        ex.close()
    _check(kps, desc, c, "gpu " + name)
    _check_masks(dm, c, "gpu " + name)


@pytest.mark.gpu
def test_gpu_mdbrief_batch_matches_reference_text(gpu):
    """mdBRIEF at the config-B budget: the three Lafida cameras as ONE device batch, each frame
    with its own camera model and mirror mask (extract_batch_device_ex), against the text."""
    import torch
    import mcs_amd
    cs = [_case(n) for n in ("Bmd_s21", "Bmd_s22", "Bmd_s23")]
    W, H, F = 754, 480, 3
    p = mcs_amd.ExtractorParams(nfeatures=2000, fast_threshold=20, do_dbrief=1, learn_masks=1)
    ex = mcs_amd.Extractor(p, W, H, max_frames=F)
    try:
        ex.set_cam_models([_cam_model(c) for c in cs])
        cap = ex.capacity
        dev = torch.device("cuda:0")
        s = torch.cuda.current_stream().cuda_stream
        d_img = torch.from_numpy(np.stack([c["img"] for c in cs])).to(dev)
        d_mask = torch.from_numpy(np.stack([c["mask"] for c in cs])).to(dev)
        ex.set_masks_device(d_mask.data_ptr(), F, s)
        d_idx = torch.arange(F, dtype=torch.int32, device=dev)
        d_kps = torch.full((F, cap * 7), -1, dtype=torch.int32, device=dev)
        d_cnt = torch.full((F,), -1, dtype=torch.int32, device=dev)
        d_desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
        d_dm = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
        ex.extract_batch_device_ex(d_img.data_ptr(), F, d_idx.data_ptr(), d_kps.data_ptr(),
                                   d_cnt.data_ptr(), d_desc.data_ptr(), d_dm.data_ptr(), s)
        torch.cuda.synchronize()
        cnt = d_cnt.cpu().numpy()
        kps = d_kps.cpu().numpy().view(mcs_amd.KEYPOINT_DTYPE).reshape(F, cap)
        desc, dm = d_desc.cpu().numpy(), d_dm.cpu().numpy()
    finally:
        ex.close()
    for f, c in enumerate(cs):
        n = int(cnt[f])
        _check(kps[f, :n], desc[f, :n], c, "gpu mdBRIEF batch camera %d" % f)
        _check_masks(dm[f, :n], c, "gpu mdBRIEF batch camera %d" % f)


@pytest.mark.gpu
def test_gpu_batch_matches_reference_text(gpu):
    """The three config-B cameras (one Lafida camera each) as ONE device batch with the mirror
    masks registered per camera: the bench's launch sequence against the reference text."""
    import torch
    import mcs_amd
    cs = [_case(n) for n in ("B_s21", "B_s22", "B_s23")]
    W, H, F = 754, 480, 3
    p = mcs_amd.ExtractorParams(nfeatures=2000, fast_threshold=20)
    ex = mcs_amd.Extractor(p, W, H, max_frames=F)
    try:
        cap = ex.capacity
        dev = torch.device("cuda:0")
        s = torch.cuda.current_stream().cuda_stream
        d_img = torch.from_numpy(np.stack([c["img"] for c in cs])).to(dev)
        d_mask = torch.from_numpy(np.stack([c["mask"] for c in cs])).to(dev)
        ex.set_masks_device(d_mask.data_ptr(), F, s)
        d_midx = torch.arange(F, dtype=torch.int32, device=dev)
        d_kps = torch.full((F, cap * 7), -1, dtype=torch.int32, device=dev)
        d_cnt = torch.full((F,), -1, dtype=torch.int32, device=dev)
        d_desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
        ex.extract_batch_device(d_img.data_ptr(), F, d_midx.data_ptr(), d_kps.data_ptr(),
                                d_cnt.data_ptr(), d_desc.data_ptr(), s)
        torch.cuda.synchronize()
        cnt = d_cnt.cpu().numpy()
        kps = d_kps.cpu().numpy().view(mcs_amd.KEYPOINT_DTYPE).reshape(F, cap)
        desc = d_desc.cpu().numpy()
    finally:
        ex.close()
    for f, c in enumerate(cs):
        n = int(cnt[f])
        _check(kps[f, :n], desc[f, :n], c, "gpu batch camera %d" % f)


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="needs the reference checkout")
def test_fixture_regenerates_from_reference_text(tmp_path):
    """Where the reference checkout exists (the build container), the generator re-derives the
    quick cases from the reference text bit for bit."""
    import subprocess
    import sys
    out = tmp_path / "q.npz"
    gen = os.path.join(os.path.dirname(__file__), "golden", "gen_extractor_ref.py")
    subprocess.check_call([sys.executable, gen, "--quick", "--out", str(out)], timeout=600)
    q, z = np.load(out), _fix()
    for name in ("A_s1", "L_s4", "mdq_s4"):
        for k in ("_kps", "_desc", "_dmask", "_nfl", "_meta"):
            assert np.array_equal(q[name + k], z[name + k]), name + k
