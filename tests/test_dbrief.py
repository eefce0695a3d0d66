"""dBRIEF / mdBRIEF descriptors on the Scaramuzza camera model (SURVEY §8 row a7').

Reference: rotateAndDistortPattern src/mdBRIEFextractorOct.cpp:250-283, compute_dBRIEF
:356-408, compute_mdBRIEF :410-554, keypoint undistortion :1304-1316; ImgToWorld /
WorldToImg src/cam_model_omni.cpp:49-163; undistortPointsOcam / distortPointsOcam
include/cam_model_omni.h:129-147.

CPU tests pin the oracle's camera model against an independent numpy restatement and the
Lafida calibration fixtures; GPU tests compare the HIP path with the oracle bit for bit
(keypoints, descriptors, mdBRIEF masks).  Parity of the oracle itself is unpinned against
the reference binary (OpenCV absent).
"""
import numpy as np
import pytest

from mcs_amd import CamModel, synth


def _cam(c=0):
    return CamModel.from_dict(synth.LAFIDA_CAMS[c])


def _np_world_to_img(cam, x, y, z):
    norm = np.hypot(x, y) if (x or y) else 1e-14
    theta = np.arctan(-z / norm)
    rho = 0.0
    for a in reversed(cam["pol"]):
        rho = rho * theta + a
    uu, vv = x / norm * rho, y / norm * rho
    return uu * cam["c"] + vv * cam["d"] + cam["u0"], uu * cam["e"] + vv + cam["v0"]


def test_cam_model_matches_numpy_and_round_trips(built):
    from tests import oracle_bind as ob
    rng = np.random.default_rng(3)
    for c in range(3):
        cam, m = synth.LAFIDA_CAMS[c], _cam(c)
        for _ in range(50):
            u, v = rng.uniform(150, 600), rng.uniform(60, 420)
            xyz = ob.cam_img_to_world(m, u, v)
            # same ray as the numpy renderer's ImgToWorld
            ref = np.array(synth.img_to_world(cam, np.array([u]), np.array([v]))).ravel()
            np.testing.assert_allclose(xyz, ref, rtol=0, atol=1e-12)
            uv = ob.cam_world_to_img(m, *xyz)
            np.testing.assert_allclose(uv, _np_world_to_img(cam, *xyz), rtol=0, atol=1e-9)
            # the fitted polynomials are inverse to well under a pixel
            assert abs(uv[0] - u) < 0.05 and abs(uv[1] - v) < 0.05


def test_oracle_dbrief_properties(built):
    from tests import oracle_bind as ob
    imgs, masks = synth.rig_sequence(1, 754, 480, 1, seed=11)
    m = _cam(0)
    k0, d0 = ob.extract(imgs[0], masks[0], nfeatures=400)
    k1, d1, dm1 = ob.extract_ex(imgs[0], m, masks[0], nfeatures=400, do_dbrief=1)
    k2, d2, dm2 = ob.extract_ex(imgs[0], m, masks[0], nfeatures=400, do_dbrief=1, learn_masks=1)
    # keypoints do not depend on the descriptor type
    assert k0.tobytes() == k1.tobytes() == k2.tobytes()
    assert not dm1.any()                      # dBRIEF masks are Mat::zeros
    # mdBRIEF uses angle / RHOf instead of angle * DEG2RADf: nearly the same pattern
    ham = np.unpackbits(d1 ^ d2, axis=1).sum(1)
    assert np.median(ham) <= 8
    # stable bits: most tests survive +-20 deg of rotation
    assert 0.3 < np.unpackbits(dm2, axis=1).mean() < 0.95
    # distortion changes the ORB pattern, but descriptors stay strongly correlated
    dd = np.unpackbits(d0 ^ d1, axis=1).sum(1)
    assert 0 < np.median(dd) < 100
    # deterministic
    k3, d3, dm3 = ob.extract_ex(imgs[0], m, masks[0], nfeatures=400, do_dbrief=1, learn_masks=1)
    assert d3.tobytes() == d2.tobytes() and dm3.tobytes() == dm2.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("desc_size,learn", [(32, 0), (16, 0), (64, 0), (32, 1), (64, 1)])
def test_dbrief_matches_oracle(gpu, desc_size, learn):
    import mcs_amd
    from tests import oracle_bind as ob
    imgs, masks = synth.rig_sequence(1, 754, 480, 2, seed=21)
    for c in range(2):
        m = _cam(c)
        p = mcs_amd.ExtractorParams(nfeatures=1000, desc_size=desc_size, do_dbrief=1,
                                    learn_masks=learn)
        ex = mcs_amd.Extractor(p, 754, 480)
        ex.set_cam_models([m])
        kg, dg, mg = ex.extract_with_masks(imgs[c], masks[c])
        ko, do_, mo = ob.extract_ex(imgs[c], m, masks[c], nfeatures=1000, desc_size=desc_size,
                                    do_dbrief=1, learn_masks=learn)
        assert kg.tobytes() == ko.tobytes()
        bad = np.nonzero((dg != do_).any(1))[0]
        assert len(bad) == 0, "descriptor mismatch at %s" % bad[:10]
        assert mg.tobytes() == mo.tobytes()
        ex.close()


@pytest.mark.gpu
def test_mdbrief_without_dbrief_uses_zero_undistortion(gpu):
    """learnMasks without do_dBrief: the reference leaves undistortedKeypoints at (0,0)
    (:1304-1316) and still runs compute_mdBRIEF; both paths must agree on that quirk."""
    import mcs_amd
    from tests import oracle_bind as ob
    imgs, masks = synth.rig_sequence(1, 754, 480, 1, seed=4)
    m = _cam(0)
    p = mcs_amd.ExtractorParams(nfeatures=500, do_dbrief=0, learn_masks=1)
    ex = mcs_amd.Extractor(p, 754, 480)
    ex.set_cam_models([m])
    kg, dg, mg = ex.extract_with_masks(imgs[0], masks[0])
    ko, do_, mo = ob.extract_ex(imgs[0], m, masks[0], nfeatures=500, do_dbrief=0, learn_masks=1)
    assert kg.tobytes() == ko.tobytes()
    assert dg.tobytes() == do_.tobytes() and mg.tobytes() == mo.tobytes()


@pytest.mark.gpu
def test_dbrief_batch_per_camera_models(gpu):
    """Batch path: frame f uses camera model d_cam_index[f] (and that camera's mask)."""
    import torch
    import mcs_amd
    from tests import oracle_bind as ob
    NC = 3
    imgs, masks = synth.rig_sequence(2, 754, 480, NC, seed=8)
    cams = [_cam(c) for c in range(NC)]
    p = mcs_amd.ExtractorParams(nfeatures=800, do_dbrief=1, learn_masks=1)
    F = len(imgs)
    ex = mcs_amd.Extractor(p, 754, 480, max_frames=F)
    ex.set_cam_models(cams)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream()
    d_img = torch.from_numpy(imgs).to(dev)
    d_mask = torch.from_numpy(masks).to(dev)
    ex.set_masks_device(d_mask.data_ptr(), NC, st.cuda_stream)
    cidx = np.tile(np.arange(NC, dtype=np.int32), F // NC)
    d_idx = torch.from_numpy(cidx).to(dev)
    cap = ex.capacity
    d_kps = torch.zeros((F, cap * 7), dtype=torch.int32, device=dev)
    d_cnt = torch.zeros(F, dtype=torch.int32, device=dev)
    d_desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
    d_dm = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
    ex.extract_batch_device_ex(d_img.data_ptr(), F, d_idx.data_ptr(), d_kps.data_ptr(),
                               d_cnt.data_ptr(), d_desc.data_ptr(), d_dm.data_ptr(),
                               st.cuda_stream)
    torch.cuda.synchronize()
    cnt = d_cnt.cpu().numpy()
    kw = d_kps.cpu().numpy()
    de = d_desc.cpu().numpy()
    dm = d_dm.cpu().numpy()
    for f in range(F):
        c = int(cidx[f])
        ko, do_, mo = ob.extract_ex(imgs[f], cams[c], masks[c], nfeatures=800, do_dbrief=1,
                                    learn_masks=1)
        n = int(cnt[f])
        assert n == len(ko)
        assert kw[f, :7 * n].tobytes() == ko.tobytes()
        assert de[f, :n].tobytes() == do_.tobytes()
        assert dm[f, :n].tobytes() == mo.tobytes()
