"""cMultiFrame work on the device: bearing rays of every keypoint
(ImgToWorld, src/cMultiFrame.cpp:143-152), the camera concatenation with keypoint_to_cam /
cont_idx_to_local_cam_idx and PosInGrid (:166-184, :342-353), and isInFrustum (:218-270).

Oracles: oracle_cam_img_to_world (cam_model_omni.cpp:49-67 restated), a literal numpy loop of
the concatenation, oracle_is_in_frustum (the reference's 4x4 path, mirror mask, distance
invariance, lower_bound level).  Tolerances: rays and concatenation exact (same correctly
rounded operations); frustum flags and levels exact, projections abs 1e-9 px and viewing
cosines abs 1e-12 (device atan vs glibc atan may differ in the last ulp)."""
import ctypes

import numpy as np
import pytest

from tests import oracle_bind as ob


def _cams():
    from mcs_amd import CamModel, synth
    return [CamModel.from_dict(c) for c in synth.LAFIDA_CAMS]


def _frustum_inputs(seed=0, n=4000):
    from mcs_amd import ba, synth
    rng = np.random.default_rng(seed)
    pr = ba.make_problem(n_local=3, n_fixed=0, n_points=800, target_edges=3000, seed=seed)
    pose = pr["poses"][1].copy()
    pts = np.concatenate([pr["gt_points"], rng.uniform(-6, 6, (n - len(pr["gt_points"]), 3))])
    nrm = rng.normal(size=pts.shape)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    d0 = rng.uniform(0.5, 4.0, len(pts))
    dist = np.stack([d0, d0 * rng.uniform(1.5, 6.0, len(pts))], 1)
    masks = np.stack([synth.mirror_mask(c) for c in synth.LAFIDA_CAMS]).astype(np.uint8)
    scale = np.array([1.2 ** i for i in range(8)], np.float64)
    # mvScaleFactors as cMultiFrame builds them: s_i = s_{i-1} * (double)(float)1.2
    sf = float(np.float32(1.2))
    scale = np.cumprod([1.0] + [sf] * 7)
    return pose, pr["mc"], pr["cam"], masks, pts, nrm, dist, scale


def _oracle_frustum(pose, mc, cam, masks, pts, nrm, dist, scale):
    L = ob.lib()
    f = L.oracle_is_in_frustum
    f.restype = ctypes.c_int
    P = ctypes.c_void_p
    f.argtypes = [P, P, P, ctypes.c_int32, P, ctypes.c_int32, ctypes.c_int32, P, P, P,
                  ctypes.c_int32, P, ctypes.c_int32, P, P, P, P]
    C, n = len(mc), len(pts)
    a = [np.ascontiguousarray(x, np.float64) for x in (pose, mc, cam, pts, nrm, dist, scale)]
    mk = np.ascontiguousarray(masks, np.uint8)
    iv = np.zeros((n, C), np.uint8)
    pj = np.zeros((n, C, 2))
    lv = np.zeros((n, C), np.int32)
    vc = np.zeros((n, C))
    f(ob._p(a[0]), ob._p(a[1]), ob._p(a[2]), C, ob._p(mk), mk.shape[2], mk.shape[1], ob._p(a[3]),
      ob._p(a[4]), ob._p(a[5]), n, ob._p(a[6]), len(scale), ob._p(iv), ob._p(pj), ob._p(lv),
      ob._p(vc))
    return iv, pj, lv, vc


def test_oracle_frustum_against_numpy_projection(built):
    """The oracle's projection equals the numpy restatement (mcs_amd.ba.project) and its flags
    follow the rules computed independently in numpy."""
    from mcs_amd import ba
    pose, mc, cam, masks, pts, nrm, dist, scale = _frustum_inputs(1, 1500)
    iv, pj, lv, vc = _oracle_frustum(pose, mc, cam, masks, pts, nrm, dist, scale)
    for c in range(len(mc)):
        uv, _ = ba.project(pose, mc[c], cam[c], pts)
        sel = iv[:, c] == 1
        assert sel.sum() > 50
        np.testing.assert_allclose(pj[sel, c], uv[sel], rtol=0, atol=1e-9)
        ur, vr = np.rint(uv[:, 0]).astype(int), np.rint(uv[:, 1]).astype(int)
        H, W = masks.shape[1:]
        inb = (ur > 0) & (ur < W) & (vr > 0) & (vr < H)
        mk = np.zeros(len(pts), bool)
        mk[inb] = masks[c][vr[inb], ur[inb]] > 0
        Rt, Rc = ba.cay2rot(pose[:3]), ba.cay2rot(mc[c][:3])
        t = Rt @ mc[c][3:] + pose[3:]
        d = np.linalg.norm(pts - t, axis=1)
        ok = mk & (d >= 0.8 * dist[:, 0]) & (d <= 1.2 * dist[:, 1])
        # boundary cases (rounding at .5 px or exactly on a distance limit) are excluded
        near = (np.abs(np.abs(uv[:, 0] - np.floor(uv[:, 0])) - 0.5) < 1e-9) | \
               (np.abs(d - 0.8 * dist[:, 0]) < 1e-12) | (np.abs(d - 1.2 * dist[:, 1]) < 1e-12)
        assert np.array_equal(iv[~near, c] == 1, ok[~near])
        lvl = np.minimum(np.searchsorted(scale, d / (0.8 * dist[:, 0]), side="left"), len(scale) - 1)
        assert np.array_equal(lv[sel, c], lvl[sel])


@pytest.mark.gpu
def test_gpu_keypoint_rays_and_concat(gpu):
    import torch
    import mcs_amd
    from mcs_amd import lib, synth, rig, KEYPOINT_DTYPE
    cams = _cams()
    imgs, masks = synth.rig_sequence(2, 754, 480, 3, seed=3)
    F = len(imgs)
    ex = mcs_amd.Extractor(mcs_amd.ExtractorParams(nfeatures=1000), 754, 480, max_frames=F)
    cap = ex.capacity
    dev = torch.device("cuda", 0)
    d_img = torch.from_numpy(np.ascontiguousarray(imgs)).to(dev)
    d_mask = torch.from_numpy(np.ascontiguousarray(masks)).to(dev)
    st = torch.cuda.current_stream().cuda_stream
    ex.set_masks_device(d_mask.data_ptr(), 3, st)
    cidx = torch.tensor(np.tile(np.arange(3, dtype=np.int32), F // 3), device=dev)
    d_kps = torch.zeros((F, cap * 7), dtype=torch.int32, device=dev)
    d_cnt = torch.zeros(F, dtype=torch.int32, device=dev)
    d_desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
    ex.extract_batch_device(d_img.data_ptr(), F, cidx.data_ptr(), d_kps.data_ptr(), d_cnt.data_ptr(),
                            d_desc.data_ptr(), st)
    camb = b"".join(bytes(c) for c in cams)
    d_cams = torch.frombuffer(bytearray(camb), dtype=torch.uint8).to(dev)
    d_rays = torch.zeros((F, cap, 3), dtype=torch.float64, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    assert lib().mcs_keypoint_rays_device(P(d_kps), P(d_cnt), F, cap, P(cidx), P(d_cams), P(d_rays),
                                          ctypes.c_void_p(st)) == 0
    torch.cuda.synchronize()
    cnt = d_cnt.cpu().numpy()
    kps = d_kps.cpu().numpy().view(KEYPOINT_DTYPE).reshape(F, cap)
    rays = d_rays.cpu().numpy()
    for f in range(F):
        for i in range(0, cnt[f], 7):
            ref = ob.cam_img_to_world(cams[f % 3], float(kps[f, i]["x"]), float(kps[f, i]["y"]))
            assert np.array_equal(rays[f, i], np.asarray(ref)), (f, i)
    # concatenation of the 3 cameras of both multi-frames + PosInGrid
    gp = np.array([[0.0, 0.0, 64.0 / 754, 48.0 / 480]] * 3)
    d_gp = torch.from_numpy(gp).to(dev)
    n_mf, C = F // 3, 3
    keys = torch.zeros((n_mf, C * cap * 7), dtype=torch.int32, device=dev)
    kr = torch.zeros((n_mf, C * cap, 3), dtype=torch.float64, device=dev)
    ds = torch.zeros((n_mf, C * cap, 32), dtype=torch.uint8, device=dev)
    k2c = torch.zeros((n_mf, C * cap), dtype=torch.int32, device=dev)
    k2l = torch.zeros_like(k2c)
    grid = torch.zeros_like(k2c)
    tot = torch.zeros(n_mf, dtype=torch.int32, device=dev)
    assert lib().mcs_multiframe_concat_device(P(d_cnt), n_mf, C, cap, P(d_kps), P(d_rays), P(d_desc), 32,
                                              P(d_gp), P(keys), P(kr), P(ds), P(k2c), P(k2l), P(grid),
                                              P(tot), ctypes.c_void_p(st)) == 0
    torch.cuda.synchronize()
    keys_h = keys.cpu().numpy().view(KEYPOINT_DTYPE).reshape(n_mf, C * cap)
    desc_h = d_desc.cpu().numpy()
    for m in range(n_mf):
        cc = cnt[3 * m:3 * m + 3]
        ref = rig.concat_multiframe(cc, kps[3 * m:3 * m + 3], desc_h[3 * m:3 * m + 3])
        N = int(tot[m])
        assert N == cc.sum()
        assert keys_h[m, :N].tobytes() == ref["mvKeys"].tobytes()
        assert np.array_equal(k2c[m, :N].cpu().numpy(), ref["keypoint_to_cam"])
        assert np.array_equal(k2l[m, :N].cpu().numpy(), ref["cont_idx_to_local_cam_idx"])
        assert np.array_equal(ds[m, :N].cpu().numpy(), np.concatenate(ref["descriptors"]))
        rr = np.concatenate([rays[3 * m + c, :cc[c]] for c in range(3)])
        assert np.array_equal(kr[m, :N].cpu().numpy(), rr)
        px, py, inside = rig.grid_positions(ref["mvKeys"]["x"], ref["mvKeys"]["y"], 754, 480)
        want = np.where(inside, px | (py << 8), -1)
        assert np.array_equal(grid[m, :N].cpu().numpy(), want)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 5])
def test_gpu_is_in_frustum_matches_oracle(gpu, seed):
    import torch
    from mcs_amd import lib
    pose, mc, cam, masks, pts, nrm, dist, scale = _frustum_inputs(seed)
    iv, pj, lv, vc = _oracle_frustum(pose, mc, cam, masks, pts, nrm, dist, scale)
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    n, C = len(pts), len(mc)
    d = [T(x) for x in (pose, mc, cam, masks, pts, nrm, dist, scale)]
    g_iv = torch.zeros((n, C), dtype=torch.uint8, device=dev)
    g_pj = torch.zeros((n, C, 2), dtype=torch.float64, device=dev)
    g_lv = torch.zeros((n, C), dtype=torch.int32, device=dev)
    g_vc = torch.zeros((n, C), dtype=torch.float64, device=dev)
    assert lib().mcs_is_in_frustum_device(P(d[0]), P(d[1]), P(d[2]), C, P(d[3]), masks.shape[2],
                                          masks.shape[1], P(d[4]), P(d[5]), P(d[6]), n, P(d[7]),
                                          len(scale), P(g_iv), P(g_pj), P(g_lv), P(g_vc), None) == 0
    torch.cuda.synchronize()
    giv = g_iv.cpu().numpy()
    assert np.array_equal(giv, iv) and iv.sum() > 100
    sel = iv == 1
    assert np.abs(g_pj.cpu().numpy()[sel] - pj[sel]).max() < 1e-9
    assert np.array_equal(g_lv.cpu().numpy()[sel], lv[sel])
    assert np.abs(g_vc.cpu().numpy()[sel] - vc[sel]).max() < 1e-12
